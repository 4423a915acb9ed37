// TEST INFRASTRUCTURE (see nocopy.hh): sptr as in /root/reference/sptr.hh
#pragma once
#include <memory>
template <class T>
using sptr = std::shared_ptr<T>;
