// TEST INFRASTRUCTURE (see nocopy.hh): the output stream the adapter writes
// its instructions to
#pragma once
#include <string>
namespace google {
namespace protobuf {
namespace io {
class ZeroCopyOutputStream {
 public:
  virtual ~ZeroCopyOutputStream() {}
  virtual void append(const std::string& s) = 0;
};
class StringOutputStream : public ZeroCopyOutputStream {
  std::string* s_;
 public:
  explicit StringOutputStream(std::string* s) : s_(s) {}
  void append(const std::string& s) override { s_->append(s); }
};
}  // namespace io
}  // namespace protobuf
}  // namespace google
