// TEST INFRASTRUCTURE (see nocopy.hh): Message::serialize = varint32 length
// + message (message.cc:16-23)
#pragma once
#include <google/protobuf/io/zero_copy_stream_impl_lite.h>
#include "zbackup.pb.h"
namespace Message {
inline void serialize(const BackupInstruction& m, google::protobuf::io::ZeroCopyOutputStream& out) {
  const std::string body = m.SerializeAsString();
  out.append(pb_varint(body.size()) + body);
}
}  // namespace Message
