// TEST INFRASTRUCTURE (see nocopy.hh): BackupInstruction's wire encoding
// (zbackup.proto:149-159: field 1 chunk_to_emit, field 2 bytes_to_emit)
#pragma once
#include <string>
inline std::string pb_varint(uint64_t v) {
  std::string o;
  while (v >= 0x80) {
    o.push_back((char)((v & 0x7F) | 0x80));
    v >>= 7;
  }
  o.push_back((char)v);
  return o;
}
class BackupInstruction {
  std::string chunk_, bytes_;
  bool has_chunk_ = false, has_bytes_ = false;
 public:
  void set_chunk_to_emit(const std::string& v) { chunk_ = v; has_chunk_ = true; }
  void set_bytes_to_emit(const std::string& v) { bytes_ = v; has_bytes_ = true; }
  std::string SerializeAsString() const {
    std::string o;
    if (has_chunk_) o += "\x0a" + pb_varint(chunk_.size()) + chunk_;
    if (has_bytes_) o += "\x12" + pb_varint(bytes_.size()) + bytes_;
    return o;
  }
};
struct BundleInfo {};
