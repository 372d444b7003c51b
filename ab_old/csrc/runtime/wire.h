// Minimal protobuf wire-format encoder/decoder (varint, fixed32/64,
// length-delimited).  Enough to emit/parse the handful of TF messages the
// runtime needs (Event, Summary, BundleHeaderProto, BundleEntryProto,
// TensorShapeProto) without linking protobuf or TF.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace dtf {
namespace wire {

enum WireType { VARINT = 0, FIXED64 = 1, LEN = 2, FIXED32 = 5 };

inline void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back(static_cast<char>((v & 0x7f) | 0x80));
    v >>= 7;
  }
  s.push_back(static_cast<char>(v));
}
inline void put_fixed32(std::string& s, uint32_t v) {
  char b[4];
  memcpy(b, &v, 4);
  s.append(b, 4);
}
inline void put_fixed64(std::string& s, uint64_t v) {
  char b[8];
  memcpy(b, &v, 8);
  s.append(b, 8);
}
inline void put_tag(std::string& s, int field, WireType wt) { put_varint(s, (uint64_t(field) << 3) | wt); }
inline void put_uint(std::string& s, int field, uint64_t v) {
  put_tag(s, field, VARINT);
  put_varint(s, v);
}
inline void put_int(std::string& s, int field, int64_t v) { put_uint(s, field, static_cast<uint64_t>(v)); }
inline void put_bytes(std::string& s, int field, const std::string& b) {
  put_tag(s, field, LEN);
  put_varint(s, b.size());
  s.append(b);
}
inline void put_double(std::string& s, int field, double d) {
  uint64_t v;
  memcpy(&v, &d, 8);
  put_tag(s, field, FIXED64);
  put_fixed64(s, v);
}
inline void put_float(std::string& s, int field, float f) {
  uint32_t v;
  memcpy(&v, &f, 4);
  put_tag(s, field, FIXED32);
  put_fixed32(s, v);
}
inline void put_fixed32_field(std::string& s, int field, uint32_t v) {
  put_tag(s, field, FIXED32);
  put_fixed32(s, v);
}

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  Reader(const void* data, size_t n)
      : p(static_cast<const uint8_t*>(data)), end(static_cast<const uint8_t*>(data) + n) {}
  bool done() const { return p >= end; }
  uint64_t varint() {
    uint64_t v = 0;
    int shift = 0;
    while (true) {
      if (p >= end) throw std::runtime_error("truncated varint");
      uint8_t b = *p++;
      v |= uint64_t(b & 0x7f) << shift;
      if (!(b & 0x80)) break;
      shift += 7;
      if (shift > 63) throw std::runtime_error("bad varint");
    }
    return v;
  }
  uint32_t fixed32() {
    if (end - p < 4) throw std::runtime_error("truncated fixed32");
    uint32_t v;
    memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  uint64_t fixed64() {
    if (end - p < 8) throw std::runtime_error("truncated fixed64");
    uint64_t v;
    memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  std::string bytes() {
    uint64_t n = varint();
    if ((uint64_t)(end - p) < n) throw std::runtime_error("truncated bytes");
    std::string s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
  // returns false at end; sets field and wire type
  bool next(int& field, int& wt) {
    if (done()) return false;
    uint64_t t = varint();
    field = int(t >> 3);
    wt = int(t & 7);
    return true;
  }
  void skip(int wt) {
    switch (wt) {
      case VARINT: varint(); break;
      case FIXED64: fixed64(); break;
      case LEN: bytes(); break;
      case FIXED32: fixed32(); break;
      default: throw std::runtime_error("unsupported wire type");
    }
  }
};

}  // namespace wire
}  // namespace dtf
