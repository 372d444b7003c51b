#include "crc32c.h"

#include <cstring>
#if defined(__x86_64__)
#include <cpuid.h>
#endif

namespace dtf {

namespace {

struct Tables {
  uint32_t t[8][256];
  Tables() {
    const uint32_t poly = 0x82f63b78u;  // reflected Castagnoli polynomial
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : (c >> 1);
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};
const Tables& tables() {
  static Tables tb;
  return tb;
}

uint32_t sw_extend(uint32_t crc, const uint8_t* p, size_t n) {
  const Tables& T = tables();
  crc = ~crc;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    crc = T.t[0][(crc ^ *p++) & 0xff] ^ (crc >> 8);
    --n;
  }
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    v ^= crc;
    crc = T.t[7][v & 0xff] ^ T.t[6][(v >> 8) & 0xff] ^ T.t[5][(v >> 16) & 0xff] ^
          T.t[4][(v >> 24) & 0xff] ^ T.t[3][(v >> 32) & 0xff] ^ T.t[2][(v >> 40) & 0xff] ^
          T.t[1][(v >> 48) & 0xff] ^ T.t[0][v >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) crc = T.t[0][(crc ^ *p++) & 0xff] ^ (crc >> 8);
  return ~crc;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t hw_extend(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = ~crc & 0xffffffffu;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
    --n;
  }
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = __builtin_ia32_crc32di(c, v);
    p += 8;
    n -= 8;
  }
  while (n--) c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
  return ~(uint32_t)c;
}
bool detect_hw() {
  unsigned a, b, c, d;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
  return (c & bit_SSE4_2) != 0;
}
#endif

}  // namespace

bool crc32c_hw_available() {
#if defined(__x86_64__)
  static bool hw = detect_hw();
  return hw;
#else
  return false;
#endif
}

uint32_t crc32c_extend(uint32_t init_crc, const void* data, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
#if defined(__x86_64__)
  if (crc32c_hw_available()) return hw_extend(init_crc, p, n);
#endif
  return sw_extend(init_crc, p, n);
}

}  // namespace dtf
