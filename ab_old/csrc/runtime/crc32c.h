// CRC32C (Castagnoli) -- used by the TFRecord/tfevents framing and the TF V2
// checkpoint bundle (block trailers and per-tensor checksums).  SSE4.2
// `crc32` instruction when the host CPU has it, slicing-by-8 tables otherwise.
#pragma once
#include <cstddef>
#include <cstdint>

namespace dtf {

uint32_t crc32c_extend(uint32_t init_crc, const void* data, size_t n);
inline uint32_t crc32c(const void* data, size_t n) { return crc32c_extend(0, data, n); }

// TF/leveldb "masked" CRC (so that CRCs of data that embeds CRCs stay useful).
constexpr uint32_t kMaskDelta = 0xa282ead8u;
inline uint32_t crc32c_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kMaskDelta; }
inline uint32_t crc32c_unmask(uint32_t m) {
  uint32_t rot = m - kMaskDelta;
  return (rot >> 17) | (rot << 15);
}
bool crc32c_hw_available();

}  // namespace dtf
