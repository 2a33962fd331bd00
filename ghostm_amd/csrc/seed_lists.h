// seed_lists.h — K1's entry -> list byte table (k_seed_filter phase 0), shared
// by the kernel and the host test tests/native/test_seed_lists.cpp.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define GHOSTM_SEED_HD __host__ __device__
#else
#define GHOSTM_SEED_HD
#endif

namespace ghostm {
namespace kern {

// The list index of entries e0 .. e0 + 15 of a block's concatenated k-mer
// lists, one byte each, little-endian in wv[0..3]. off[0..nl] are the lists'
// exclusive offsets (off[nl] = total entries) and j the list holding entry e0
// (off[j] <= e0 < off[j + 1]). The 16 bytes start as j; each list boundary
// inside the window (off[j + 1] < e0 + 16, equal ones for empty lists) adds
// one to the bytes at and after it: a loop over the boundaries, usually none
// or one, instead of a test per entry. Bytes past the last list keep its
// index (entries >= off[nl] are never read).
GHOSTM_SEED_HD inline void ListBytes16(uint32_t e0, uint32_t j, const uint32_t *off, uint32_t nl, uint32_t wv[4]) {
  const uint32_t fill = j * 0x01010101u;
  for (int w = 0; w < 4; ++w) wv[w] = fill;
  for (uint32_t nxt = off[j + 1]; nxt < e0 + 16 && j + 1 < nl; nxt = off[++j + 1]) {
    const uint32_t b = nxt - e0;
    for (uint32_t w = 0; w < 4; ++w) {
      // +1 in the bytes k >= b of word w (k = 4 w .. 4 w + 3)
      const uint32_t c = b > 4 * w ? b - 4 * w : 0u;
      wv[w] += c >= 4 ? 0u : 0x01010101u << (8 * c);
    }
  }
}

}  // namespace kern
}  // namespace ghostm
