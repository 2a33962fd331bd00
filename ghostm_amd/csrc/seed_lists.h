// seed_lists.h — K1 arithmetic shared by the kernels and the host tests: the
// entry -> list byte table (k_seed_filter phase 0, tests/native/test_seed_lists.cpp)
// and the exact bin table's bucket hash (BinTable, tests/native/test_bin_bucket.cpp).
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

GHOSTM_SEED_HD constexpr uint32_t CeilLog2(uint32_t v) {
  uint32_t l = 0;
  while ((1u << l) < v) ++l;
  return l;
}

// v_mul_u32_u24: the low 32 bits of the product of both operands' low 24 bits.
// (__umul24 is int-typed: its result is cast before any shift.)
GHOSTM_SEED_HD inline uint32_t Mul24(uint32_t x, uint32_t y) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__umul24(x, y);
#else
  return (uint32_t)((uint64_t)(x & 0xFFFFFFu) * (uint64_t)(y & 0xFFFFFFu));
#endif
}

// K1 bins are < 2^21 (the hash path's limit); BinBucket must hold for every
// bin <= kHashBinLimit + 1 (the emission also looks up b + 1).
constexpr uint32_t kHashBinLimit = 1u << 21;

// The bucket of bin b in a table of `buckets` buckets. HASH24: b * C from a
// full-rate 24-bit multiply, then ((h >> s) * buckets) >> (32 - s) with
// 2^s >= buckets, so the product stays below 2^32 and the bucket below
// `buckets`. Else the 32-bit multiplicative hash's high word.
template <uint32_t kBuckets, bool HASH24>
GHOSTM_SEED_HD inline uint32_t BinBucket(uint32_t b) {
  if constexpr (HASH24) {
    constexpr uint32_t kS = CeilLog2(kBuckets);
    static_assert(kS >= 8 && kS < 24, "(h >> s) and the bucket count fit 24 bits");
    const uint32_t h = Mul24(b, 0x9E3779u);
    return Mul24(h >> kS, kBuckets) >> (32 - kS);
  } else {
    return (uint32_t)(((uint64_t)(b * 2654435761u) * kBuckets) >> 32);
  }
}

}  // namespace kern
}  // namespace ghostm
