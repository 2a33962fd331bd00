// K1's exact bin table (kernels.h BinTable): every bucket BinBucket returns must
// lie inside the table, for every bin the kernels can look up (b <= kHashBinLimit
// + 1: the emission reads c(b + 1)) and for every table size the library
// instantiates (passed as -DBUCKETS=..., parsed from device.hip by
// tests/test_seed_lists.py). Round 5's hang (profiles/r5au/): the
// int-typed __umul24 result was shifted arithmetically, the bucket fell outside
// the table and the unbounded probe loop never met an empty slot. The negative
// control below recomputes that signed form and must find out-of-range buckets.
#include <cstdio>
#include <cstdlib>

#include "../../ghostm_amd/csrc/seed_lists.h"

using ghostm::kern::BinBucket;
using ghostm::kern::CeilLog2;
using ghostm::kern::kHashBinLimit;
using ghostm::kern::Mul24;

template <uint32_t kBuckets>
static int Check() {
  int bad = 0;
  uint64_t signed_bad = 0;
  uint32_t lo = kBuckets, hi = 0;
  for (uint32_t b = 0; b <= kHashBinLimit + 1; ++b) {
    const uint32_t k24 = BinBucket<kBuckets, true>(b), k32 = BinBucket<kBuckets, false>(b);
    if (k24 >= kBuckets || k32 >= kBuckets) {
      if (bad++ < 5) printf("buckets %u: bin %u -> %u / %u\n", kBuckets, b, k24, k32);
    }
    lo = k24 < lo ? k24 : lo;
    hi = k24 > hi ? k24 : hi;
    // the round-5 form: (int)__umul24(...) >> (32 - s), an arithmetic shift
    constexpr uint32_t kS = CeilLog2(kBuckets);
    const int p = (int)Mul24(Mul24(b, 0x9E3779u) >> kS, kBuckets);
    if ((uint32_t)(p >> (32 - kS)) >= kBuckets) ++signed_bad;
  }
  printf("buckets %u: range [%u, %u], signed-shift form out of range for %llu bins\n", kBuckets, lo, hi,
         (unsigned long long)signed_bad);
  if (hi != kBuckets - 1 || lo != 0) {
    printf("buckets %u: the hash does not reach the whole table\n", kBuckets);
    ++bad;
  }
  if (signed_bad == 0) {
    printf("buckets %u: negative control found nothing\n", kBuckets);
    ++bad;
  }
  return bad;
}

template <uint32_t... B>
static int CheckAll() {
  return (Check<B>() + ... + 0);
}

int main() {
  const int bad = CheckAll<BUCKETS>();
  if (bad) {
    printf("FAILED (%d)\n", bad);
    return 1;
  }
  printf("all buckets in range\n");
  return 0;
}
