// K1 phase 0 (ghostm_amd/csrc/seed_lists.h ListBytes16): the byte table of
// entry -> list index built from the list boundaries inside each 16-entry
// window must equal a per-entry walk over the offsets, on random list sets with
// empty, one-entry and long lists (entries past the last list are not compared:
// the kernel never reads them).
#include <cstdio>
#include <random>
#include <vector>

#include "../../ghostm_amd/csrc/seed_lists.h"

int main() {
  std::mt19937 rng(7);
  const uint32_t lens[] = {0, 0, 0, 1, 2, 3, 5, 15, 16, 17, 40, 120, 300};
  int trials = 0;
  for (int t = 0; t < 4000; ++t) {
    const uint32_t nl = 1 + rng() % 128;
    std::vector<uint32_t> off(nl + 1, 0);
    for (uint32_t j = 0; j < nl; ++j) off[j + 1] = off[j] + lens[rng() % (sizeof(lens) / sizeof(lens[0]))];
    const uint32_t n = off[nl];
    for (uint32_t e0 = 0; e0 < n; e0 += 16) {
      uint32_t j = 0;
      while (off[j + 1] <= e0) ++j;
      uint32_t wv[4];
      ghostm::kern::ListBytes16(e0, j, off.data(), nl, wv);
      uint32_t jw = j;  // the walk
      for (uint32_t k = 0; k < 16 && e0 + k < n; ++k) {
        while (off[jw + 1] <= e0 + k) ++jw;
        const uint32_t got = (wv[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        if (got != jw) {
          std::printf("mismatch: trial %d nl %u e0 %u k %u: %u != %u\n", t, nl, e0, k, got, jw);
          return 1;
        }
      }
    }
    ++trials;
  }
  std::printf("%d trials ok\n", trials);
  return 0;
}
