// Checks ghostm_amd/csrc/libstdcxx_sort.h against the real libstdc++ std::sort:
// identical permutations of (score, index) pairs under "score descending" (the
// reference's AlignmentComp), on tie-heavy random inputs of many sizes, plus
// sorted / reversed / constant inputs that drive the heap-sort fallback.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#include "../../ghostm_amd/csrc/libstdcxx_sort.h"

struct Item {
  uint32_t score, idx;
};

int main(int argc, char **argv) {
  const long trials = argc > 1 ? atol(argv[1]) : 200000;
  std::mt19937_64 rng(12345);
  auto less = [](const Item &a, const Item &b) { return a.score > b.score; };
  long bad = 0, total = 0;
  long lazy_bad = 0;
  auto check = [&](std::vector<Item> v) {
    std::vector<Item> a = v, b = v, c = v;
    std::sort(a.begin(), a.end(), less);
    ghostm::stdsort::Sort(b.data(), (long)b.size(), less);
    ++total;
    for (size_t i = 0; i < a.size(); ++i)
      if (a[i].idx != b[i].idx) { ++bad; return; }
    // lazy form: every finalized prefix already equals std::sort's
    ghostm::stdsort::LazySort<Item, decltype(less)> ls(c.data(), (long)c.size(), less);
    long prev = 0;
    while (ls.Advance()) {
      if (ls.done <= prev || ls.done > (long)c.size()) { ++lazy_bad; return; }
      for (long i = prev; i < ls.done; ++i)
        if (a[i].idx != c[i].idx) { ++lazy_bad; return; }
      prev = ls.done;
    }
    if (prev != (long)c.size()) ++lazy_bad;
  };
  for (long t = 0; t < trials; ++t) {
    const long n = (long)(rng() % (t % 10 == 0 ? 2000 : 300));
    const uint32_t range = 1 + (uint32_t)(rng() % (t % 3 == 0 ? 4 : t % 3 == 1 ? 40 : 4000));
    std::vector<Item> v(n);
    for (long i = 0; i < n; ++i) v[i] = Item{(uint32_t)(rng() % range), (uint32_t)i};
    check(v);
  }
  for (long n : {0L, 1L, 2L, 15L, 16L, 17L, 33L, 100L, 1000L, 5000L}) {
    std::vector<Item> v(n);
    for (long i = 0; i < n; ++i) v[i] = Item{(uint32_t)i, (uint32_t)i};
    check(v);
    std::reverse(v.begin(), v.end());
    for (long i = 0; i < n; ++i) v[i].idx = (uint32_t)i;
    check(v);
    for (long i = 0; i < n; ++i) v[i] = Item{7u, (uint32_t)i};
    check(v);
    // median-of-3 killer style input to reach the depth limit
    for (long i = 0; i < n; ++i) v[i] = Item{(uint32_t)((i % 2) ? i : n - i), (uint32_t)i};
    check(v);
  }
  // the depth-limit fallback == std::partial_sort(first, last, last) (make_heap + sort_heap)
  long heap_bad = 0;
  for (long t = 0; t < trials / 10; ++t) {
    const long n = (long)(rng() % 500);
    const uint32_t range = 1 + (uint32_t)(rng() % (t % 2 ? 5 : 1000));
    std::vector<Item> a(n);
    for (long i = 0; i < n; ++i) a[i] = Item{(uint32_t)(rng() % range), (uint32_t)i};
    std::vector<Item> b = a;
    std::partial_sort(a.begin(), a.end(), a.end(), less);
    ghostm::stdsort::HeapSortRange(b.data(), b.data() + n, less);
    for (long i = 0; i < n; ++i)
      if (a[i].idx != b[i].idx) { ++heap_bad; break; }
  }
  bad += heap_bad + lazy_bad;
  printf("lazy prefixes: %ld mismatches\n", lazy_bad);
  printf("heap fallback: %ld mismatches\n", heap_bad);
  printf("stdsort emulation: %ld arrays, %ld mismatches\n", total, bad);
  return bad != 0;
}
