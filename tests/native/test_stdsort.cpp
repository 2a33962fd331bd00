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

// k_merge_wave's partition (ghostm_amd/csrc/kernels.h), restated sequentially
// from the two stop lists of the input: left stops = positions in
// [first+1, last) whose element is not less than the pivot (ascending), right
// stops = positions in [first, last) the pivot is not less than (ascending,
// used from the end). Pairs k = 1, 2, ... are swapped while the k-th left stop
// lies below the k-th right stop from the end; the cut is the first failing
// left stop, or the last swapped right stop when that comes first.
template <class T, class Less> T *StopListPartition(T *first, T *last, Less less) {
  std::vector<long> ls(1, 0), rs(1, 0);  // 1-based
  for (T *x = first; x < last; ++x) {
    if (x > first && !less(*x, *first)) ls.push_back(x - first);
    if (!less(*first, *x)) rs.push_back(x - first);
  }
  const long nl = (long)ls.size() - 1, nr = (long)rs.size() - 1;
  long kf = nl + 1;
  for (long k = 1; k <= nl; ++k)
    if (!(k <= nr && rs[nr + 1 - k] > ls[k])) { kf = k; break; }
  for (long k = 1; k < kf; ++k) std::swap(first[ls[k]], first[rs[nr + 1 - k]]);
  long cut = kf <= nl ? ls[kf] : (long)(last - first);
  if (kf >= 2) cut = std::min(cut, rs[nr + 2 - kf]);
  return first + cut;
}

// std::sort with that partition (otherwise stdsort::Sort's loop)
template <class T, class Less> void StopListSort(T *first, long n, Less less) {
  namespace ss = ghostm::stdsort;
  if (n <= 0) return;
  T *last = first + n;
  struct Frame {
    T *first, *last;
    int depth;
  };
  std::vector<Frame> stack{Frame{first, last, ss::Lg(n) * 2}};
  while (!stack.empty()) {
    Frame f = stack.back();
    stack.pop_back();
    while (f.last - f.first > ss::kThreshold) {
      if (f.depth == 0) {
        ss::HeapSortRange(f.first, f.last, less);
        break;
      }
      --f.depth;
      T *mid = f.first + (f.last - f.first) / 2;
      ss::MoveMedianToFirst(f.first, f.first + 1, mid, f.last - 1, less);
      T *cut = StopListPartition(f.first, f.last, less);
      stack.push_back(Frame{cut, f.last, f.depth});
      f.last = cut;
    }
  }
  if (n > ss::kThreshold) {
    ss::InsertionSort(first, first + ss::kThreshold, less);
    for (T *i = first + ss::kThreshold; i != last; ++i) ss::UnguardedLinearInsert(i, less);
  } else {
    ss::InsertionSort(first, last, less);
  }
}

int main(int argc, char **argv) {
  const long trials = argc > 1 ? atol(argv[1]) : 200000;
  std::mt19937_64 rng(12345);
  auto less = [](const Item &a, const Item &b) { return a.score > b.score; };
  long bad = 0, total = 0;
  long lazy_bad = 0, stop_bad = 0;
  auto check = [&](std::vector<Item> v) {
    std::vector<Item> a = v, b = v, c = v, d = v;
    std::sort(a.begin(), a.end(), less);
    ghostm::stdsort::Sort(b.data(), (long)b.size(), less);
    StopListSort(d.data(), (long)d.size(), less);
    ++total;
    for (size_t i = 0; i < a.size(); ++i)
      if (a[i].idx != d[i].idx) { ++stop_bad; break; }
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
  bad += heap_bad + lazy_bad + stop_bad;
  printf("stop-list partition (k_merge_wave): %ld mismatches\n", stop_bad);
  printf("lazy prefixes: %ld mismatches\n", lazy_bad);
  printf("heap fallback: %ld mismatches\n", heap_bad);
  printf("stdsort emulation: %ld arrays, %ld mismatches\n", total, bad);
  return bad != 0;
}
