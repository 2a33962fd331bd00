// libstdcxx_sort.h — the exact element permutation of libstdc++'s std::sort
// (GCC 11 bits/stl_algo.h: __introsort_loop, __unguarded_partition_pivot,
// __move_median_to_first, __final_insertion_sort; bits/stl_heap.h for the
// depth-limit fallback), usable on host and device.
//
// The reference merges hits with std::sort (aligner.cpp:702, 745), which is not
// stable: the order of equal scores is whatever introsort leaves, and that order
// decides which subject wins a tie and therefore the printed hit list. A device
// merge must reproduce the permutation, not just "a" sort. std::sort's moves and
// swaps depend only on comparison outcomes, so running the same algorithm on
// (score, index) pairs with the same comparator yields the same permutation.
// The recursion on the right partition is replaced by an explicit stack: the two
// partitions are disjoint and the final insertion pass runs over the whole range
// afterwards, so the processing order of partitions does not change the result.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GHOSTM_HD __host__ __device__ inline
#else
#define GHOSTM_HD inline
#endif

namespace ghostm {
namespace stdsort {

constexpr long kThreshold = 16;  // _S_threshold

template <class T> GHOSTM_HD void Swap(T *a, T *b) {
  T t = *a;
  *a = *b;
  *b = t;
}

GHOSTM_HD int Lg(long n) {  // std::__lg: floor(log2(n))
  int r = -1;
  while (n) { n >>= 1; ++r; }
  return r;
}

template <class T, class Less>
GHOSTM_HD void PushHeap(T *first, long hole, long top, T value, Less less) {
  long parent = (hole - 1) / 2;
  while (hole > top && less(first[parent], value)) {
    first[hole] = first[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  first[hole] = value;
}

template <class T, class Less>
GHOSTM_HD void AdjustHeap(T *first, long hole, long len, T value, Less less) {
  const long top = hole;
  long child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (less(first[child], first[child - 1])) child--;
    first[hole] = first[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    first[hole] = first[child - 1];
    hole = child - 1;
  }
  PushHeap(first, hole, top, value, less);
}

template <class T, class Less> GHOSTM_HD void HeapSortRange(T *first, T *last, Less less) {
  // __partial_sort(first, last, last): __make_heap then __sort_heap
  const long len = last - first;
  if (len >= 2) {
    long parent = (len - 2) / 2;
    while (true) {
      AdjustHeap(first, parent, len, first[parent], less);
      if (parent == 0) break;
      parent--;
    }
  }
  while (last - first > 1) {
    --last;
    T value = *last;
    *last = *first;
    AdjustHeap(first, 0L, (long)(last - first), value, less);
  }
}

template <class T, class Less>
GHOSTM_HD void MoveMedianToFirst(T *result, T *a, T *b, T *c, Less less) {
  if (less(*a, *b)) {
    if (less(*b, *c)) Swap(result, b);
    else if (less(*a, *c)) Swap(result, c);
    else Swap(result, a);
  } else if (less(*a, *c)) {
    Swap(result, a);
  } else if (less(*b, *c)) {
    Swap(result, c);
  } else {
    Swap(result, b);
  }
}

template <class T, class Less> GHOSTM_HD T *UnguardedPartition(T *first, T *last, T *pivot, Less less) {
  while (true) {
    while (less(*first, *pivot)) ++first;
    --last;
    while (less(*pivot, *last)) --last;
    if (!(first < last)) return first;
    Swap(first, last);
    ++first;
  }
}

template <class T, class Less> GHOSTM_HD void UnguardedLinearInsert(T *last, Less less) {
  T val = *last;
  T *next = last - 1;
  while (less(val, *next)) {
    *last = *next;
    last = next;
    --next;
  }
  *last = val;
}

template <class T, class Less> GHOSTM_HD void InsertionSort(T *first, T *last, Less less) {
  if (first == last) return;
  for (T *i = first + 1; i != last; ++i) {
    if (less(*i, *first)) {
      T val = *i;
      for (T *p = i; p != first; --p) *p = *(p - 1);
      *first = val;
    } else {
      UnguardedLinearInsert(i, less);
    }
  }
}

// std::sort(first, first + n, less)
template <class T, class Less> GHOSTM_HD void Sort(T *first, long n, Less less) {
  if (n <= 0) return;
  T *last = first + n;
  struct Frame {
    T *first, *last;
    int depth;
  };
  Frame stack[96];
  int sp = 0;
  stack[sp++] = Frame{first, last, Lg(n) * 2};
  while (sp > 0) {
    Frame f = stack[--sp];
    while (f.last - f.first > kThreshold) {
      if (f.depth == 0) {
        HeapSortRange(f.first, f.last, less);
        break;
      }
      --f.depth;
      T *mid = f.first + (f.last - f.first) / 2;
      MoveMedianToFirst(f.first, f.first + 1, mid, f.last - 1, less);
      T *cut = UnguardedPartition(f.first + 1, f.last, f.first, less);
      stack[sp++] = Frame{cut, f.last, f.depth};
      f.last = cut;
    }
  }
  if (n > kThreshold) {
    InsertionSort(first, first + kThreshold, less);
    for (T *i = first + kThreshold; i != last; ++i) UnguardedLinearInsert(i, less);
  } else {
    InsertionSort(first, last, less);
  }
}

// Lazy form of Sort: finalizes the array left to right, one partition at a
// time, so a caller that only needs a prefix (the Merge walk stops after -b
// subjects) skips the rest. After Advance() returns true, [first, first + done)
// holds exactly what std::sort leaves there: introsort's partitions are
// disjoint and ordered (every element of a left part is not "less" than any of
// its right part), so the final insertion pass never moves an element across a
// partition boundary and may be run per partition; a heap-sorted partition is
// already in order. Right parts wait on a stack; LIFO order is left to right.
template <class T, class Less> struct LazySort {
  struct Frame {
    T *first, *last;
    int depth;
  };
  T *base;
  Less less;
  Frame stack[96];
  int sp = 0;
  long done = 0;
  GHOSTM_HD LazySort(T *first, long n, Less l) : base(first), less(l) {
    if (n > 0) stack[sp++] = Frame{first, first + n, Lg(n) * 2};
  }
  GHOSTM_HD bool Advance() {
    if (sp == 0) return false;
    Frame f = stack[--sp];
    while (f.last - f.first > kThreshold) {
      if (f.depth == 0) {
        HeapSortRange(f.first, f.last, less);
        done = f.last - base;
        return true;
      }
      --f.depth;
      T *mid = f.first + (f.last - f.first) / 2;
      MoveMedianToFirst(f.first, f.first + 1, mid, f.last - 1, less);
      T *cut = UnguardedPartition(f.first + 1, f.last, f.first, less);
      stack[sp++] = Frame{cut, f.last, f.depth};
      f.last = cut;
    }
    InsertionSort(f.first, f.last, less);
    done = f.last - base;
    return true;
  }
};

}  // namespace stdsort
}  // namespace ghostm
