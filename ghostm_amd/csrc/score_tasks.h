// score_tasks.h — K2 task lists (host only; included by device.hip, unit-tested
// with g++ by tests/native/test_score_tasks.cpp). A task is one workgroup of
// k_score*: up to per_block candidates and the profiles of the queries they
// belong to.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <utility>
#include <vector>

#include "score_task.h"


namespace ghostm {

// Runs fn(k) for k in [0, parts) on host worker threads and returns when all are
// done (the session's ParallelFor; null = one thread).
using HostParallelFn = std::function<void(size_t parts, const std::function<void(size_t)> &fn)>;

// K2 tasks: runs of <= per_block consecutive candidates spanning <= Qmax queries,
// written straight into page-locked staging (no fresh host vector per segment:
// its first touch cost more than the loop). A task closes when full, when it
// spans Qmax queries, or at the end, so ScoreTaskBound is an upper bound.
inline size_t ScoreTaskBound(uint64_t n, uint32_t q_first, uint32_t q_end, uint32_t per_block, uint32_t qmax) {
  // paired unit tasks: full blocks plus at most one remainder task per query
  return (size_t)(n / per_block) + (q_end - q_first) + 2;
}
inline size_t BuildScoreTasks(uint64_t cand_begin, uint64_t n, uint32_t q_first, uint32_t q_end,
                              const std::vector<uint32_t> &counts, const std::vector<uint64_t> &offsets,
                              uint32_t per_block, uint32_t qmax, kern::ScoreTask *out) {
  size_t nt = 0;
  kern::ScoreTask cur{};
  bool open_task = false;
  auto flush = [&]() {
    if (open_task && cur.count) out[nt++] = cur;
    open_task = false;
  };
  const uint64_t cand_end = cand_begin + n;
  for (uint32_t qi = q_first; qi < q_end; ++qi) {
    uint64_t lo = std::max<uint64_t>(offsets[qi], cand_begin);
    const uint64_t hi = std::min<uint64_t>(offsets[qi] + counts[qi], cand_end);
    while (lo < hi) {
      if (open_task && (cur.count == per_block || qi - cur.q_first >= qmax)) flush();
      if (!open_task) {
        cur = kern::ScoreTask{};
        cur.begin = lo;
        cur.q_first = qi;
        open_task = true;
      }
      const uint64_t take = std::min<uint64_t>(hi - lo, per_block - cur.count);
      cur.count += (uint32_t)take;
      cur.q_count = qi - cur.q_first + 1;
      // the unit kernel reads a task as two ranges: the first query's
      // candidates, then (contiguous here) the second query's
      if (qi == cur.q_first) cur.count1 += (uint32_t)take;
      cur.begin2 = cur.begin + cur.count1;
      cur.q_second = cur.q_first + 1;
      lo += take;
    }
  }
  flush();
  return nt;
}

// Tasks of k_score16f's unit-pair kernel (two query profiles per block): each
// query's candidates in full blocks of per_block, and the remainders paired two
// queries to a block, best fit: each remainder (largest first) takes the
// largest remainder that still fits beside it. A block holds its LDS rows for
// a whole wave-duration however few of its waves are live (the LDS, not the
// waves, limits the unit kernel to four blocks per CU), so what counts is the
// number of blocks. At 63 candidates per query (cfg 3) consecutive runs of two
// queries make 17 % more blocks than the pairs (Poisson counts: 58.4 K against
// 50.0 K per 100 K queries); from ~80 per query on they win instead (pairs of
// remainders above 64 cannot share a block, consecutive runs split queries).
inline size_t BuildScoreTasksPaired(uint64_t cand_begin, uint64_t n, uint32_t q_first, uint32_t q_end,
                                    const std::vector<uint32_t> &counts, const std::vector<uint64_t> &offsets,
                                    uint32_t per_block, kern::ScoreTask *out) {
  size_t nt = 0;
  auto single = [&](uint32_t q, uint64_t begin, uint32_t count) {
    kern::ScoreTask t{};
    t.begin = begin;
    t.count = count;
    t.count1 = count;
    t.q_first = q;
    t.q_count = 1;
    t.begin2 = begin + count;
    t.q_second = q;
    out[nt++] = t;
  };
  // the remainders (query, first candidate) grouped by size with a counting
  // sort (flat arrays; a per-size stack of vectors cost ~1 ms per segment on
  // the critical path of a chunk's first segment)
  const uint64_t cand_end = cand_begin + n;
  std::vector<uint32_t> start(per_block + 1, 0);
  auto range = [&](uint32_t qi, uint64_t *lo, uint64_t *hi) {
    *lo = std::max<uint64_t>(offsets[qi], cand_begin);
    *hi = std::min<uint64_t>(offsets[qi] + counts[qi], cand_end);
  };
  for (uint32_t qi = q_first; qi < q_end; ++qi) {
    uint64_t lo, hi;
    range(qi, &lo, &hi);
    if (lo < hi && (hi - lo) % per_block) ++start[(hi - lo) % per_block + 1];
  }
  for (uint32_t r = 1; r <= per_block; ++r) start[r] += start[r - 1];
  std::vector<uint32_t> top(start.begin(), start.end() - 1);  // fill cursor per size
  std::vector<std::pair<uint32_t, uint64_t>> rem(start[per_block]);
  for (uint32_t qi = q_first; qi < q_end; ++qi) {
    uint64_t lo, hi;
    range(qi, &lo, &hi);
    if (lo >= hi) continue;
    while (hi - lo >= per_block) {
      single(qi, lo, per_block);
      lo += per_block;
    }
    if (hi > lo) rem[top[hi - lo]++] = {qi, lo};
  }
  // greedy best fit, largest first; a size's entries are taken from the end
  // of its range (top[r] = one past the last unused entry of size r)
  for (uint32_t r1 = per_block - 1; r1 >= 1; --r1) {
    while (top[r1] > start[r1]) {
      const std::pair<uint32_t, uint64_t> a = rem[--top[r1]];
      uint32_t pick = 0;
      for (uint32_t r2 = std::min(r1, per_block - r1); r2 >= 1 && !pick; --r2)
        if (top[r2] > start[r2]) pick = r2;
      if (!pick) {
        single(a.first, a.second, r1);
        continue;
      }
      const std::pair<uint32_t, uint64_t> b = rem[--top[pick]];
      kern::ScoreTask t{};
      t.begin = a.second;
      t.count1 = r1;
      t.q_first = a.first;
      t.begin2 = b.second;
      t.q_second = b.first;
      t.count = r1 + pick;
      t.q_count = 2;
      out[nt++] = t;
    }
  }
  return nt;
}

// Consecutive runs of at most qmax queries without building them: the blocks
// the 16-bit-row kernel (four query profiles per block) would launch.
inline size_t CountScoreTasks(uint64_t cand_begin, uint64_t n, uint32_t q_first, uint32_t q_end,
                              const std::vector<uint32_t> &counts, const std::vector<uint64_t> &offsets,
                              uint32_t per_block, uint32_t qmax) {
  size_t nt = 0;
  uint32_t cur = 0, open_q = 0;
  bool open_task = false;
  const uint64_t cand_end = cand_begin + n;
  for (uint32_t qi = q_first; qi < q_end; ++qi) {
    uint64_t lo = std::max<uint64_t>(offsets[qi], cand_begin);
    const uint64_t hi = std::min<uint64_t>(offsets[qi] + counts[qi], cand_end);
    while (lo < hi) {
      if (open_task && (cur == per_block || qi - open_q >= qmax)) {
        ++nt;
        open_task = false;
      }
      if (!open_task) {
        cur = 0;
        open_q = qi;
        open_task = true;
      }
      const uint64_t take = std::min<uint64_t>(hi - lo, per_block - cur);
      cur += (uint32_t)take;
      lo += take;
    }
  }
  return nt + (open_task && cur ? 1 : 0);
}

// BuildScoreTasks in parts on host threads: the query range is cut into parts,
// each part's tasks counted (CountScoreTasks), then written at the part's
// prefix. A task never spans two parts (a part starts a fresh task), which
// changes only how candidates are grouped into blocks, never a score; at most
// one task more per part, inside ScoreTaskBound's one-per-query slack. A
// chunk's first segment builds its tasks while the GPU waits (125 K-query shard:
// 74 K tasks, 0.34 ms on one thread, profiles/r5ap/). GHOSTM_K2_TASKS_PAR=0 keeps
// one thread (A/B).
inline size_t BuildScoreTasksParallel(uint64_t cand_begin, uint64_t n, uint32_t q_first, uint32_t q_end,
                                      const std::vector<uint32_t> &counts, const std::vector<uint64_t> &offsets,
                                      uint32_t per_block, uint32_t qmax, kern::ScoreTask *out,
                                      const HostParallelFn *par) {
  constexpr uint32_t kPartQueries = 4096;
  const uint32_t nqr = q_end > q_first ? q_end - q_first : 0;
  const char *e = getenv("GHOSTM_K2_TASKS_PAR");
  if (!par || !*par || nqr < 2 * kPartQueries || (e && strcmp(e, "0") == 0))
    return BuildScoreTasks(cand_begin, n, q_first, q_end, counts, offsets, per_block, qmax, out);
  const size_t parts = std::min<size_t>(16, nqr / kPartQueries);
  auto cut = [&](size_t k) { return q_first + (uint32_t)((uint64_t)nqr * k / parts); };
  std::vector<size_t> at(parts + 1, 0);
  (*par)(parts, [&](size_t k) {
    at[k + 1] = CountScoreTasks(cand_begin, n, cut(k), cut(k + 1), counts, offsets, per_block, qmax);
  });
  for (size_t k = 0; k < parts; ++k) at[k + 1] += at[k];
  (*par)(parts, [&](size_t k) {
    BuildScoreTasks(cand_begin, n, cut(k), cut(k + 1), counts, offsets, per_block, qmax, out + at[k]);
  });
  return at[parts];
}

// The blocks BuildScoreTasksPaired would make, from a histogram of the
// remainders (no tasks built).
// Blocks the pairing makes from a histogram of remainder sizes (rem[r] =
// remainders of size r; rem[0] ignored): BuildScoreTasksPaired's greedy in
// batches, every remainder of size r1 taking the same partner size while
// partners of that size last.
inline size_t PairedFromRemainders(std::vector<uint64_t> rem, uint32_t per_block) {
  size_t nt = 0;
  rem[0] = 0;
  for (uint32_t r1 = per_block - 1; r1 >= 1; --r1) {
    while (rem[r1]) {
      uint32_t r2 = std::min(r1, per_block - r1);
      while (r2 >= 1 && !(r2 == r1 ? rem[r1] >= 2 : rem[r2] >= 1)) --r2;
      if (r2 == 0) {
        nt += rem[r1];  // no partner fits: singles
        rem[r1] = 0;
      } else if (r2 == r1) {
        const uint64_t k = rem[r1] / 2;
        nt += k;
        rem[r1] -= 2 * k;
      } else {
        const uint64_t k = std::min(rem[r1], rem[r2]);
        nt += k;
        rem[r1] -= k;
        rem[r2] -= k;
      }
    }
  }
  return nt;
}

// The blocks BuildScoreTasksPaired would make (no tasks built).
inline size_t CountPairedTasks(uint64_t cand_begin, uint64_t n, uint32_t q_first, uint32_t q_end,
                               const std::vector<uint32_t> &counts, const std::vector<uint64_t> &offsets,
                               uint32_t per_block) {
  std::vector<uint64_t> rem(per_block, 0);
  size_t full = 0;
  const uint64_t cand_end = cand_begin + n;
  for (uint32_t qi = q_first; qi < q_end; ++qi) {
    const uint64_t lo = std::max<uint64_t>(offsets[qi], cand_begin);
    const uint64_t hi = std::min<uint64_t>(offsets[qi] + counts[qi], cand_end);
    if (lo >= hi) continue;
    full += (hi - lo) / per_block;
    ++rem[(hi - lo) % per_block];
  }
  return full + PairedFromRemainders(std::move(rem), per_block);
}

// The three block counts the chooser compares, in one pass over the queries:
// consecutive runs of two and of four queries (CountScoreTasks) and the pairs
// (CountPairedTasks).
inline void CountTasks(uint64_t cand_begin, uint64_t n, uint32_t q_first, uint32_t q_end,
                       const std::vector<uint32_t> &counts, const std::vector<uint64_t> &offsets, uint32_t per_block,
                       size_t *n2, size_t *n4, size_t *np) {
  struct Runs {
    uint32_t qmax, cur = 0, open_q = 0;
    bool open = false;
    size_t nt = 0;
    void Add(uint32_t qi, uint64_t len, uint32_t per_block) {
      while (len) {
        if (open && (cur == per_block || qi - open_q >= qmax)) {
          ++nt;
          open = false;
        }
        if (!open) {
          cur = 0;
          open_q = qi;
          open = true;
        }
        const uint64_t take = std::min<uint64_t>(len, per_block - cur);
        cur += (uint32_t)take;
        len -= take;
      }
    }
    size_t Done() const { return nt + (open && cur ? 1 : 0); }
  } two{kern::kScoreQmaxUnit}, four{kern::kScoreQmax};
  std::vector<uint64_t> rem(per_block, 0);
  size_t full = 0;
  const uint64_t cand_end = cand_begin + n;
  for (uint32_t qi = q_first; qi < q_end; ++qi) {
    const uint64_t lo = std::max<uint64_t>(offsets[qi], cand_begin);
    const uint64_t hi = std::min<uint64_t>(offsets[qi] + counts[qi], cand_end);
    if (lo >= hi) continue;
    two.Add(qi, hi - lo, per_block);
    four.Add(qi, hi - lo, per_block);
    full += (hi - lo) / per_block;
    ++rem[(hi - lo) % per_block];
  }
  *n2 = two.Done();
  *n4 = four.Done();
  *np = full + PairedFromRemainders(rem, per_block);
}

// Sparse segments (k_score_pair): each query's candidates in pairs, the local
// index (from cand_begin) of a pair's first candidate, kPairSingle set when it
// has no second (a query's odd last one). Returns the number of pairs; `out`
// has room for n entries.
// With `par` and many queries the query range is cut into parts: each part's
// pairs are counted, then written at the part's prefix (the same list).
inline size_t BuildScorePairs(uint64_t cand_begin, uint64_t n, uint32_t q_first, uint32_t q_end,
                              const std::vector<uint32_t> &counts, const std::vector<uint64_t> &offsets,
                              uint32_t *out, const HostParallelFn *par = nullptr) {
  const uint64_t cand_end = cand_begin + n;
  auto write = [&](uint32_t qa, uint32_t qb, size_t np) {
    for (uint32_t qi = qa; qi < qb; ++qi) {
      const uint64_t lo = std::max<uint64_t>(offsets[qi], cand_begin);
      const uint64_t hi = std::min<uint64_t>(offsets[qi] + counts[qi], cand_end);
      for (uint64_t c = lo; c < hi; c += 2)
        out[np++] = (uint32_t)(c - cand_begin) | (c + 1 < hi ? 0u : kern::kPairSingleBit);
    }
    return np;
  };
  constexpr uint32_t kPartQueries = 4096;
  const uint32_t nqr = q_end > q_first ? q_end - q_first : 0;
  if (!par || !*par || nqr < 2 * kPartQueries) return write(q_first, q_end, 0);
  const size_t parts = std::min<size_t>(16, nqr / kPartQueries);
  auto cut = [&](size_t k) { return q_first + (uint32_t)((uint64_t)nqr * k / parts); };
  std::vector<size_t> at(parts + 1, 0);
  (*par)(parts, [&](size_t k) {
    size_t np = 0;
    for (uint32_t qi = cut(k); qi < cut(k + 1); ++qi) {
      const uint64_t lo = std::max<uint64_t>(offsets[qi], cand_begin);
      const uint64_t hi = std::min<uint64_t>(offsets[qi] + counts[qi], cand_end);
      if (hi > lo) np += (size_t)((hi - lo + 1) / 2);
    }
    at[k + 1] = np;
  });
  for (size_t k = 0; k < parts; ++k) at[k + 1] += at[k];
  (*par)(parts, [&](size_t k) { write(cut(k), cut(k + 1), at[k]); });
  return at[parts];
}

// Which K2 kernel runs a segment (ScoreKind) and its work list.
enum ScoreKind { kScoreRows = 0, kScoreUnit = 1, kScorePairs = 2, kScoreRowsSparse = 3 };
// below this many candidates per query the pair-table kernel runs (cfg 2: ~9
// per query, K2 5.1 -> 3.4 ms per step, profiles/r5d/; at cfg 3's 63 per query
// it lost to the unit kernel, 14.8 -> 18.4 ms; GHOSTM_K2_PAIR_MAX overrides,
// GHOSTM_K2=pair forces it)
constexpr uint64_t kScorePairMax = 16;

// The K2 tasks of a segment, and which kernel runs them (GHOSTM_K2=unit|swar16
// and GHOSTM_K2_TASKS=paired|consecutive force a choice). With 16-bit integer
// patterns (swar) the unit-pair kernel is used where its blocks, each ~7 %
// cheaper (6.5 instead of 7.5 VALU instructions per row pair; same box,
// cfg 4: 19.00 against 20.30 ms per launch), are at most 1.07x as many as the
// 16-bit-row kernel's (four queries per block). Its tasks are consecutive runs
// of two queries unless the pairs make at least 5 % fewer blocks: at equal
// counts the runs measured faster (cfg 4: 19.0 against 19.5 ms per launch),
// at 63 candidates per query the pairs (cfg 3: 4.83 against 5.57 ms, 14 %
// fewer blocks). Only the chosen list is built; the others are counted.
// Below kScorePairMax candidates per query (and with integer patterns) the
// segment runs k_score_pair over BuildScorePairs' list instead, written into
// `out` as uint32 entries. `out` has room for ScoreTaskBound(...) tasks and n
// uint32 entries. pairs_ok = false (a launch with the re-score guard, which
// only k_score16f implements) keeps the profile kernels.
// Sparse segments run the 16-bit-row profile kernel at 16 rows per lane with
// kScoreQmaxSparse profiles per block (kScoreRowsSparse, `sparse_per_block`
// candidates per block; 0 = not available for this query width / DB): cfg 2 K2
// 3.33-3.40 against 3.38-3.46 ms per step with k_score_pair, two boxes
// (profiles/r6i/, profiles/r6j/: 7 profiles per block beat 6, 5, 4 — block fill
// over occupancy). GHOSTM_K2_SPARSE=pair keeps k_score_pair (A/B), GHOSTM_K2=sparse
// forces the rows kernel at any density.
inline bool SparseRowsDefault() {
  const char *e = getenv("GHOSTM_K2_SPARSE");
  return !(e && strcmp(e, "pair") == 0);
}

inline size_t BuildTasks(bool swar, uint64_t cand_begin, uint64_t n, uint32_t q_first, uint32_t q_end,
                         const std::vector<uint32_t> &counts, const std::vector<uint64_t> &offsets,
                         uint32_t per_block, kern::ScoreTask *out, int *kind_out, bool pairs_ok = true,
                         const HostParallelFn *par = nullptr, uint32_t sparse_per_block = 0) {
  const char *k2 = getenv("GHOSTM_K2");
  const char *how = getenv("GHOSTM_K2_TASKS");
  const bool force_unit = k2 && strcmp(k2, "unit") == 0, force_rows = k2 && strcmp(k2, "swar16") == 0;
  const bool force_pair = k2 && strcmp(k2, "pair") == 0;
  const bool force_sparse = k2 && strcmp(k2, "sparse") == 0 && sparse_per_block;
  bool unit = false, paired = false;
  const uint64_t per_query = n / std::max<uint32_t>(1, q_end - q_first);
  uint64_t pair_max = kScorePairMax;
  if (const char *e = getenv("GHOSTM_K2_PAIR_MAX")) pair_max = strtoull(e, nullptr, 10);
  if (swar && q_end > q_first && (force_sparse || (!force_pair && sparse_per_block && pairs_ok && !force_unit &&
                                                    !force_rows && !how && per_query < pair_max &&
                                                    SparseRowsDefault()))) {
    *kind_out = kScoreRowsSparse;
    return BuildScoreTasksParallel(cand_begin, n, q_first, q_end, counts, offsets, sparse_per_block,
                                   kern::SparseSlots(), out, par);
  }
  if (swar && pairs_ok && q_end > q_first && !force_unit && !force_rows && !how &&
      (force_pair || per_query < pair_max)) {
    *kind_out = kScorePairs;
    return BuildScorePairs(cand_begin, n, q_first, q_end, counts, offsets, reinterpret_cast<uint32_t *>(out), par);
  }
  if (swar && q_end > q_first && !force_rows && !how && !force_unit && per_query >= 96) {
    unit = true;  // dense (cfg 4: 127 per query): runs of two queries fill their blocks, no count needed
  } else if (swar && q_end > q_first && !force_rows && (how || force_unit || per_query >= 24)) {
    // (the count is on the critical path of a chunk's first segment: ~0.5 ms
    // per 125 K queries; below 24 per query the rows kernel always won)
    size_t nc, n4, np;
    CountTasks(cand_begin, n, q_first, q_end, counts, offsets, per_block, &nc, &n4, &np);
    paired = how ? strcmp(how, "paired") == 0 : np * 100 <= nc * 95;
    const size_t nu = paired ? np : nc;
    unit = force_unit || nu * 100 <= n4 * 107;
    if (getenv("GHOSTM_DEBUG_TASKS"))
      fprintf(stderr, "k2 tasks: %llu candidates, %u queries: consecutive(2) %zu, paired %zu, consecutive(4) %zu -> %s\n",
              (unsigned long long)n, q_end - q_first, nc, np, n4, unit ? (paired ? "unit paired" : "unit consecutive") : "rows");
  }
  *kind_out = unit ? kScoreUnit : kScoreRows;
  if (unit && paired) return BuildScoreTasksPaired(cand_begin, n, q_first, q_end, counts, offsets, per_block, out);
  return BuildScoreTasksParallel(cand_begin, n, q_first, q_end, counts, offsets, per_block,
                                 unit ? kern::kScoreQmaxUnit : kern::kScoreQmax, out, par);
}

}  // namespace ghostm
