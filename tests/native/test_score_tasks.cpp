// K2 task lists (ghostm_amd/csrc/score_tasks.h) on random candidate counts:
// every candidate of the segment is in exactly one task, each task's candidates
// belong to the queries whose profiles it builds (the unit kernel reads a task
// as two ranges, the others as one consecutive run over q_first..), and no
// task exceeds a workgroup. The sparse kernel's pair lists: every candidate in
// exactly one pair, both candidates of a pair of one query, the single flag
// only on a query's odd last candidate.
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

#include "../../ghostm_amd/csrc/score_tasks.h"

using ghostm::kern::ScoreTask;

static int Check(const char *what, const std::vector<ScoreTask> &tasks, size_t nt, bool unit, uint32_t qmax,
                 uint64_t cand_begin, uint64_t n, const std::vector<uint32_t> &qid_of, uint32_t per_block) {
  std::vector<int> seen(n, 0);
  for (size_t k = 0; k < nt; ++k) {
    const ScoreTask &t = tasks[k];
    if (t.count == 0 || t.count > per_block) { printf("%s: task %zu has %u candidates\n", what, k, t.count); return 1; }
    for (uint32_t l = 0; l < t.count; ++l) {
      uint64_t c;
      uint32_t q;
      if (unit) {
        const bool second = l >= t.count1;
        c = second ? t.begin2 + (l - t.count1) : t.begin + l;
        q = second ? t.q_second : t.q_first;
        if (t.q_count != (t.count1 < t.count ? 2u : 1u)) { printf("%s: task %zu q_count\n", what, k); return 1; }
      } else {
        c = t.begin + l;
        q = qid_of[c];
        if (q < t.q_first || q - t.q_first >= t.q_count || t.q_count > qmax) {
          printf("%s: task %zu query outside its slots\n", what, k);
          return 1;
        }
      }
      if (c < cand_begin || c >= cand_begin + n) { printf("%s: task %zu candidate outside\n", what, k); return 1; }
      if (qid_of[c] != q) { printf("%s: task %zu candidate %llu of query %u read as %u\n", what, k,
                                   (unsigned long long)c, qid_of[c], q); return 1; }
      if (seen[c - cand_begin]++) { printf("%s: candidate twice\n", what); return 1; }
    }
  }
  for (uint64_t c = 0; c < n; ++c)
    if (!seen[c]) { printf("%s: candidate %llu missing\n", what, (unsigned long long)(c + cand_begin)); return 1; }
  return 0;
}

static int CheckPairs(const uint32_t *pairs, size_t np, uint64_t cand_begin, uint64_t n,
                      const std::vector<uint32_t> &qid_of) {
  std::vector<int> seen(n, 0);
  for (size_t k = 0; k < np; ++k) {
    const bool single = pairs[k] & ghostm::kern::kPairSingleBit;
    const uint64_t a = pairs[k] & ~ghostm::kern::kPairSingleBit;
    if (a >= n || (!single && a + 1 >= n)) { printf("pair %zu outside the segment\n", k); return 1; }
    if (seen[a]++) { printf("pair %zu: candidate twice\n", k); return 1; }
    if (!single) {
      if (seen[a + 1]++) { printf("pair %zu: second candidate twice\n", k); return 1; }
      if (qid_of[cand_begin + a] != qid_of[cand_begin + a + 1]) { printf("pair %zu spans two queries\n", k); return 1; }
    } else if (a + 1 < n && qid_of[cand_begin + a] == qid_of[cand_begin + a + 1]) {
      printf("pair %zu single though its query has a next candidate\n", k);
      return 1;
    }
  }
  for (uint64_t c = 0; c < n; ++c)
    if (!seen[c]) { printf("pairs: candidate %llu missing\n", (unsigned long long)c); return 1; }
  return 0;
}

int main() {
  std::mt19937_64 rng(7);
  const uint32_t per_block = 128, wave_slots = 32;
  uint64_t trials = 0, paired_waves = 0, consec_waves = 0;
  for (int trial = 0; trial < 400; ++trial) {
    const uint32_t nq = 1 + rng() % 400;
    const double mean = (double)(rng() % 300);
    std::vector<uint32_t> counts(nq);
    std::vector<uint64_t> offsets(nq);
    std::poisson_distribution<uint32_t> pois(mean);
    uint64_t total = 0;
    for (uint32_t q = 0; q < nq; ++q) {
      counts[q] = (rng() % 7 == 0) ? 0 : pois(rng);
      offsets[q] = total;
      total += counts[q];
    }
    std::vector<uint32_t> qid_of(total);
    for (uint32_t q = 0; q < nq; ++q)
      for (uint32_t c = 0; c < counts[q]; ++c) qid_of[offsets[q] + c] = q;
    if (!total) continue;
    // a segment: a candidate range that may start and end inside queries
    const uint64_t b = rng() % total, e = b + 1 + rng() % (total - b);
    uint32_t q0 = 0, q1 = nq;
    while (q0 < nq && offsets[q0] + counts[q0] <= b) ++q0;
    while (q1 > 0 && offsets[q1 - 1] >= e) --q1;
    const uint64_t n = e - b;
    for (int mode = 0; mode < 5; ++mode) {
      const bool unit = true;
      const uint32_t qmax = 2;
      // room for the bound's tasks and for n pair entries
      std::vector<ScoreTask> tasks(std::max<size_t>(ghostm::ScoreTaskBound(n, q0, q1, per_block, qmax),
                                                    n * 4 / sizeof(ScoreTask) + 1));
      if (mode == 4) {  // the sparse kernel's pairs
        const size_t np = ghostm::BuildScorePairs(b, n, q0, q1, counts, offsets, reinterpret_cast<uint32_t *>(tasks.data()));
        if (CheckPairs(reinterpret_cast<const uint32_t *>(tasks.data()), np, b, n, qid_of)) return 1;
        continue;
      }
      size_t nt;
      const char *what;
      if (mode == 0) {
        what = "paired";
        nt = ghostm::BuildScoreTasksPaired(b, n, q0, q1, counts, offsets, per_block, tasks.data());
        if (nt != ghostm::CountPairedTasks(b, n, q0, q1, counts, offsets, per_block)) {
          printf("CountPairedTasks %zu disagrees with BuildScoreTasksPaired %zu\n",
                 ghostm::CountPairedTasks(b, n, q0, q1, counts, offsets, per_block), nt);
          return 1;
        }
      } else if (mode == 1) {
        what = "consecutive (unit)";
        nt = ghostm::BuildScoreTasks(b, n, q0, q1, counts, offsets, per_block, qmax, tasks.data());
      } else if (mode == 2) {
        what = "consecutive (unit, counted)";
        nt = ghostm::BuildScoreTasks(b, n, q0, q1, counts, offsets, per_block, qmax, tasks.data());
        if (nt != ghostm::CountScoreTasks(b, n, q0, q1, counts, offsets, per_block, qmax)) {
          printf("CountScoreTasks disagrees (two queries)\n");
          return 1;
        }
      } else {
        {
          size_t c2, c4, cp;
          ghostm::CountTasks(b, n, q0, q1, counts, offsets, per_block, &c2, &c4, &cp);
          if (c2 != ghostm::CountScoreTasks(b, n, q0, q1, counts, offsets, per_block, 2) ||
              c4 != ghostm::CountScoreTasks(b, n, q0, q1, counts, offsets, per_block, 4) ||
              cp != ghostm::CountPairedTasks(b, n, q0, q1, counts, offsets, per_block)) {
            printf("CountTasks disagrees with the single counters\n");
            return 1;
          }
        }
        what = "chosen kernel";
        int kind = -1;
        nt = ghostm::BuildTasks(true, b, n, q0, q1, counts, offsets, per_block, tasks.data(), &kind);
        if (kind == ghostm::kScorePairs) {  // sparse: fewer than kScorePairMax per query
          if (n / std::max<uint32_t>(1, q1 - q0) >= ghostm::kScorePairMax) { printf("pairs chosen when dense\n"); return 1; }
          if (CheckPairs(reinterpret_cast<const uint32_t *>(tasks.data()), nt, b, n, qid_of)) return 1;
          ++trials;
          continue;
        }
        const bool unit_k = kind == ghostm::kScoreUnit;
        if (Check(what, tasks, nt, unit_k, unit_k ? 2u : 4u, b, n, qid_of, per_block)) return 1;
        if (!unit_k && nt != ghostm::CountScoreTasks(b, n, q0, q1, counts, offsets, per_block, 4)) {
          printf("CountScoreTasks disagrees with BuildScoreTasks\n");
          return 1;
        }
        ++trials;
        continue;
      }
      if (nt > tasks.size()) { printf("%s: %zu tasks over the bound %zu\n", what, nt, tasks.size()); return 1; }
      if (Check(what, tasks, nt, unit, qmax, b, n, qid_of, per_block)) return 1;
      uint64_t w = 0;
      for (size_t k = 0; k < nt; ++k) w += (tasks[k].count + wave_slots - 1) / wave_slots;
      if (mode == 0) paired_waves += w;
      if (mode == 1) consec_waves += w;
    }
  }
  // the pair list built in parts on threads equals the one-thread list
  // (BuildScorePairs with a HostParallelFn, many queries)
  for (int trial = 0; trial < 20; ++trial) {
    const uint32_t nq = 8192 + (uint32_t)(rng() % 60000);
    std::vector<uint32_t> counts(nq);
    std::vector<uint64_t> offsets(nq);
    std::poisson_distribution<uint32_t> pois(1.0 + (double)(rng() % 20));
    uint64_t total = 0;
    for (uint32_t q = 0; q < nq; ++q) {
      offsets[q] = total;
      counts[q] = rng() % 5 == 0 ? 0 : pois(rng);
      total += counts[q];
    }
    if (total < 2) continue;
    const uint64_t b = rng() % (total / 2), e = total - rng() % (total / 4 + 1);
    uint32_t q0 = 0, q1 = nq;
    while (q0 < nq && offsets[q0] + counts[q0] <= b) ++q0;
    while (q1 > 0 && offsets[q1 - 1] >= e) --q1;
    std::vector<uint32_t> one(e - b + 1), many(e - b + 1);
    const size_t n1 = ghostm::BuildScorePairs(b, e - b, q0, q1, counts, offsets, one.data());
    ghostm::HostParallelFn par = [](size_t parts, const std::function<void(size_t)> &fn) {
      std::vector<std::thread> ts;
      for (size_t k = parts; k-- > 0;) ts.emplace_back(fn, k);  // parts started in reverse order
      for (auto &t : ts) t.join();
    };
    const size_t n2 = ghostm::BuildScorePairs(b, e - b, q0, q1, counts, offsets, many.data(), &par);
    if (n1 != n2 || !std::equal(one.begin(), one.begin() + (long)n1, many.begin())) {
      printf("parallel pair list differs (%zu against %zu pairs, %u queries)\n", n2, n1, q1 - q0);
      return 1;
    }
    // consecutive tasks built in parts on threads (a part starts a fresh task):
    // every candidate once, every task within per_block and qmax, inside the
    // bound; two and four queries per block, and the sparse kernel's seven
    std::vector<uint32_t> qid_of(total);
    for (uint32_t q = 0; q < nq; ++q)
      for (uint32_t c = 0; c < counts[q]; ++c) qid_of[offsets[q] + c] = q;
    for (uint32_t qmax : {2u, 4u, 7u}) {
      const uint32_t pb = qmax == 7 ? 64u : per_block;
      std::vector<ScoreTask> tasks(ghostm::ScoreTaskBound(e - b, q0, q1, pb, qmax));
      const size_t nt = ghostm::BuildScoreTasksParallel(b, e - b, q0, q1, counts, offsets, pb, qmax, tasks.data(), &par);
      if (nt > tasks.size()) { printf("parallel tasks over the bound\n"); return 1; }
      if (Check("consecutive in parts", tasks, nt, qmax == 2, qmax, b, e - b, qid_of, pb)) return 1;
    }
    // the chosen kernel with the sparse rows kernel available: below
    // kScorePairMax per query it takes seven-profile tasks of 64 candidates
    {
      std::vector<ScoreTask> tasks(std::max<size_t>(ghostm::ScoreTaskBound(e - b, q0, q1, 64, 7),
                                                    (e - b) * 4 / sizeof(ScoreTask) + 1));
      int kind = -1;
      const size_t nt = ghostm::BuildTasks(true, b, e - b, q0, q1, counts, offsets, per_block, tasks.data(), &kind,
                                           true, &par, 64);
      if ((e - b) / std::max<uint32_t>(1, q1 - q0) < ghostm::kScorePairMax) {
        if (kind != ghostm::kScoreRowsSparse) { printf("sparse segment without the sparse kernel\n"); return 1; }
        if (Check("sparse rows", tasks, nt, false, 7, b, e - b, qid_of, 64)) return 1;
      }
    }
    ++trials;
  }
  printf("%llu trials ok; waves: paired %llu, consecutive %llu\n", (unsigned long long)trials,
         (unsigned long long)paired_waves, (unsigned long long)consec_waves);
  return 0;
}
