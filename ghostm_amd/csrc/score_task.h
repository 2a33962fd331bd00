// score_task.h — one K2 workgroup's work (shared by the kernels in kernels.h and
// the host task builders in score_tasks.h).
#pragma once
#include <cstdint>
#include <cstdlib>

namespace ghostm {
namespace kern {

constexpr int kScoreQmax = 4;       // query profiles per K2 block (16-bit rows)
constexpr int kScoreQmaxUnit = 2;   // k_score16f UNIT: 32-bit profile words, half the queries per block
// k_score16f<16, true> over sparse segments (kScoreRowsSparse): 16 rows per
// lane (64 candidates per block), the profiles of up to 7 queries with their 27
// code rows (0..24, END, fill): 53 KB, three blocks per CU
constexpr int kScoreQmaxSparse = 7;
// (GHOSTM_K2_SPARSE_SLOTS = 1..7 lowers it, A/B)
inline uint32_t SparseSlots() {
  static const uint32_t v = [] {
    const char *e = getenv("GHOSTM_K2_SPARSE_SLOTS");
    const int k = e ? atoi(e) : kScoreQmaxSparse;
    return (uint32_t)(k >= 1 && k <= kScoreQmaxSparse ? k : kScoreQmaxSparse);
  }();
  return v;
}
constexpr uint32_t kProfRowsSparse = 27;
constexpr uint32_t kPairSingleBit = 0x80000000u;  // k_score_pair entry: a pair without its second candidate

struct ScoreTask {
  unsigned long long begin;  // first candidate (global index)
  uint32_t count;            // candidates in this task
  uint32_t q_first;          // first query of the task (profile slot 0)
  uint32_t q_count;          // profile slots used
  // k_score16f UNIT (paired tasks, BuildScoreTasksPaired): candidates
  // [begin, begin + count1) of query q_first (slot 0), then [begin2, begin2 +
  // count - count1) of query q_second (slot 1); the other kernels take
  // [begin, begin + count) over the consecutive queries q_first.. instead
  uint32_t count1;
  unsigned long long begin2;
  uint32_t q_second;
  uint32_t pad;
};

}  // namespace kern
}  // namespace ghostm
