// score_task.h — one K2 workgroup's work (shared by the kernels in kernels.h and
// the host task builders in score_tasks.h).
#pragma once
#include <cstdint>

namespace ghostm {
namespace kern {

constexpr int kScoreQmax = 4;       // query profiles per K2 block (16-bit rows)
constexpr int kScoreQmaxUnit = 2;   // k_score16f UNIT: 32-bit profile words, half the queries per block
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
