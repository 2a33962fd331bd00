// aligner.h — the `aln` driver: the reference Aligner (aligner.h:42-92,
// aligner.cpp:65-1012) re-built around the gfx950 device module.
//
// Same options, same chunk loops, same batch cuts, same Merge order (libstdc++
// std::sort), same tie rules and the same text output as the reference CPU path.
// Seed search, score DP, merge selection and traceback run on the GPU when a query
// chunk is one batch against one DB chunk (the common case, and the benchmark);
// otherwise the merge runs on host threads with the reference's exact semantics.
// Output text is produced by a background formatter while the GPU works on the
// next segment.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ghostm_hip.h"
#include "device.h"
#include "formats.h"
#include "scoring.h"

namespace ghostm {

struct LineFormat;  // output line writer with per-session caches (aligner.cpp)

// reference AlignerOption (aligner.h:42-61), defaults of SetOption (aligner.cpp:226-243)
struct AlignerOptions {
  std::string output_file;
  std::string query_prefix;
  std::string db_prefix;
  uint32_t start_query_chunk = UINT32_MAX;
  uint32_t end_query_chunk = UINT32_MAX;
  uint32_t log_region = 4;
  uint32_t shift = 2;
  uint32_t threshold = 2;
  uint32_t max_list_length = 1u << 27;
  int open_gap = -11;
  int extend_gap = -1;
  uint32_t extend = 2;
  uint32_t best = 10;
  int device = 0;            // -D; the GPU path is the only path here
  int output_style = 0;      // -y
  bool verbose = false;
  ScoreMatrix matrix;
  KarlinParams karlin;
};

// getopt "b:d:D:e:E:G:i:l:M:o:r:s:t:S:L:y:v" (aligner.cpp:248); throws
// std::invalid_argument like the reference.
AlignerOptions ParseAlignerOptions(int argc, char **argv);

// A resolved hit: what the reference keeps in an Alignment (alignment.h:136-145).
struct HitRecord {
  uint32_t query = 0;        // index within its query chunk
  uint32_t db_chunk = 0;
  uint32_t subject = 0;      // index within its DB chunk
  uint32_t score = 0;
  uint32_t start = 0;        // absolute until traceback + rebase, then subject-relative
  uint32_t end = 0;
  uint32_t aln_len = 0;
  uint32_t aln_match = 0;
  float seq_id = 0.f;
};

// Number of host worker threads: GHOSTM_THREADS, else this process's share of
// the CPUs it may run on (affinity mask, cgroup quota) divided among the ranks
// of this node (LOCAL_WORLD_SIZE), between 1 and 16.
unsigned HostThreads();

// One batch of the reference's batch loop (aligner.cpp:131-171 with
// SearchNextCpu's cut, :511-514): queries [q0, q1) of a query chunk.
struct Batch {
  uint32_t q0, q1;
};

// The CPU path's batch cuts of one query chunk against one DB chunk, from every
// query's candidate count.
std::vector<Batch> CpuBatches(const std::vector<uint32_t> &counts, uint64_t max_list);

// The collective a rank-local shard session uses at creation
// (GhostmSessionCreateShardEx): an all-gather of byte buffers in rank order.
struct ShardExchange {
  GhostmAllGatherFn fn = nullptr;
  void *ctx = nullptr;
};

// Parallel for over [0, n) in contiguous blocks.
void ParallelFor(size_t n, unsigned threads, const std::function<void(size_t, size_t, unsigned)> &fn);
// ... in PieceCount(n, pieces) contiguous blocks, claimed in order by at most
// `threads` threads (fn's third argument is the block's index)
size_t PieceCount(size_t n, size_t pieces);
void ParallelForPieces(size_t n, size_t pieces, unsigned threads,
                       const std::function<void(size_t, size_t, unsigned)> &fn);

// One background thread running submitted tasks in order.
class TaskQueue {
 public:
  TaskQueue();
  ~TaskQueue();
  void Submit(std::function<void()> fn);
  void Drain();  // waits for every submitted task; rethrows the first error
 private:
  void Loop();
  std::mutex mu_;
  std::condition_variable cv_, idle_;
  std::deque<std::function<void()>> tasks_;
  bool stop_ = false, busy_ = false;
  std::exception_ptr error_;
  std::thread worker_;
};

// Multi-GPU shards: cuts[0..world] splitting n queries into
// contiguous ranges of about equal total weight, cut only where group_start[i]
// is set (a name group's first query); ghostm_amd/shard.py balanced_cuts is the
// same rule.
void ShardCuts(uint64_t n, const uint32_t *weight, const uint8_t *group_start, uint32_t world, uint64_t *cuts);

class Session {
 public:
  // shard_rank/shard_world: search only that shard of the query set (one
  // process per GPU); the shards' outputs concatenated in rank order are the
  // unsharded output, and hit records keep global query indices. Every shard
  // replays the unsharded run's batch cuts (the batch plan, fixed here): with
  // `exchange`, the rank reads and counts only its own queries and the ranks
  // all-gather their candidate counts; without, the rank counts every query
  // of the set itself once.
  explicit Session(const AlignerOptions &opt, uint32_t shard_rank = 0, uint32_t shard_world = 1,
                   const ShardExchange *exchange = nullptr);
  uint64_t ShardBegin() const { return shard_begin_; }
  uint64_t ShardEnd() const { return shard_end_; }
  // the most hit records one run can return: name groups x max(-b, 1)
  uint64_t HitCapacity() const;
  ~Session();

  // whole search; replaces previous results. stream_to_file: also write the
  // output file (-o) while the search runs, each segment's text as soon as it
  // is formatted, in order (WriteOutputFile is then a no-op for this run)
  void Run(bool stream_to_file = false);
  const std::string &Output();         // text of the last run (joined on first use)
  void WriteOutputFile();
  const std::vector<GhostmHit> &Hits();
  // Hit records of the last run in device memory (this session's GPU): copies
  // min(n, cap) records to dst_device; returns n.
  size_t DeviceHits(void *dst_device, size_t cap);
  const GhostmStats &Stats() const { return stats_; }

 private:
  struct QueryData {
    QueryChunk chunk;
    DevQuery *dev = nullptr;
    std::vector<uint32_t> group_end;   // per query: one past the last query of its name group
    std::vector<uint32_t> group_first, group_last;  // name groups in order
    std::vector<uint32_t> qlen;        // WriteOutput's query length (last non-X + 1)
    uint32_t global_base = 0;          // index of the chunk's first query over all chunks
    // shard sessions: this slice is queries [slice_lo, slice_lo + nseq) of a
    // chunk of chunk_nseq queries, and plan[d] holds the whole chunk's batch
    // cuts against DB chunk d (chunk indices); plan_sum[d] / plan_hash[d] are
    // the slice's candidate total and count hash, checked on every run
    bool planned = false;
    uint32_t slice_lo = 0, chunk_nseq = 0;
    std::vector<std::vector<Batch>> plan;
    std::vector<uint64_t> plan_sum, plan_hash;
  };
  struct DbData {
    DbChunk chunk;
    DevDb *dev = nullptr;
    uint32_t global_base = 0;
  };
  // Output of one segment: one piece per formatting worker, in output order.
  // Parts are reused across runs, so their buffers keep their capacity (no
  // release and re-fault of ~100 bytes per hit on every run).
  struct Part {
    std::vector<std::string> text;
    std::vector<std::vector<GhostmHit>> hits;
    // a streamed run (FormatSelected) writes each piece as soon as it is
    // formatted, in order: the formatting workers mark pieces done, the writer
    // waits for the next one; Abandon (formatting failed) releases the writer
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint8_t> done;
    bool abandoned = false, streaming = false;
    void Reset(size_t pieces);
    void MarkDone(size_t k);
    void Abandon();
    bool Wait(size_t k);  // false: abandoned before piece k was formatted
  };
  using Results = std::vector<std::vector<HitRecord>>;

  static void PrepareQueryChunk(QueryData *q, bool qlen = true);
  void QueryLengths(std::vector<QueryData *> chunks);
  void ApplyShard(uint32_t rank, uint32_t world);
  // shard sessions: the batch plan of every (query chunk, DB chunk)
  void PlanFromCounts(QueryData &q, size_t di, const std::vector<uint32_t> &chunk_counts, uint32_t n);
  void Create(uint32_t shard_rank, uint32_t shard_world, const ShardExchange *ex);
  void Load(uint32_t shard_rank, uint32_t shard_world, bool local, std::vector<uint32_t> *chunk_nseq,
            std::vector<std::vector<uint64_t>> *rank_lo);
  void AgreeOnCreate(uint32_t rank, uint32_t world, const ShardExchange &ex, const std::string &err,
                     const std::vector<uint32_t> &chunk_nseq, const std::vector<std::vector<uint64_t>> &rank_lo);
  void PlanExchange(uint32_t rank, uint32_t world, const ShardExchange &ex,
                    const std::vector<uint32_t> &chunk_nseq, const std::vector<std::vector<uint64_t>> &rank_lo);
  // the passes of one Seed() result: the plan's batches restricted to the
  // slice (local indices, possibly empty), or the slice's own cuts unsharded
  // (total: the counts' sum when known, else UINT64_MAX)
  std::vector<Batch> Passes(QueryData &q, size_t di, const std::vector<uint32_t> &counts,
                            uint64_t total = UINT64_MAX) const;
  void RunQueryChunk(QueryData &q);
  void RunQueryChunkHostMerge(QueryData &q);
  void DevicePass(QueryData &q, DbData &d, const std::vector<uint32_t> &counts,
                  const std::vector<uint64_t> &offsets, uint32_t bq0, uint32_t bq1, uint64_t c_lo, uint64_t c_hi,
                  bool carry_in, bool final_pass);
  void HostMergeBatch(QueryData &q, DbData &d, uint32_t bq0, uint32_t bq1, uint64_t cand_begin,
                      const uint32_t *score, const uint32_t *end, const std::vector<uint32_t> &counts,
                      const std::vector<uint64_t> &offsets, Results *results);
  void FormatResults(const QueryData &q, const Results &results, Part *out);
  void FormatSelected(const QueryData &q, uint32_t g0, const std::vector<uint32_t> &counts,
                      const HostHits &hits, uint32_t cap, Part *out);
  Part *NewPart();
  // a part's text is complete: hands it to the output writer when streaming
  void PartDone(const Part *part);
  void StreamPart(Part *part);
  const LineFormat &Format();

  AlignerOptions opt_;
  uint64_t shard_begin_ = 0, shard_end_ = UINT64_MAX;  // query range over the loaded chunks
  uint32_t shard_world_ = 1;
  std::vector<QueryData> queries_;
  std::vector<DbData> dbs_;
  uint32_t db_sum_u32_ = 0;           // DBReader::GetSumDbLength() truncates to u32
  uint64_t merge_epoch_ = 0;
  std::deque<Part> parts_;             // parts_[0, used_parts_) hold the last run
  size_t used_parts_ = 0;
  std::string joined_;
  bool joined_valid_ = false;
  std::vector<GhostmHit> hits_;
  bool hits_valid_ = false;
  bool records_on_device_ = false;
  GhostmStats stats_{};
  unsigned threads_ = 1;
  std::unique_ptr<TaskQueue> formatter_;
  std::unique_ptr<TaskQueue> writer_;  // streamed output (Run(true)), in part order
  int stream_fd_ = -1;
  bool run_sync_ = true;  // drain the streams at run and chunk starts (Run)
  std::vector<uint32_t> seed_counts_;  // K1 counts/offsets of the current chunk (RunQueryChunk)
  std::vector<uint64_t> seed_offsets_;
  uint64_t stream_off_ = 0;
  bool stream_failed_ = false, streamed_ = false;
  std::unique_ptr<LineFormat> format_;
};

}  // namespace ghostm
