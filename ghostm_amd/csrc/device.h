// device.h — host-side interface of the gfx950 device module (device.hip).
//
// The module owns one HIP device per process, one stream, the score tables and
// the resident query/DB chunks, and runs the three kernel families of the `aln`
// hot path:
//   K1 seed      k-mer lists -> diagonal-bin candidates   (SearchNextCpu, aligner.cpp:383-521)
//   K2 score     Gotoh local score + end per candidate    (CalculateScoreCpu, aligner.cpp:545-685)
//   K3 traceback reverse DP -> start, length, matches    (TraceBack, aligner.cpp:771-949)
// Everything on the device is exact integer work; the host keeps the merge
// (libstdc++ std::sort order) and the float E-value formatting.
#pragma once
#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace ghostm {

namespace kern {
struct TbArgs;
}

struct SeedConfig {
  uint32_t seed_mask = 15;   // index seed bits (db -k 4 -> 0b1111)
  uint32_t threshold = 2;    // aln -t
  uint32_t shift = 2;        // aln -s
  uint32_t log_region = 4;   // log2(aln -r)
};

struct GapConfig {
  uint32_t extend = 2;       // aln -e
  uint32_t log_region = 4;
  int open = -11;            // negated -G
  int ext = -1;              // negated -E
};

// Device-resident chunk handles (opaque to callers).
struct DevQuery;
struct DevDb;

// One hit chosen by the device merge (K4), after its traceback (K3):
// subject-relative coordinates, ml = (aln_len << 8) | matches.
struct SelectedHit {
  uint32_t sid, score, start, end, ml, chunk;  // chunk: the hit's DB chunk
};

// Selected hits landed on the host: an uninitialised block, freed when the last
// copy of `block` goes (the formatter releases it).
struct HostHits {
  std::shared_ptr<void> block;
  SelectedHit *data = nullptr;
  size_t n = 0;
  const SelectedHit &operator[](size_t i) const { return data[i]; }
};

// One K4 pass: the batch's candidate range (absolute; a batch may cut a name
// group) and the carried result lists (reference result_list, aligner.cpp:114):
// carry_in merges them with the batch's candidates, carry_out keeps the new
// lists for the next batch or DB chunk.
struct MergePass {
  uint64_t cand_lo = 0, cand_hi = UINT64_MAX;
  bool carry_in = false, carry_out = false;
  uint32_t chunk = 0;  // DB chunk id of the new hits
};

struct DeviceTimes {
  double seed = 0, score = 0, traceback = 0, merge = 0;  // seconds of device time (HIP events)
  double traceback_scan = 0;  // ... of which K3's scan phase (prep, pairs, sorts, k_tb_scan)
  uint64_t seed_bytes = 0, seed_list_entries = 0;
  uint64_t score_launches = 0, score_launches_packed = 0, score_launches_half = 0;
  uint64_t score_cells = 0, traceback_cells = 0;
  uint64_t traceback_launches = 0, traceback_launches_key = 0;
  uint64_t seed_launches_hash = 0;  // Seed() calls whose slot pass used k_seed_hash
  uint64_t score_rechecks = 0;      // guarded f16 candidates re-scored in int16
  uint64_t traceback_launches_scan = 0, traceback_scan_cells = 0;  // K3a scores-only pass
  uint64_t score_launches_framed = 0;  // f16 K2 launches of the column-framed kernel (k_score16f)
  uint64_t merge_launches = 0, merge_launches_wave = 0;            // K4 (k_merge_wave: one wave per group)
  uint64_t seed_queries_class[4] = {0, 0, 0, 0};  // K1 queries per size class (3 = global merge)
  uint64_t seed_queries_wide = 0;                 // ... redone by the offset pass (more than a slot)
  uint64_t seed_launches_filter = 0;              // Seed() calls whose classes 0/1 ran k_seed_filter
  uint64_t traceback_launches_scan_swar = 0;  // K3a scans over 16-bit integer patterns
  uint64_t traceback_launches_strips = 0;  // key DPs run by strip class (lanes of strips 0..i* only)
  uint64_t score_launches_swar = 0;  // ... of the framed kernel over 16-bit integer patterns (k_score16f<S, true>)
  uint64_t score_launches_unit = 0;  // ... of its unit-pair profile variant (k_score16f<S, true, true>)
  uint64_t score_launches_pair = 0;  // sparse segments: the pair-table kernel (k_score_pair)
  uint64_t seed_compact_redo = 0;    // K1 compactions re-run by the host (overflow, buffer growth)
  uint64_t seed_filter_overflows = 0;             // ... queries redone by k_seed_hash (queue overflow)
  uint64_t score_launches_levels = 0;             // K2 launches with restart levels (k_score16f<S, true, false, true>)
  uint64_t traceback_launches_keyframe = 0;       // K3 key DPs with the column-framed E chain (k_traceback_key FRAME)
  uint64_t score_launches_sparse = 0;             // K2 launches of sparse segments run by k_score16f<16, true> (kScoreRowsSparse)
  uint64_t seed_table_full = 0;                   // ... queries redone by k_seed (bin table probe bound reached)
  uint64_t traced_hits = 0;                       // device merge: hits selected from new candidates (K3 run)
};

class DeviceModule {
 public:
  struct Impl;  // device.hip
  static DeviceModule &Get();

  void Bind(int device);                 // hipSetDevice + stream; idempotent; one device per process
  void Use() const;                      // make the bound device current on this thread
  int device() const { return device_; }
  void SetMatrix(const int *m32x32);     // M[db*32 + q]
  std::string DeviceName() const;
  size_t TotalMemory() const;

  // Copies n bytes host to host (the session sets a parallel one; default memcpy).
  using HostCopyFn = std::function<void(void *dst, const void *src, size_t n)>;
  void SetHostCopy(HostCopyFn fn);
  // Runs fn(k), k < parts, on host worker threads (the session sets its pool;
  // used by the K2 pair-list build and K1's count pass).
  using HostParallelFn = std::function<void(size_t parts, const std::function<void(size_t)> &fn)>;
  void SetHostParallel(HostParallelFn fn);
  // Host to device through page-locked staging on the main stream (see device.hip).
  void StagedUpload(void *dst, const void *src, size_t bytes);
  DevQuery *UploadQuery(const uint8_t *seq, uint32_t nseq, uint32_t L);
  DevDb *UploadDb(const uint8_t *seq, uint32_t len, const uint32_t *keys_count, uint32_t kcl,
                  const uint32_t *positions, uint32_t npos);
  // Name groups of a query chunk (consecutive equal names), for the device merge.
  void SetQueryGroups(DevQuery *q, const uint32_t *first, const uint32_t *last, uint32_t ng);
  // Subject start offsets (.pos) of a DB chunk, for the device merge.
  void SetDbSubjects(DevDb *d, const uint32_t *starts, uint32_t nsubj);
  void Free(DevQuery *q);
  void Free(DevDb *d);

  // K1 over every query of q against d. On return: counts[nseq] (host) and the
  // compact device candidate arrays (start, qid) ordered by (query, start).
  // offsets[q] = first candidate of query q. Returns total candidates.
  uint64_t Seed(DevQuery *q, DevDb *d, const SeedConfig &cfg, std::vector<uint32_t> *counts,
                std::vector<uint64_t> *offsets);
  // Copy candidate starts [begin, begin+n) to host.
  void CopyStarts(uint64_t begin, uint64_t n, uint32_t *out);

  // K2 over candidates [cand_begin, cand_begin + n) whose queries are
  // [q_first, q_end) with per-query counts/offsets as returned by Seed.
  // Scores/ends land in host arrays score[n], end[n] (when not null). With
  // `next`, the host builds and uploads the next segment's tasks while this
  // launch runs, and the Score() call for that segment launches at once.
  struct ScoreSegment {
    uint64_t cand_begin, n;
    uint32_t q_first, q_end;
  };
  void Score(DevQuery *q, DevDb *d, uint64_t cand_begin, uint64_t n, uint32_t q_first,
             uint32_t q_end, const std::vector<uint32_t> &counts,
             const std::vector<uint64_t> &offsets, uint32_t base_search_length,
             const GapConfig &gap, uint32_t *score, uint32_t *end, const ScoreSegment *next = nullptr);
  // Score() in two steps for the device-merge pipeline: ScoreLaunch enqueues K2
  // and uploads `next`'s tasks (copy stream) with no host wait; ScoreFinish
  // waits for K2 and re-scores its guard list. A guarded launch (ScoreGuarded)
  // must be finished before anything reads its scores.
  void ScoreLaunch(DevQuery *q, DevDb *d, uint64_t cand_begin, uint64_t n, uint32_t q_first, uint32_t q_end,
                   const std::vector<uint32_t> &counts, const std::vector<uint64_t> &offsets,
                   uint32_t base_search_length, const GapConfig &gap, const ScoreSegment *next);
  bool ScoreGuarded() const;
  void ScoreFinish();
  // With ScoreDeferNext(true), ScoreLaunch only records `next`; ScorePrepareNext
  // builds and uploads its tasks (call it after enqueueing the segment's K4/K3).
  void ScoreDeferNext(bool on) { defer_next_ = on; }
  void ScorePrepareNext(const std::vector<uint32_t> &counts, const std::vector<uint64_t> &offsets);

  uint32_t ScorePerBlock(DevQuery *q, uint32_t base_search_length, const GapConfig &gap) const;

  // K4 + K3 for a batch that covers every group of the chunk and starts from
  // empty result lists (first batch, first DB chunk): the reference Merge
  // selection on the device, then the traceback of every selected hit. Uses the
  // scores/ends left on the device by the preceding Score() over the same range.
  // counts[g] hits per group; hits[g*cap + k], cap = max(best, 1) (hits may be
  // null: nothing but the counts is copied back).
  void MergeSelect(DevQuery *q, DevDb *d, uint32_t g0, uint32_t g1, uint64_t cand_begin, uint64_t n, uint32_t best,
                   uint32_t tb_base, int open, int ext, std::vector<uint32_t> *counts,
                   HostHits *hits, const MergePass &pass = MergePass());
  // MergeSelect in two steps: MergeLaunch enqueues K4/K3 behind the segment's
  // K2 with no host wait; MergeCollect copies the selection back on the copy
  // stream (the main stream meanwhile runs the next segment's K2). One launch
  // may be outstanding; AppendRecords for it must precede the next MergeLaunch.
  void MergeLaunch(DevQuery *q, DevDb *d, uint32_t g0, uint32_t g1, uint64_t cand_begin, uint64_t n, uint32_t best,
                   uint32_t tb_base, int open, int ext, const MergePass &pass);
  void MergeCollect(std::vector<uint32_t> *counts, HostHits *hits);
  // Carried result lists of a query chunk (all groups empty), and their copy to
  // the host (counts[g], hits[g * cap + k]).
  void ResetCarry(DevQuery *q, uint32_t cap);
  void CarryToHost(DevQuery *q, uint32_t g0, uint32_t g1, uint32_t cap, std::vector<uint32_t> *counts,
                   HostHits *hits);
  // a block of n SelectedHit slots (contents undefined)
  void AcquireHostHits(size_t n, HostHits *out);
  // Global index of each DB chunk's first subject (hit records' db_id).
  void SetChunkBases(const uint32_t *bases, uint32_t n);

  // Device-resident hit records of the current run (GhostmHit layout, 32 B),
  // for the multi-GPU gather. AppendRecords turns the last MergeSelect's hits
  // (groups [g0, g0 + counts.size())) into records at the end of the array.
  // expect: the run's record bound (its groups x -b), reserved up front so
  // the array does not grow (reallocate and free) while the run's kernels are
  // queued; at most kRecordReserveMax bytes, beyond that it grows on demand
  void ResetRecords(uint64_t expect = 0);
  void AppendRecords(DevQuery *q, uint32_t g0, const std::vector<uint32_t> &counts, uint32_t cap,
                     uint32_t q_base, bool from_carry = false);  // from_carry: groups' carried lists
  void UploadRecords(const void *records, uint64_t n);  // host records (other paths)
  uint64_t RecordCount() const { return records_; }
  void CopyRecords(void *dst_device, uint64_t n);         // device-to-device, synchronous

  // K3 on n hits (query id, absolute db end).
  void TraceBack(DevQuery *q, DevDb *d, uint32_t n, const uint32_t *qid, const uint32_t *db_end,
                 uint32_t base_search_length, int open, int ext, uint32_t *db_start,
                 uint32_t *aln_len, uint32_t *aln_match, float *seq_id);

  DeviceTimes &times() {
    SettleSeedTime();
    return times_;
  }
  void SettleSeedTime();
  void ResetTimes() { times_ = DeviceTimes(); }
  void Synchronize();

 private:
  DeviceModule() = default;
  // span: runs of slots whose hits may pair (a name group's slots)
  void LaunchTraceback(kern::TbArgs a, DevQuery *q, uint32_t n, const DevDb *d, uint32_t span);
  int device_ = -1;
  void *stream_ = nullptr;
  HostCopyFn host_copy_;
  HostParallelFn host_par_;
  bool defer_next_ = false;
  void *copy_stream_ = nullptr;  // D2H of selections and K2 task uploads, beside the kernels
  DeviceTimes times_;
  uint64_t records_ = 0;
  Impl *impl_ = nullptr;
  friend struct DeviceModuleAccess;
};

const char *DeviceBuildInfo();

}  // namespace ghostm
