// device.hip — gfx950 device module: buffers, launches, and the reference C ABI
// (include/ghostm_hip.h Part 1 + the device-level extensions of Part 2).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ghostm_hip.h"
#include "common.h"
#include "device.h"
#include "formats.h"
#include "kernels.h"
#include "score_tasks.h"

namespace ghostm {

#define HIP_CHECK(expr)                                                                  \
  do {                                                                                   \
    hipError_t err_ = (expr);                                                            \
    if (err_ != hipSuccess)                                                              \
      throw Error(std::string("HIP error '") + hipGetErrorString(err_) + "' at " #expr); \
  } while (0)

namespace {

// Page-locked host staging (hipHostMalloc), grown on demand, never shrunk.
struct PinnedBuf {
  void *p = nullptr;
  size_t bytes = 0;
  void Reserve(size_t b) {
    if (b <= bytes) return;
    if (p) HIP_CHECK(hipHostFree(p));
    p = nullptr;
    bytes = 0;
    if (TraceOn()) TraceMark("pin_alloc", b);
    HIP_CHECK(hipHostMalloc(&p, std::max<size_t>(b, 256), hipHostMallocDefault));
    bytes = std::max<size_t>(b, 256);
  }
  template <class T> T *as() const { return static_cast<T *>(p); }
};

// Device blocks released by a buffer stay cached for the next one (a session's
// query/DB/index buffers are released at its end and the next session's create
// asks for the same sizes: hipMalloc/hipFree cost ~1.5 ms of a cfg3 create,
// profiles/r5f/cfg3_e2e_trace.log). A block is cached after a device
// synchronisation, as hipFree would do; a request takes the smallest cached block
// of 1-2x its size. At most GHOSTM_DEV_POOL_MB (default 8192) stay cached; 0
// turns the cache off. The cache never costs an allocation: a hipMalloc that
// runs out of memory empties it and tries once more (DevBuf::Reserve), and a
// caller sharing the device (torch, RCCL) can empty it (GhostmDevicePoolTrim).
class DevPool {
 public:
  static DevPool &Get() {
    static DevPool pool;
    return pool;
  }
  void *Take(size_t *bytes) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lock(mu_);
    size_t best = blocks_.size();
    for (size_t k = 0; k < blocks_.size(); ++k)
      if (blocks_[k].dev == dev && blocks_[k].bytes >= *bytes && blocks_[k].bytes <= 2 * *bytes &&
          (best == blocks_.size() || blocks_[k].bytes < blocks_[best].bytes))
        best = k;
    if (best == blocks_.size()) return nullptr;
    void *p = blocks_[best].p;
    *bytes = blocks_[best].bytes;
    cached_ -= *bytes;
    blocks_.erase(blocks_.begin() + (long)best);
    return p;
  }
  void Give(void *p, size_t bytes) {
    if (!p) return;
    (void)hipDeviceSynchronize();  // no queued work may still use the block
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lock(mu_);
    if (cached_ + bytes > cap_) {
      (void)hipFree(p);
      return;
    }
    blocks_.push_back(Block{p, bytes, dev});
    cached_ += bytes;
  }
  // frees every cached block; returns the bytes freed
  size_t Trim() {
    std::lock_guard<std::mutex> lock(mu_);
    size_t freed = 0;
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (const Block &b : blocks_) {
      (void)hipSetDevice(b.dev);
      (void)hipFree(b.p);
      freed += b.bytes;
    }
    (void)hipSetDevice(cur);
    blocks_.clear();
    cached_ = 0;
    return freed;
  }
  // hipMalloc through the cache's out-of-memory rule: on failure, empty the cache
  // and try once more. GHOSTM_DEV_OOM_TEST=1 (tests) makes the first attempt fail
  // whenever blocks are cached, so the retry path runs on any data set.
  hipError_t Malloc(void **p, size_t bytes) {
    const char *t = getenv("GHOSTM_DEV_OOM_TEST");
    hipError_t err = (t && *t == '1' && Cached()) ? hipErrorOutOfMemory : hipMalloc(p, bytes);
    if (err == hipErrorOutOfMemory && Cached()) {
      (void)hipGetLastError();  // clear the failed call's error state
      Trim();
      ++oom_retries_;
      err = hipMalloc(p, bytes);
    }
    if (err != hipSuccess) *p = nullptr;
    return err;
  }
  size_t Cached() {
    std::lock_guard<std::mutex> lock(mu_);
    return cached_;
  }
  uint64_t OomRetries() const { return oom_retries_.load(); }

 private:
  DevPool() {
    const char *e = getenv("GHOSTM_DEV_POOL_MB");
    cap_ = (size_t)(e ? strtoull(e, nullptr, 10) : 8192ull) << 20;
  }
  struct Block {
    void *p;
    size_t bytes;
    int dev;
  };
  std::mutex mu_;
  std::vector<Block> blocks_;
  size_t cached_ = 0, cap_ = 0;
  std::atomic<uint64_t> oom_retries_{0};
};

struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  void Reserve(size_t b) {
    if (b <= bytes) return;
    Release();
    size_t want = std::max<size_t>(b, 256);
    if ((p = DevPool::Get().Take(&want))) {
      if (TraceOn()) TraceMark("dev_reuse", want);
    } else {
      if (TraceOn()) TraceMark("dev_alloc", want);
      HIP_CHECK(DevPool::Get().Malloc(&p, want));
    }
    bytes = want;
  }
  void Release() {
    if (p && TraceOn()) TraceMark("dev_free", bytes);
    DevPool::Get().Give(p, bytes);
    p = nullptr;
    bytes = 0;
  }
  template <class T> T *as() const { return static_cast<T *>(p); }
};

// Rows per lane (S) and lanes per candidate (G) for a query width L: the layout
// with the fewest lane-steps per useful cell among S in {8, 16, 32}.
struct Layout {
  int S;
  uint32_t G, Lpad, gpw;
};

Layout ChooseLayout(uint32_t L, uint32_t width) {
  Layout best{32, 1, 32, 64};
  double best_cost = 1e300;
  for (int S : {32, 16, 8}) {
    const uint32_t G = (L + S - 1) / S;
    if (G == 0 || G > 16) continue;
    const uint32_t gpw = 64 / G;
    const double cost = (double)(G * S) * (double)(width + G - 1) / (double)(gpw * G);
    if (cost < best_cost * 0.999) {
      best_cost = cost;
      best = Layout{S, G, G * (uint32_t)S, gpw};
    }
  }
  return best;
}

thread_local std::string g_last_error;


}  // namespace

struct DevQuery {
  DevBuf seq;
  DevBuf rcodes;                   // K3a row code offsets (kern::k_rev_codes) for rcodes_lpad
  uint32_t rcodes_lpad = 0;
  DevBuf fcodes;                   // k_score_pair's forward row code offsets (kern::k_fwd_codes)
  uint32_t fcodes_lpad = 0;
  uint32_t nseq = 0, L = 0;
  DevBuf group_first, group_last;  // name groups (device merge)
  uint32_t ngroups = 0;
};

// DB residues live at seq + kDbFront, with END bytes in front of and behind
// them, so K2 can load window residues unconditionally (the window test picks
// END for columns outside it).
constexpr uint32_t kDbFront = kern::kDbFrontPad, kDbBack = 65536;

struct DevDb {
  DevBuf seq, kc, pos;
  DevBuf low;                      // kern::k_low_keys' bitmap
  uint32_t len = 0, kcl = 0, npos = 0;
  bool codes_le26 = false;         // every residue code <= 26 (the sparse K2 profiles hold rows 0..26)
  uint32_t end_gap = UINT32_MAX;   // fewest positions from one END to the next (K2 restart levels)
  const uint8_t *Residues() const { return seq.as<uint8_t>() + kDbFront; }
  DevBuf subj;                     // subject starts (device merge)
  DevBuf subj_bucket;              // kern::SubjectOfBucketed's table
  uint32_t nsubj = 0;
};

struct DeviceModule::Impl {
  int h_matrix[32 * 32] = {0};
  // StagedUpload: a ring of page-locked slots and the event of each slot's last copy
  static constexpr int kStageSlots = 4;
  static constexpr size_t kStagePiece = 8u << 20;
  PinnedBuf stage[kStageSlots];
  hipEvent_t stage_ev[kStageSlots] = {};
  bool stage_busy[kStageSlots] = {};
  int stage_turn = 0;
  DevBuf mat_k2, mat_tb, mat_tbk;  // mat_tbk: two 32x32 key tables (MLW 16, 17)
  DevBuf mat_raw;                  // the matrix itself (K3a pair table)
  // K1 work
  DevBuf counts, nelem, slots, offsets, qlist, gbuf, gbuf_off, list_beg, list_len;
  DevBuf cand_start, cand_qid;
  DevBuf records, rec_prefix;    // hit records of the run (HitRecord32)
  std::vector<uint32_t> h_rec_prefix;
  uint64_t ncand = 0;
  // K2 work: two task buffers (a launch reads one while the next segment's
  // tasks are uploaded into the other), the guard re-score's tasks
  DevBuf task_buf[2], tasks_redo, score_out, end_out, guard_list;
  int task_turn = 0;
  struct Prepared {
    bool valid = false;
    uint64_t cand_begin = 0, n = 0;
    uint32_t count = 0, per_block = 0;
    bool swar = false;  // the encoding they were built for
    int kind = kScoreRows;  // the kernel they chose (score_tasks.h ScoreKind)
    int buf = 0;
  } prepared;
  struct ScoreState {                       // the launched, not yet finished K2
    bool active = false, guarded = false;
    uint64_t cand_begin = 0, n = 0;
    size_t lds = 0;
    int S = 32;
    kern::ScoreArgs args{};
  } score_state;
  struct DeferredNext {  // ScoreLaunch's next segment, built by ScorePrepareNext
    bool valid = false;
    DeviceModule::ScoreSegment seg{};
    bool swar = false, pairs_ok = true;
    uint32_t per_block = 0;
    size_t bytes = 0;
    uint32_t sparse_per_block = 0;
  } deferred;
  // K3 work (tb_sort: two histograms + total, two cursor arrays)
  DevBuf tb_qid, tb_end, tb_start, tb_ml;
  DevBuf tb_width, tb_ncols, tb_skey, tb_key, tb_order1, tb_order2, tb_sort, tb_pair_a, tb_pair_b, tb_best;
  int cus = 256;
  // K4 work
  DevBuf keys, sel_count, sel_score, sel_sid, slot_hits, sel_from;
  struct MergeState {  // the launched, not yet collected K4/K3
    bool active = false;
    uint32_t ng = 0;
    size_t slots = 0;
  } merge_state;
  // result lists carried across batches / DB chunks (per group of the query
  // chunk: carry_count[g] SlotHits at carry_hits[g * cap]); DB chunk bases
  DevBuf carry_hits, carry_count, chunk_base;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;          // K2 launch (and the synchronous paths)
  hipEvent_t ev_s0 = nullptr, ev_s1 = nullptr;      // K1: read once the stream has passed them
  hipEvent_t ev_nb = nullptr;                       // K1a's bin counts on the host
  int seed_early = 1;                               // K1b class launched before the host class pass
  bool seed_pending = false;
  PinnedBuf h_tasks[2];                             // K2 task staging, one per task buffer
  std::vector<uint32_t> h_wide;                     // K1 wide-pass query list and group offsets: kept
  std::vector<unsigned long long> h_wide_goff;      // until the next K1, past their async uploads
  hipEvent_t ev_m0 = nullptr, ev_m1 = nullptr;      // K4
  hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr;      // K3
  hipEvent_t ev_tk = nullptr;                       // K3: the scan phase's end (key DP start)
  bool tk_recorded = false;                         // ... recorded by the last LaunchTraceback
  hipEvent_t ev_done = nullptr, ev_tasks = nullptr; // end of a segment's selection; next tasks uploaded
  // K1 read-backs (per-query bin and candidate counts) land in page-locked
  // staging: GHOSTM_K1_PINNED=0 keeps the pageable copies (A/B)
  PinnedBuf h_nbins, h_counts, h_qlist, h_offsets;
  DevBuf offset_parts;                              // K1 device offsets: per-block sums, then prefixes
  DevBuf counters;     // K2: u64 [0] score cells, u32 at [2] guard count
  DevBuf tb_counters;  // K3: u64 [0] traceback cells, [1] K3a scan cells, [2] hits traced (k_finalize)
  bool matrix_set = false;
};

static constexpr uint32_t kSlotCap = kern::kMaxSlotCap;
// Filtered slot pass (k_seed_filter) of classes 0, 1 and 2, thresholds >= 2:
// <BLOCK, filter cells, table slots, queue, alias> and its dynamic LDS bytes.
// The bitmap shares its LDS with the exact table (alias), which doubled the
// cells each class can afford at the same occupancy: half the aliased cells,
// so about half the lone entries that passed the filter only by aliasing are
// no longer queued and counted (class 1, cfg4: 13.7 -> 11.4 ms per launch,
// profiles/r4_k1/). GHOSTM_K1_ALIAS=0 builds the separate regions with the
// earlier cell counts (A/B).
#ifndef GHOSTM_K1_ALIAS
#define GHOSTM_K1_ALIAS 1
#endif
#ifndef GHOSTM_K1_STAGE2  // A/B: a second, hashed bitmap over the queue (kernels.h STAGE2)
#define GHOSTM_K1_STAGE2 0
#endif
constexpr bool kFilterAlias = GHOSTM_K1_ALIAS != 0;
constexpr bool kFilterStage2 = kFilterAlias && GHOSTM_K1_STAGE2 != 0;
constexpr uint32_t kFilterScale = kFilterAlias ? 2 : 1;
#define GHOSTM_FILTER0 kern::k_seed_filter<256, 32768 * kFilterScale, 2304, 1536, kFilterAlias, kFilterStage2>
#define GHOSTM_FILTER1 kern::k_seed_filter<512, 65536 * kFilterScale, 4608, 3072, kFilterAlias, kFilterStage2>
#define GHOSTM_FILTER2 kern::k_seed_filter<1024, 131072 * kFilterScale, 9216, 6144, kFilterAlias, kFilterStage2>
constexpr size_t FilterLds(size_t cells, size_t table, size_t queue) {
  const size_t words = kern::FilterWords((uint32_t)cells);
  const size_t region = (kFilterAlias ? std::max(words, table) : words + table) + queue;
  return kern::FilterStaticLds((uint32_t)region) ? 0 : region * 4;  // dynamic LDS bytes
}
constexpr size_t kFilterLds0 = FilterLds(32768 * kFilterScale, 2304, 1536);
constexpr size_t kFilterLds1 = FilterLds(65536 * kFilterScale, 4608, 3072);
constexpr size_t kFilterLds2 = FilterLds(131072 * kFilterScale, 9216, 6144);

// K3a: the pair table (32 x 32 codes x 32 query codes, one word each) + histogram
static constexpr size_t kScanLds = (size_t)kern::kPairWords * 4 + kern::kSortBins * 4;
static constexpr size_t kScanLdsPriv = (size_t)kern::kPrivWords * 4 + kern::kSortBins * 4;  // GHOSTM_K3_SCAN=priv

// Host landing of a segment's selected hits (HostHits): a fresh, uninitialised
// heap block per segment, freed by the formatter when it is done with it.
// Measured alternatives (cfg4, GHOSTM_TRACE timelines): a zero-filled
// std::vector per segment costs ~3 ms of host time per 16 M-candidate segment;
// reusing blocks from a pool (pageable or hipHostMalloc'd) made the next K1
// launch wait 10-27 ms for the device on most chunks (426 -> 467-475 ms/step).
void DeviceModule::AcquireHostHits(size_t n, HostHits *out) {
  SelectedHit *p = new SelectedHit[std::max<size_t>(n, 1)];
  out->block = std::shared_ptr<void>(p, [](void *v) { delete[] static_cast<SelectedHit *>(v); });
  out->data = p;
  out->n = n;
}

DeviceModule &DeviceModule::Get() {
  static DeviceModule *m = new DeviceModule();
  return *m;
}

// HIP's current device is per host thread: every entry that allocates or
// launches makes this module's device current on the calling thread first.
void DeviceModule::Use() const {
  thread_local int current = -1;  // this thread's device as last set here
  if (device_ >= 0 && current != device_) {
    HIP_CHECK(hipSetDevice(device_));
    current = device_;
  }
}

void DeviceModule::Bind(int device) {
  if (device_ == device && impl_) {
    Use();
    return;
  }
  // one device per process: buffers, stream and events belong to the first one
  if (impl_ && device_ >= 0)
    throw Error("the device module is bound to device " + std::to_string(device_) + "; one device per process");
  int n = 0;
  HIP_CHECK(hipGetDeviceCount(&n));
  if (n <= 0) throw Error("no HIP device visible");
  if (device < 0 || device >= n) throw Error("device id " + std::to_string(device) + " out of range");
  HIP_CHECK(hipSetDevice(device));
  if (!impl_) impl_ = new Impl();
  hipStream_t s, c;
  HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  HIP_CHECK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
  stream_ = s;
  copy_stream_ = c;
#ifdef GHOSTM_LDS_POISON
  {  // the pattern every kernel writes over its LDS before its own code runs
    uint32_t v = 0xA5A5A5A5u;
    if (const char *e = getenv("GHOSTM_LDS_POISON_PATTERN")) v = (uint32_t)strtoul(e, nullptr, 0);
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(kern::g_lds_poison), &v, sizeof(v)));
  }
#endif
  for (hipEvent_t *e : {&impl_->ev0, &impl_->ev1, &impl_->ev_m0, &impl_->ev_m1, &impl_->ev_t0, &impl_->ev_t1, &impl_->ev_tk,
                        &impl_->ev_done, &impl_->ev_tasks, &impl_->ev_s0, &impl_->ev_s1, &impl_->ev_nb})
    HIP_CHECK(hipEventCreate(e));
  for (hipEvent_t &e : impl_->stage_ev) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_CHECK(hipFuncSetAttribute((const void *)kern::k_seed<1024, 16384, false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 16384 * 4));
  HIP_CHECK(hipFuncSetAttribute((const void *)kern::k_seed<512, 8192, false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 8192 * 4));
  HIP_CHECK(hipFuncSetAttribute((const void *)kern::k_seed<256, 4096, false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 4096 * 4));
  HIP_CHECK(hipFuncSetAttribute((const void *)kern::k_seed_hash<256, 8192>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 8192 * 4));
  HIP_CHECK(hipFuncSetAttribute((const void *)kern::k_seed_hash<512, 12288>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 12288 * 4));
  HIP_CHECK(hipFuncSetAttribute((const void *)kern::k_seed_hash<1024, 24576>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 24576 * 4));
  HIP_CHECK(hipFuncSetAttribute((const void *)GHOSTM_FILTER0, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)kFilterLds0));
  HIP_CHECK(hipFuncSetAttribute((const void *)GHOSTM_FILTER1, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)kFilterLds1));
  HIP_CHECK(hipFuncSetAttribute((const void *)GHOSTM_FILTER2, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)kFilterLds2));
  // the sparse rows K2 (kScoreRowsSparse): seven 27-row profiles, ~53 KB at L = 127
  for (const void *f : {(const void *)kern::k_score16f<16, true>, (const void *)kern::k_score16f<16, true, false, true>})
    HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(kern::kScoreQmaxSparse * kern::kProfRowsSparse * ((kMaxQueryLength + 15) / 16 * 16 + 8) * 2 +
                                        32 * 32 * 2)));
  const int scan_lds = (int)kScanLds;
#define GHOSTM_SCAN_ATTR(SS, HH, EE, FF)                                             \
  HIP_CHECK(hipFuncSetAttribute((const void *)kern::k_tb_scan<SS, HH, EE, FF>,       \
                                hipFuncAttributeMaxDynamicSharedMemorySize, scan_lds));
#define GHOSTM_SCAN_ATTR2(SS, HH) GHOSTM_SCAN_ATTR(SS, HH, true, false) GHOSTM_SCAN_ATTR(SS, HH, false, false)
  GHOSTM_SCAN_ATTR2(32, true) GHOSTM_SCAN_ATTR2(32, false) GHOSTM_SCAN_ATTR2(16, true)
  GHOSTM_SCAN_ATTR2(16, false) GHOSTM_SCAN_ATTR2(8, true) GHOSTM_SCAN_ATTR2(8, false)
  GHOSTM_SCAN_ATTR(32, true, true, true) GHOSTM_SCAN_ATTR(32, true, false, true)
  GHOSTM_SCAN_ATTR(16, true, true, true) GHOSTM_SCAN_ATTR(16, true, false, true)
  GHOSTM_SCAN_ATTR(8, true, true, true) GHOSTM_SCAN_ATTR(8, true, false, true)
#define GHOSTM_SCAN_ATTRW(SS, EE)                                                      \
  HIP_CHECK(hipFuncSetAttribute((const void *)kern::k_tb_scan<SS, true, EE, true, true>, \
                                hipFuncAttributeMaxDynamicSharedMemorySize, scan_lds));
  GHOSTM_SCAN_ATTRW(32, true) GHOSTM_SCAN_ATTRW(32, false) GHOSTM_SCAN_ATTRW(16, true)
  GHOSTM_SCAN_ATTRW(16, false) GHOSTM_SCAN_ATTRW(8, true) GHOSTM_SCAN_ATTRW(8, false)
#undef GHOSTM_SCAN_ATTRW
#define GHOSTM_SCAN_ATTRP(SS, EE)                                                            \
  HIP_CHECK(hipFuncSetAttribute((const void *)kern::k_tb_scan<SS, true, EE, true, true, true>, \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kScanLdsPriv));
  GHOSTM_SCAN_ATTRP(32, true) GHOSTM_SCAN_ATTRP(32, false) GHOSTM_SCAN_ATTRP(16, true)
  GHOSTM_SCAN_ATTRP(16, false) GHOSTM_SCAN_ATTRP(8, true) GHOSTM_SCAN_ATTRP(8, false)
#undef GHOSTM_SCAN_ATTRP
  for (const void *f : {(const void *)kern::k_score_pair<32>, (const void *)kern::k_score_pair<16>,
                        (const void *)kern::k_score_pair<8>})
    HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kern::kPairK2Words * 4)));
#undef GHOSTM_SCAN_ATTR2
#undef GHOSTM_SCAN_ATTR
  {
    hipDeviceProp_t p;
    HIP_CHECK(hipGetDeviceProperties(&p, device));
    impl_->cus = p.multiProcessorCount > 0 ? p.multiProcessorCount : 256;
  }
  device_ = device;
}

static hipStream_t S(void *s) { return static_cast<hipStream_t>(s); }

std::string DeviceModule::DeviceName() const {
  hipDeviceProp_t p;
  HIP_CHECK(hipGetDeviceProperties(&p, device_ < 0 ? 0 : device_));
  return std::string(p.name) + " (" + p.gcnArchName + ")";
}

size_t DeviceModule::TotalMemory() const {
  hipDeviceProp_t p;
  HIP_CHECK(hipGetDeviceProperties(&p, device_ < 0 ? 0 : device_));
  return p.totalGlobalMem;
}

void DeviceModule::SetMatrix(const int *m) {
  Use();
  if (!impl_) throw Error("device not bound");
  std::memcpy(impl_->h_matrix, m, sizeof(impl_->h_matrix));
  int k2[32 * 32], tb[32 * 32];
  for (int c = 0; c < 32; ++c) {
    for (int q = 0; q < 32; ++q) {
      const int v = m[c * 32 + q];
      k2[c * 32 + q] = q == (int)kern::kPadCode ? kern::kNeg : v;
      const int inc = 0x100 | (c == q ? 1 : 0);
      tb[c * 32 + q] = q == (int)kern::kPadCode ? (int)((unsigned)kern::kNeg << 16)
                                                : (int)(((unsigned)v << 16) | (unsigned)inc);
    }
  }
  // K3 key tables (k_traceback_key): (score << (MLW+2)) | (2 << MLW) | (0x80 | eq)
  // for MLW = 16 and 17; padding rows score far below any reachable h
  // h field: 14 bits signed (MLW 16) or 13 (MLW 17); the padding score is the
  // field minimum, below -hmax for every launch LaunchTraceback allows
  int tbk[2][32 * 32];
  for (int w = 0; w < 2; ++w) {
    const int mlw = 16 + w, lim = w ? 4095 : 8191;
    for (int c = 0; c < 32; ++c) {
      for (int q = 0; q < 32; ++q) {
        const int v = q == (int)kern::kPadCode ? -lim - 1 : std::max(-lim, std::min(lim, m[c * 32 + q]));
        tbk[w][c * 32 + q] =
            (int)(((uint32_t)v << (mlw + 2)) | (2u << mlw) | 0x80u | (c == q ? 1u : 0u));
      }
    }
  }
  impl_->mat_raw.Reserve(sizeof(impl_->h_matrix));
  HIP_CHECK(hipMemcpy(impl_->mat_raw.p, impl_->h_matrix, sizeof(impl_->h_matrix), hipMemcpyHostToDevice));
  impl_->mat_k2.Reserve(sizeof(k2));
  impl_->mat_tb.Reserve(sizeof(tb));
  impl_->mat_tbk.Reserve(sizeof(tbk));
  HIP_CHECK(hipMemcpy(impl_->mat_k2.p, k2, sizeof(k2), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(impl_->mat_tb.p, tb, sizeof(tb), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(impl_->mat_tbk.p, tbk, sizeof(tbk), hipMemcpyHostToDevice));
  impl_->matrix_set = true;
}

void DeviceModule::SetHostCopy(HostCopyFn fn) { host_copy_ = std::move(fn); }
void DeviceModule::SetHostParallel(HostParallelFn fn) { host_par_ = std::move(fn); }

// Host bytes to the device through page-locked staging: pieces of kStagePiece
// bytes, each copied into a ring slot by the host copy function (the session's
// parallel workers) and sent by hipMemcpyAsync on the main stream; a slot is
// reused once its last copy has landed. A pageable hipMemcpy (HIP's own
// staging, one host thread) moved the chunk files at ~15 GB/s (cfg 4: 181 MB in
// 12 ms of session create). Returns after the last host copy (the source may be
// released); the device copies complete in stream order.
void DeviceModule::StagedUpload(void *dst, const void *src, size_t bytes) {
  Impl &I = *impl_;
  if (bytes < (1u << 20) || !host_copy_) {  // small: one pageable copy
    if (bytes) HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, S(stream_)));
    if (bytes) HIP_CHECK(hipStreamSynchronize(S(stream_)));
    return;
  }
  for (size_t off = 0; off < bytes; off += Impl::kStagePiece) {
    const size_t n = std::min(Impl::kStagePiece, bytes - off);
    const int k = I.stage_turn;
    I.stage_turn = (k + 1) % Impl::kStageSlots;
    if (I.stage_busy[k]) HIP_CHECK(hipEventSynchronize(I.stage_ev[k]));
    I.stage[k].Reserve(Impl::kStagePiece);
    host_copy_(I.stage[k].p, static_cast<const char *>(src) + off, n);
    HIP_CHECK(hipMemcpyAsync(static_cast<char *>(dst) + off, I.stage[k].p, n, hipMemcpyHostToDevice, S(stream_)));
    HIP_CHECK(hipEventRecord(I.stage_ev[k], S(stream_)));
    I.stage_busy[k] = true;
  }
}

DevQuery *DeviceModule::UploadQuery(const uint8_t *seq, uint32_t nseq, uint32_t L) {
  Use();
  if (!impl_) throw Error("device not bound");
  if (L == 0 || L > kMaxQueryLength)
    throw Error("query record width " + std::to_string(L) + " outside 1..127");
  DevQuery *q = new DevQuery();
  q->nseq = nseq;
  q->L = L;
  const size_t b = (size_t)nseq * L;
  q->seq.Reserve(b + 16);
  StagedUpload(q->seq.p, seq, b);
  return q;
}

DevDb *DeviceModule::UploadDb(const uint8_t *seq, uint32_t len, const uint32_t *kc, uint32_t kcl,
                              const uint32_t *pos, uint32_t npos) {
  Use();
  if (!impl_) throw Error("device not bound");
  // the kernels index 32-entry tables by residue code (checked 8 bytes at a time)
  uint64_t over26 = 0;  // a byte >= 27 sets its top bit in (byte + 101) (codes < 32 do not carry)
  {
    uint64_t hi = 0;
    uint32_t k = 0;
    for (; k + 8 <= len; k += 8) {
      uint64_t w;
      std::memcpy(&w, seq + k, 8);
      hi |= w;
      over26 |= (w & 0x1F1F1F1F1F1F1F1Full) + 0x6565656565656565ull;
    }
    for (; k < len; ++k) {
      hi |= seq[k];
      over26 |= (uint64_t)((seq[k] & 0x1Fu) + 0x65u);
    }
    if (hi & 0xE0E0E0E0E0E0E0E0ull) throw Error("database residue code out of range");
  }
  // the closest two ENDs (subject boundaries): bounds the ENDs a K2 window can
  // meet, which the restart-level kernel needs below the f16 infinity pattern
  uint32_t end_gap = UINT32_MAX;
  for (const uint8_t *p = seq, *last = nullptr, *e = seq + len;
       (p = static_cast<const uint8_t *>(std::memchr(p, (int)kern::kSeqEnd, (size_t)(e - p)))) != nullptr; ++p) {
    if (last) end_gap = std::min<uint32_t>(end_gap, (uint32_t)(p - last));
    last = p;
  }
  DevDb *d = new DevDb();
  d->end_gap = end_gap;
  d->codes_le26 = (over26 & 0x8080808080808080ull) == 0;
  d->len = len;
  d->kcl = kcl;
  d->npos = npos;
  d->seq.Reserve((size_t)kDbFront + len + kDbBack);
  d->kc.Reserve((size_t)kcl * 4);
  d->pos.Reserve(((size_t)npos + kern::kPosTailPad) * 4);
  HIP_CHECK(hipMemsetAsync(d->seq.p, (int)kern::kSeqEnd, (size_t)kDbFront + len + kDbBack, S(stream_)));
  StagedUpload(static_cast<uint8_t *>(d->seq.p) + kDbFront, seq, len);
  StagedUpload(d->kc.p, kc, (size_t)kcl * 4);
  StagedUpload(d->pos.p, pos, (size_t)npos * 4);
  HIP_CHECK(hipMemsetAsync(static_cast<uint32_t *>(d->pos.p) + npos, 0, (size_t)kern::kPosTailPad * 4, S(stream_)));
  const uint32_t nkeys = kcl ? kcl - 1 : 0;
  d->low.Reserve(((size_t)nkeys + 63) / 64 * 8 + 8);
  if (nkeys) {
    hipLaunchKernelGGL(kern::k_low_keys, dim3((nkeys + 255) / 256), dim3(256), 0, S(stream_), d->kc.as<uint32_t>(),
                       d->pos.as<uint32_t>(), nkeys, d->low.as<unsigned long long>());
    HIP_CHECK(hipGetLastError());
  }
  return d;
}

void DeviceModule::Free(DevQuery *q) {
  if (device_ >= 0) (void)hipSetDevice(device_);  // destructors: never throw
  if (!q) return;
  q->seq.Release();
  q->rcodes.Release();
  q->fcodes.Release();
  q->group_first.Release();
  q->group_last.Release();
  delete q;
}

void DeviceModule::Free(DevDb *d) {
  if (device_ >= 0) (void)hipSetDevice(device_);  // destructors: never throw
  if (!d) return;
  d->seq.Release();
  d->kc.Release();
  d->pos.Release();
  d->low.Release();
  d->subj.Release();
  d->subj_bucket.Release();
  delete d;
}

void DeviceModule::SetQueryGroups(DevQuery *q, const uint32_t *first, const uint32_t *last,
                                  uint32_t ng) {
  Use();
  q->ngroups = ng;
  q->group_first.Reserve((size_t)ng * 4);
  q->group_last.Reserve((size_t)ng * 4);
  if (ng) {
    HIP_CHECK(hipMemcpy(q->group_first.p, first, (size_t)ng * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(q->group_last.p, last, (size_t)ng * 4, hipMemcpyHostToDevice));
  }
}

void DeviceModule::SetDbSubjects(DevDb *d, const uint32_t *starts, uint32_t nsubj) {
  Use();
  d->nsubj = nsubj;
  d->subj.Reserve((size_t)nsubj * 4);
  if (nsubj) HIP_CHECK(hipMemcpy(d->subj.p, starts, (size_t)nsubj * 4, hipMemcpyHostToDevice));
  // bucket[k] = the last subject starting at or before k << shift (kNoSlot: none),
  // for k = 0 .. (len >> shift) + 1
  if (nsubj) {
    const uint32_t nb = (d->len >> kern::kSubjBucketShift) + 2;
    std::vector<uint32_t> bucket(nb);
    uint32_t s = 0;
    for (uint32_t k = 0; k < nb; ++k) {
      const uint64_t at = (uint64_t)k << kern::kSubjBucketShift;
      while (s + 1 < nsubj && starts[s + 1] <= at) ++s;
      bucket[k] = starts[s] <= at ? s : kern::kNoSlot;
    }
    d->subj_bucket.Reserve((size_t)nb * 4);
    HIP_CHECK(hipMemcpy(d->subj_bucket.p, bucket.data(), (size_t)nb * 4, hipMemcpyHostToDevice));
  }
}

void DeviceModule::Synchronize() {
  if (stream_) HIP_CHECK(hipStreamSynchronize(S(stream_)));
  if (copy_stream_) HIP_CHECK(hipStreamSynchronize(S(copy_stream_)));
}

static float ElapsedMs(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  HIP_CHECK(hipEventSynchronize(b));
  HIP_CHECK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

// K1's device time, read when something has waited for the stream anyway (the
// K1 stage itself returns without waiting for its last kernels)
void DeviceModule::SettleSeedTime() {
  if (!impl_ || !impl_->seed_pending) return;
  impl_->seed_pending = false;
  times_.seed += ElapsedMs(impl_->ev_s0, impl_->ev_s1) * 1e-3;
}

// K1 size classes: (threads, LDS bins per buffer). Bigger queries get bigger
// workgroups; the last class merges in global memory.
struct SeedClass {
  uint32_t block, cap;
};
static const SeedClass kSeedClasses[] = {{256, 4096}, {512, 8192}, {1024, 16384}, {1024, 0}};

// Test knobs (read per Seed call): GHOSTM_K1_CAPS="c0,c1,c2" lowers the three
// LDS class caps (never raises them: every kernel keeps its LDS sizing), so
// small datasets reach every class and the global-merge class 3;
// GHOSTM_K1_SLOT_CAP lowers the per-query slot, sending more queries through
// the offset pass that rewrites wide queries in place.
static void SeedCaps(uint32_t caps[3], uint32_t *slot_cap) {
  for (int k = 0; k < 3; ++k) caps[k] = kSeedClasses[k].cap;
  if (const char *e = getenv("GHOSTM_K1_CAPS")) {
    const char *p = e;
    for (int k = 0; k < 3 && *p; ++k) {
      char *end = nullptr;
      const unsigned long v = strtoul(p, &end, 10);
      if (end == p) break;
      caps[k] = std::min<uint32_t>(caps[k], (uint32_t)v);
      p = *end == ',' ? end + 1 : end;
    }
    for (int k = 1; k < 3; ++k) caps[k] = std::max(caps[k], caps[k - 1]);
  }
  *slot_cap = kSlotCap;
  if (const char *e = getenv("GHOSTM_K1_SLOT_CAP")) {
    const unsigned long v = strtoul(e, nullptr, 10);
    if (v >= 1) *slot_cap = std::min<uint32_t>(kSlotCap, (uint32_t)v);
  }
}

template <uint32_t B, uint32_t C, bool G>
static void LaunchSeed(const kern::SeedArgs &a, uint32_t items, hipStream_t s) {
  const size_t lds = G ? 0 : (size_t)2 * C * 4;
  hipLaunchKernelGGL((kern::k_seed<B, C, G>), dim3(items), dim3(B), lds, s, a);
}

static void LaunchSeedFilterClass(int cls, const kern::SeedArgs &a, uint32_t items, hipStream_t s) {
  if (items == 0) return;
  if (cls == 0) hipLaunchKernelGGL((GHOSTM_FILTER0), dim3(items), dim3(256), kFilterLds0, s, a);
  else if (cls == 1) hipLaunchKernelGGL((GHOSTM_FILTER1), dim3(items), dim3(512), kFilterLds1, s, a);
  else hipLaunchKernelGGL((GHOSTM_FILTER2), dim3(items), dim3(1024), kFilterLds2, s, a);
  HIP_CHECK(hipGetLastError());
}

// Slot pass of the three LDS classes: the hash-count kernel (table >= 1.5 x cap).
static void LaunchSeedHashClass(int cls, const kern::SeedArgs &a, uint32_t items, hipStream_t s) {
  if (items == 0) return;
  switch (cls) {
    case 0:
      hipLaunchKernelGGL((kern::k_seed_hash<256, 8192>), dim3(items), dim3(256), 8192 * 4, s, a);
      break;
    case 1:  // load <= 2/3: 48 KB, three workgroups per CU
      hipLaunchKernelGGL((kern::k_seed_hash<512, 12288>), dim3(items), dim3(512), 12288 * 4, s, a);
      break;
    default:
      hipLaunchKernelGGL((kern::k_seed_hash<1024, 24576>), dim3(items), dim3(1024), 24576 * 4, s, a);
      break;
  }
  HIP_CHECK(hipGetLastError());
}

static void LaunchSeedClass(int cls, const kern::SeedArgs &a, uint32_t items, hipStream_t s) {
  if (items == 0) return;
  switch (cls) {
    case 0: LaunchSeed<256, 4096, false>(a, items, s); break;
    case 1: LaunchSeed<512, 8192, false>(a, items, s); break;
    case 2: LaunchSeed<1024, 16384, false>(a, items, s); break;
    default: LaunchSeed<1024, 1, true>(a, items, s); break;
  }
  HIP_CHECK(hipGetLastError());
}

uint64_t DeviceModule::Seed(DevQuery *q, DevDb *d, const SeedConfig &cfg,
                            std::vector<uint32_t> *counts, std::vector<uint64_t> *offsets) {
  Use();
  Impl &I = *impl_;
  const uint32_t nq = q->nseq;
  // every element is written below (counts by the count pass or the read-back,
  // offsets by the offset pass): a reused vector is not cleared first
  counts->resize(nq);
  offsets->resize(nq);
  I.ncand = 0;
  const uint32_t seed_len = SeedLength(cfg.seed_mask);
  if (nq == 0 || seed_len == 0 || seed_len > q->L) {
    std::fill(counts->begin(), counts->end(), 0u);
    std::fill(offsets->begin(), offsets->end(), 0ull);
    return 0;
  }
  if (cfg.shift == 0) throw Error("shift size must be positive");
  const uint32_t nlists = (q->L - seed_len) / cfg.shift + 1;
  if (nlists > kern::kMaxLists) throw Error("too many seed lists");
  if (d->kcl == 0) throw Error("database index missing");

  uint32_t caps[3], slot_cap;
  SeedCaps(caps, &slot_cap);
  I.counts.Reserve((size_t)nq * 4);
  I.nelem.Reserve((size_t)nq * 4);
  I.slots.Reserve((size_t)nq * slot_cap * 4);
  I.offsets.Reserve((size_t)nq * 8);
  I.list_beg.Reserve((size_t)nq * nlists * 4);
  I.list_len.Reserve((size_t)nq * nlists * 4);
  SettleSeedTime();
  if (TraceOn()) {  // timeline only: is the stream idle before K1 starts?
    HIP_CHECK(hipEventRecord(I.ev_nb, S(stream_)));
    HIP_CHECK(hipEventSynchronize(I.ev_nb));
    TraceMark("k1_idle");
  }
  HIP_CHECK(hipEventRecord(I.ev_s0, S(stream_)));
  HIP_CHECK(hipMemsetAsync(I.counts.p, 0, (size_t)nq * 4, S(stream_)));
  TraceMark("k1a_memset");

  // K1a: list segments + bin count per query
  kern::SeedListArgs la{};
  la.qseq = q->seq.as<uint8_t>();
  la.L = q->L;
  la.nq = nq;
  la.keys_count = d->kc.as<uint32_t>();
  la.positions = d->pos.as<uint32_t>();
  la.low_keys = d->low.as<unsigned long long>();
  la.seed_mask = cfg.seed_mask;
  la.nlists = nlists;
  la.shift = cfg.shift;
  la.list_beg = I.list_beg.as<uint32_t>();
  la.list_len = I.list_len.as<uint32_t>();
  la.nbins = I.nelem.as<uint32_t>();
  hipLaunchKernelGGL(kern::k_seed_lists, dim3((nq + 3) / 4), dim3(256), 0, S(stream_), la);
  HIP_CHECK(hipGetLastError());
  TraceMark("k1a_launch");
  const char *pin_env = getenv("GHOSTM_K1_PINNED");
  const bool pinned = !(pin_env && strcmp(pin_env, "0") == 0);
  std::vector<uint32_t> nbins_v;
  const uint32_t *nbins = nullptr;
  if (pinned) {
    I.h_nbins.Reserve((size_t)nq * 4);
    HIP_CHECK(hipMemcpyAsync(I.h_nbins.p, I.nelem.p, (size_t)nq * 4, hipMemcpyDeviceToHost, S(stream_)));
    nbins = I.h_nbins.as<uint32_t>();
  } else {
    nbins_v.resize(nq);
    HIP_CHECK(hipMemcpyAsync(nbins_v.data(), I.nelem.p, (size_t)nq * 4, hipMemcpyDeviceToHost, S(stream_)));
    nbins = nbins_v.data();
  }
  HIP_CHECK(hipEventRecord(I.ev_nb, S(stream_)));
  // K1b path: the LDS classes count bins in a hash table when every bin + 2 <
  // 2^21; classes 0, 1 and 2 put the presence filter in front of it when T >= 2
  // (GHOSTM_K1=merge keeps the merge kernel, =hash the unfiltered table)
  const char *k1 = getenv("GHOSTM_K1");
  const bool hash = !(k1 && strcmp(k1, "merge") == 0) && d->len > 0 &&
                    ((uint64_t)(d->len - 1) >> cfg.log_region) + 2 < kern::kHashBinLimit;
  const bool filter = hash && cfg.threshold >= 2 && !(k1 && strcmp(k1, "hash") == 0);
  kern::SeedArgs a{};
  a.positions = d->pos.as<uint32_t>();
  a.nlists = nlists;
  a.shift = cfg.shift;
  a.log_region = cfg.log_region;
  a.threshold = cfg.threshold;
  a.list_beg = I.list_beg.as<uint32_t>();
  a.list_len = I.list_len.as<uint32_t>();
  a.counts = I.counts.as<uint32_t>();
  a.slots = I.slots.as<uint32_t>();
  a.slot_cap = slot_cap;
  a.probe_windows = 0xFFFFFFFFu;  // BinTable's own bound
  if (const char *e = getenv("GHOSTM_K1_PROBE_WINDOWS")) a.probe_windows = (uint32_t)strtoul(e, nullptr, 10);
  // the class that held most queries last time is launched now, over every
  // query (its blocks pick their queries from the device bin counts), so the
  // GPU works through it while the host sorts the rest into class lists
  const int n_lds = hash ? 3 : 0;  // classes with an identity launch
  const char *early_env = getenv("GHOSTM_K1_EARLY");
  int early = early_env && strcmp(early_env, "0") == 0 ? -1 : std::min(I.seed_early, n_lds - 1);
  if (early >= 0) {
    kern::SeedArgs b = a;
    b.query_list = nullptr;
    b.nbins = I.nelem.as<uint32_t>();
    b.nb_lo = early == 0 ? 0u : caps[early - 1];
    b.nb_hi = caps[early];
    if (filter) LaunchSeedFilterClass(early, b, nq, S(stream_));
    else LaunchSeedHashClass(early, b, nq, S(stream_));
  }
  TraceMark("k1a_enq");
  HIP_CHECK(hipEventSynchronize(I.ev_nb));
  TraceMark("k1a_done");

  // size classes (queries without any position keep count 0): one counting
  // pass, then the lists written by class straight into page-locked staging
  // (cls[c] views it) and uploaded asynchronously
  uint32_t ncls[4] = {0, 0, 0, 0};
  uint64_t bins_total = 0;
  auto class_of = [&](uint32_t n) { return n <= caps[0] ? 0 : n <= caps[1] ? 1 : n <= caps[2] ? 2 : 3; };
  for (uint32_t i = 0; i < nq; ++i) {
    const uint32_t n = nbins[i];
    bins_total += n;
    if (n) ++ncls[class_of(n)];
  }
  const size_t list_total = (size_t)ncls[0] + ncls[1] + ncls[2] + ncls[3];
  for (int c = 0; c < n_lds; ++c)
    if (ncls[c] > ncls[I.seed_early < n_lds ? I.seed_early : 0]) I.seed_early = c;
  I.h_qlist.Reserve(list_total * 4 + 4);
  uint32_t *hl = I.h_qlist.as<uint32_t>();
  struct Span {
    const uint32_t *p;
    size_t n;
    const uint32_t *begin() const { return p; }
    const uint32_t *end() const { return p + n; }
    size_t size() const { return n; }
  } cls[4];
  {
    uint32_t at[4];
    size_t o = 0;
    for (int c = 0; c < 4; ++c) {
      cls[c] = Span{hl + o, ncls[c]};
      at[c] = (uint32_t)o;
      o += ncls[c];
    }
    for (uint32_t i = 0; i < nq; ++i)
      if (nbins[i]) hl[at[class_of(nbins[i])]++] = i;
  }
  std::vector<unsigned long long> goff;  // class 3: global merge buffer offsets
  unsigned long long gtotal = 0;
  for (uint32_t qi : cls[3]) {
    goff.push_back(gtotal);
    gtotal += 2ull * nbins[qi];
  }
  I.qlist.Reserve(list_total * 4 + 4);
  if (list_total)
    HIP_CHECK(hipMemcpyAsync(I.qlist.p, hl, list_total * 4, hipMemcpyHostToDevice, S(stream_)));
  if (gtotal) {
    I.gbuf.Reserve(gtotal * 4);
    I.gbuf_off.Reserve(goff.size() * 8);
    HIP_CHECK(hipMemcpyAsync(I.gbuf_off.p, goff.data(), goff.size() * 8, hipMemcpyHostToDevice, S(stream_)));
  }

  a.gbuf = I.gbuf.as<uint32_t>();
  a.gbuf_off = I.gbuf_off.as<unsigned long long>();
  // K1b pass 1: every other class, candidates into per-query slots (largest first)
  {
    size_t at = list_total;
    for (int c = 3; c >= 0; --c) {
      at -= cls[c].size();
      if (c == early) continue;
      kern::SeedArgs b = a;
      b.query_list = I.qlist.as<uint32_t>() + at;
      if (filter && c < 3) LaunchSeedFilterClass(c, b, (uint32_t)cls[c].size(), S(stream_));
      else if (hash && c < 3) LaunchSeedHashClass(c, b, (uint32_t)cls[c].size(), S(stream_));
      else LaunchSeedClass(c, b, (uint32_t)cls[c].size(), S(stream_));
    }
  }
  times_.seed_launches_hash += hash ? 1 : 0;
  times_.seed_launches_filter += filter ? 1 : 0;
  if (const char *e = getenv("GHOSTM_K1_FORCE_OVERFLOW"); e && filter && atoi(e) > 0)
    hipLaunchKernelGGL(kern::k_force_overflow, dim3((nq + 255) / 256), dim3(256), 0, S(stream_),
                       I.counts.as<uint32_t>(), I.nelem.as<uint32_t>(), nq, (uint32_t)atoi(e), caps[2]);
  if (pinned) {
    I.h_counts.Reserve((size_t)nq * 4);
    HIP_CHECK(hipMemcpyAsync(I.h_counts.p, I.counts.p, (size_t)nq * 4, hipMemcpyDeviceToHost, S(stream_)));
  } else {
    HIP_CHECK(hipMemcpyAsync(counts->data(), I.counts.p, (size_t)nq * 4, hipMemcpyDeviceToHost, S(stream_)));
  }
  HIP_CHECK(hipEventRecord(I.ev_nb, S(stream_)));
  // the offsets and the compaction on the device behind the count read-back,
  // while the host reads the counts (it re-runs the copy only after a queue
  // overflow or when the candidate buffers had to grow; GHOSTM_K1_DEVOFF=0 keeps
  // the host offsets, A/B)
  const char *devoff_env = getenv("GHOSTM_K1_DEVOFF");
  const bool dev_off = !(devoff_env && strcmp(devoff_env, "0") == 0);
  // (GHOSTM_K1_CAND_CAP, tests: the device compaction sees at most that many
  // candidates of room, so its partial-write guard and the host's re-run run)
  uint64_t cand_cap = std::min(I.cand_start.bytes, I.cand_qid.bytes) / 4;
  if (const char *e = getenv("GHOSTM_K1_CAND_CAP")) cand_cap = std::min<uint64_t>(cand_cap, strtoull(e, nullptr, 10));
  auto launch_compact = [&](uint64_t cap) {
    hipLaunchKernelGGL(kern::k_compact, dim3((nq + 3) / 4), dim3(256), 0, S(stream_),
                       I.slots.as<uint32_t>(), slot_cap, I.counts.as<uint32_t>(), (const uint8_t *)nullptr,
                       I.offsets.as<unsigned long long>(), nq, I.cand_start.as<uint32_t>(),
                       I.cand_qid.as<uint32_t>(), (unsigned long long)cap);
    HIP_CHECK(hipGetLastError());
  };
  if (dev_off) {
    const uint32_t nparts = (nq + kern::kOffsetBlock - 1) / kern::kOffsetBlock;
    I.offset_parts.Reserve((size_t)nparts * 8 + 8);
    hipLaunchKernelGGL(kern::k_count_sums, dim3(nparts), dim3(256), 0, S(stream_), I.counts.as<uint32_t>(), nq,
                       I.offset_parts.as<unsigned long long>());
    hipLaunchKernelGGL(kern::k_count_scan, dim3(1), dim3(1024), 0, S(stream_),
                       I.offset_parts.as<unsigned long long>(), nparts, (unsigned long long *)nullptr);
    hipLaunchKernelGGL(kern::k_count_offsets, dim3(nparts), dim3(256), 0, S(stream_), I.counts.as<uint32_t>(), nq,
                       I.offset_parts.as<unsigned long long>(), I.offsets.as<unsigned long long>());
    HIP_CHECK(hipGetLastError());
    if (cand_cap) launch_compact(cand_cap);
  }
  TraceMark("k1b_enq");
  HIP_CHECK(hipEventSynchronize(I.ev_nb));
  TraceMark("k1b_done");
  // counts into the host vector, offsets into it and into page-locked staging
  // (uploaded by DMA), in parts on the worker threads: the GPU waits for this
  // pass (cfg4: 505 K queries per chunk)
  I.h_offsets.Reserve((size_t)nq * 8);
  unsigned long long *h_off = I.h_offsets.as<unsigned long long>();
  const size_t parts = nq >= 65536 && host_par_ ? 16 : 1;
  auto part_lo = [&](size_t k) { return (uint32_t)((uint64_t)nq * k / parts); };
  auto for_parts = [&](const std::function<void(size_t)> &fn) {
    if (parts > 1) host_par_(parts, fn);
    else fn(0);
  };
  std::vector<uint64_t> part_sum(parts + 1, 0);
  std::vector<uint8_t> part_over(parts, 0);
  std::vector<std::vector<uint32_t>> part_wide(parts);
  auto count_pass = [&](const uint32_t *src) {
    for_parts([&](size_t k) {
      uint64_t s = 0;
      bool over = false;
      uint32_t *dst = counts->data();
      for (uint32_t i = part_lo(k); i < part_lo(k + 1); ++i) {
        const uint32_t c = src[i];
        if (src != dst) dst[i] = c;
        s += c;
        over |= c == kern::kOverflow;
      }
      part_sum[k + 1] = s;
      part_over[k] = over;
    });
  };
  count_pass(pinned ? I.h_counts.as<uint32_t>() : counts->data());
  bool overflow = false;
  for (uint8_t o : part_over) overflow |= o != 0;
  if (hash && overflow) {
    // queries a class-0..2 kernel marked kOverflow: a filtered queue that
    // overflowed (or a filter table that found no free slot) is redone by the
    // unfiltered table (k_seed_hash); a table that found no free slot within its
    // probe bound (BinTable) is redone by the LDS merge kernel (k_seed), which
    // has no table. Each stage reads the counts back before the next.
    for (int stage = filter ? 0 : 1; stage < 2; ++stage) {
      std::vector<uint32_t> redo[3];
      for (int c = 0; c < 3; ++c)
        for (uint32_t qi : cls[c])
          if ((*counts)[qi] == kern::kOverflow) redo[c].push_back(qi);
      std::vector<uint32_t> all(redo[0]);
      all.insert(all.end(), redo[1].begin(), redo[1].end());
      all.insert(all.end(), redo[2].begin(), redo[2].end());
      if (all.empty()) break;
      I.qlist.Reserve(all.size() * 4);
      HIP_CHECK(hipMemcpyAsync(I.qlist.p, all.data(), all.size() * 4, hipMemcpyHostToDevice, S(stream_)));
      size_t at = 0;
      for (int c = 0; c < 3; ++c) {
        kern::SeedArgs b = a;
        b.query_list = I.qlist.as<uint32_t>() + at;
        if (stage == 0) LaunchSeedHashClass(c, b, (uint32_t)redo[c].size(), S(stream_));
        else LaunchSeedClass(c, b, (uint32_t)redo[c].size(), S(stream_));
        at += redo[c].size();
      }
      HIP_CHECK(hipMemcpyAsync(counts->data(), I.counts.p, (size_t)nq * 4, hipMemcpyDeviceToHost, S(stream_)));
      HIP_CHECK(hipStreamSynchronize(S(stream_)));
      (stage == 0 ? times_.seed_filter_overflows : times_.seed_table_full) += all.size();
      count_pass(counts->data());
    }
  }
  for (size_t k = 0; k < parts; ++k) part_sum[k + 1] += part_sum[k];
  const uint64_t total = part_sum[parts];
  for_parts([&](size_t k) {
    uint64_t o = part_sum[k];
    const uint32_t *cnt = counts->data();
    uint64_t *off = offsets->data();
    for (uint32_t i = part_lo(k); i < part_lo(k + 1); ++i) {
      off[i] = o;
      h_off[i] = o;
      if (cnt[i] > slot_cap) part_wide[k].push_back(i);
      o += cnt[i];
    }
  });
  // queries with more candidates than a slot, by size class in query order
  std::vector<uint32_t> wide[4];
  std::vector<unsigned long long> &wide_goff = I.h_wide_goff;  // outlive the async copies below
  wide_goff.clear();
  for (const std::vector<uint32_t> &pw : part_wide)
    for (uint32_t qi : pw) {
      const int c = class_of(nbins[qi]);
      wide[c].push_back(qi);
      if (c == 3) wide_goff.push_back(goff[(size_t)(std::lower_bound(cls[3].begin(), cls[3].end(), qi) - cls[3].begin())]);
    }
  I.ncand = total;
  // the device copy stands when its offsets were the final ones (no overflow)
  // and it had room for every candidate
  const bool redo_copy = !dev_off || overflow || total + 1 > cand_cap;
  I.cand_start.Reserve(total * 4 + 4);
  I.cand_qid.Reserve(total * 4 + 4);
  if (redo_copy) {
    if (!dev_off || overflow)
      HIP_CHECK(hipMemcpyAsync(I.offsets.p, h_off, (size_t)nq * 8, hipMemcpyHostToDevice, S(stream_)));
    launch_compact(total + 1);  // slot -> compact
  }
  times_.seed_compact_redo += dev_off && redo_copy ? 1 : 0;
  // pass 2: queries with more candidates than a slot, written straight into place
  size_t nwide = 0;
  for (auto &v : wide) nwide += v.size();
  for (int c = 0; c < 4; ++c) times_.seed_queries_class[c] += cls[c].size();
  times_.seed_queries_wide += nwide;
  std::vector<uint32_t> &all = I.h_wide;
  all.clear();
  if (nwide) {
    all.reserve(nwide);
    for (auto &v : wide) all.insert(all.end(), v.begin(), v.end());
    I.qlist.Reserve(all.size() * 4);
    HIP_CHECK(hipMemcpyAsync(I.qlist.p, all.data(), all.size() * 4, hipMemcpyHostToDevice, S(stream_)));
    if (!wide_goff.empty())
      HIP_CHECK(hipMemcpyAsync(I.gbuf_off.p, wide_goff.data(), wide_goff.size() * 8, hipMemcpyHostToDevice,
                               S(stream_)));
    size_t at = 0;
    for (int c = 0; c < 4; ++c) {
      kern::SeedArgs b = a;
      b.query_list = I.qlist.as<uint32_t>() + at;
      b.slots = nullptr;
      b.offsets = I.offsets.as<unsigned long long>();
      b.out_start = I.cand_start.as<uint32_t>();
      b.out_qid = I.cand_qid.as<uint32_t>();
      LaunchSeedClass(c, b, (uint32_t)wide[c].size(), S(stream_));
      at += wide[c].size();
    }
  }
  HIP_CHECK(hipEventRecord(I.ev_s1, S(stream_)));
  I.seed_pending = true;  // the compaction and wide pass run on while the host cuts batches
  TraceMark("k1c_enq");
  // algorithmic bytes: query record + 2 CSR words per list + one u32 per
  // position + 8 bytes (start, query) per candidate
  times_.seed_bytes += (uint64_t)nq * (q->L + 8ull * nlists) + bins_total * 4ull + total * 8ull;
  times_.seed_list_entries += bins_total;
  return total;
}

void DeviceModule::CopyStarts(uint64_t begin, uint64_t n, uint32_t *out) {
  Use();
  if (n == 0) return;
  // the K1 stage returns with its last kernels still queued on stream_
  HIP_CHECK(hipMemcpyAsync(out, impl_->cand_start.as<uint32_t>() + begin, n * 4, hipMemcpyDeviceToHost,
                           S(stream_)));
  HIP_CHECK(hipStreamSynchronize(S(stream_)));
  SettleSeedTime();
}


// the packed K2 encodings (two candidates per lane) whenever every value fits
static bool ScorePacked(const int *h_matrix, uint32_t L, uint32_t base, const GapConfig &gap) {
  int max_abs = 0;
  for (int k = 0; k < 32 * 32; ++k) max_abs = std::max(max_abs, h_matrix[k] < 0 ? -h_matrix[k] : h_matrix[k]);
  const char *force = getenv("GHOSTM_K2");
  const bool gaps_ok = gap.open <= 0 && gap.ext <= 0 && -gap.open < 2000 && -gap.ext < 2000;
  const int64_t bound = (int64_t)L * max_abs;
  const bool allow_packed = !(force && strcmp(force, "int32") == 0);
  return allow_packed && gaps_ok && bound < 30000 && base + 64 < kDbBack;
}

uint32_t DeviceModule::ScorePerBlock(DevQuery *q, uint32_t base, const GapConfig &gap) const {
  const Layout lay = ChooseLayout(q->L, base);
  return (kern::kScoreBlock / 64) * lay.gpw * (ScorePacked(impl_->h_matrix, q->L, base, gap) ? 2 : 1);
}

// The sparse rows kernel's layout (16 rows per lane) and its candidates per
// block; per_block 0 when it cannot run (a DB code above 26, or more than 16
// lanes per candidate)
static Layout SparseLayout(uint32_t L) {
  const uint32_t G = (L + 15) / 16;
  return Layout{16, G, G * 16, G ? 64 / G : 64};
}
static uint32_t SparsePerBlock(const DevQuery *q, const DevDb *d) {
  const Layout s = SparseLayout(q->L);
  if (!d->codes_le26 || s.G == 0 || s.G > 16) return 0;
  return (kern::kScoreBlock / 64) * s.gpw * 2;
}

// K2 in two steps for the device-merge pipeline: ScoreLaunch enqueues the
// launch (no host wait) and prepares the next segment's tasks; ScoreFinish
// waits for it, reads its counters on the copy stream (the main stream may
// already hold the segment's K4/K3) and re-scores the guard list.
void DeviceModule::ScoreLaunch(DevQuery *q, DevDb *d, uint64_t cand_begin, uint64_t n, uint32_t q_first,
                               uint32_t q_end, const std::vector<uint32_t> &counts,
                               const std::vector<uint64_t> &offsets, uint32_t base, const GapConfig &gap,
                               const ScoreSegment *next) {
  Use();
  Impl &I = *impl_;
  Impl::ScoreState &P = I.score_state;
  P = Impl::ScoreState();
  if (n == 0) return;
  if (gap.ext > 0) throw Error("positive gap extension score is not supported");
  const Layout lay = ChooseLayout(q->L, base);
  int max_abs = 0;
  for (int v : I.h_matrix) max_abs = std::max(max_abs, v < 0 ? -v : v);
  // encoding: f16 pairs when every score fits the exact-integer range of f16,
  // else int16 pairs, else int32 (GHOSTM_K2=int32|int16|f16 restricts the choice)
  const char *force = getenv("GHOSTM_K2");
  const int64_t bound = (int64_t)q->L * max_abs;
  const bool packed = ScorePacked(I.h_matrix, q->L, base, gap);
  // f16 is exact below 2048; beyond that it runs with a guard and the int16
  // kernel re-scores the (rare) candidates whose best reaches it
  const bool half = packed && !(force && strcmp(force, "int16") == 0);
  // the column-framed f16 kernel (k_score16f) holds values up to best + the
  // largest frame, (steps + 1) * ext_pen; GHOSTM_K2=f16plain keeps k_score16<S, true>
  // (the frame before a window's first END starts at -2040 + G * ext_pen)
  const int64_t sigma_max = (int64_t)(base + 2 * lay.G) * (-gap.ext);
  const bool framed = half && sigma_max <= 1000 && !(force && strcmp(force, "f16plain") == 0);
  // the framed kernel over 16-bit integer patterns (k_score16f<S, true>, the
  // default): exact with no guard while the largest pattern, the restart value
  // + the frame + L * max|M| (+ the open step), stays below f16 infinity;
  // GHOSTM_K2=f16frame keeps the f16-number frame
  const int64_t swar_low = 1024 + 64 + (-(int64_t)gap.open) + (-(int64_t)gap.ext);
  const int64_t swar_restart = swar_low + sigma_max + bound + 32;
  const int64_t swar_top = swar_restart + sigma_max + bound + std::abs((int64_t)gap.open - gap.ext) + 32;
  const bool swar = framed && swar_top < 0x7C00 && !(force && strcmp(force, "f16frame") == 0);
  // restart levels (k_score16f<S, true, false, true>): the k-th END of a window
  // restarts at swar_restart + (k - 1) * step, step above the largest rise after
  // a restart; the window's most ENDs (from the DB's closest two) must fit below
  // f16 infinity. GHOSTM_K2_LEVELS=0 keeps the second END's reset.
  const int64_t swar_rise = swar_top - swar_restart;
  const int64_t swar_step = swar_rise + 32;
  const uint64_t max_ends = d->end_gap == UINT32_MAX || base == 0 ? 1 : (uint64_t)(base - 1) / d->end_gap + 1;
  const int64_t swar_cap = swar_restart + (int64_t)(max_ends - 1) * swar_step;
  const char *levels_env = getenv("GHOSTM_K2_LEVELS");
  const bool levels = swar && !(levels_env && strcmp(levels_env, "0") == 0) && max_ends <= 64 && swar_cap + swar_rise < 0x7C00;
  // framed: values stay exact and the -2040-based frame stays below the
  // post-END one while best + sigma_max < 2040; beyond, the guard flags them
  int guard = swar ? 0 : framed ? (bound + sigma_max < 2040 ? 0 : (int)(2040 - sigma_max)) : (bound < 2048 ? 0 : 2000);
  if (half && getenv("GHOSTM_K2_GUARD")) guard = atoi(getenv("GHOSTM_K2_GUARD"));  // tests: force re-scores
  const uint32_t per_block = ScorePerBlock(q, base, gap);
  const uint32_t sparse_pb = swar ? SparsePerBlock(q, d) : 0u;
  // tasks, and with them the kernel (score_tasks.h BuildTasks: the unit-pair
  // kernel where its blocks are not too many more): prepared for this range by
  // the previous launch (uploaded on the copy stream into the other task
  // buffer), else built and uploaded here
  int kind = kScoreRows;
  int buf = -1;
  size_t ntasks = 0;
  // staging and task buffers hold ScoreTaskBound tasks, or n pair entries
  auto task_bytes = [&](uint64_t cn, uint32_t q0, uint32_t q1) {
    const uint32_t pb = sparse_pb ? std::min(per_block, sparse_pb) : per_block;
    return std::max<size_t>(ScoreTaskBound(cn, q0, q1, pb, kern::kScoreQmaxUnit) * sizeof(kern::ScoreTask),
                            (size_t)cn * 4);
  };
  if (I.prepared.valid && I.prepared.cand_begin == cand_begin && I.prepared.n == n &&
      I.prepared.per_block == per_block && I.prepared.swar == swar) {
    buf = I.prepared.buf;
    ntasks = I.prepared.count;
    kind = I.prepared.kind;
    HIP_CHECK(hipStreamWaitEvent(S(stream_), I.ev_tasks, 0));
  }
  const bool stale = I.prepared.valid;  // an upload nothing will use may still read its staging
  I.prepared.valid = false;
  if (buf < 0) {
    buf = I.task_turn;
    if (stale) HIP_CHECK(hipEventSynchronize(I.ev_tasks));
    // page-locked staging per task buffer: this one's last upload was read by
    // a launch that has been waited for, so the copy needs no wait either
    PinnedBuf &hs = I.h_tasks[buf];
    hs.Reserve(task_bytes(n, q_first, q_end));
    ntasks = BuildTasks(swar, cand_begin, n, q_first, q_end, counts, offsets, per_block, hs.as<kern::ScoreTask>(),
                        &kind, guard == 0, &host_par_, sparse_pb);
    TraceMark("tasks", ntasks);
    if (const char *dump = getenv("GHOSTM_DEBUG_TASKS")) {  // diagnostics: the launch's tasks and counts
      if (FILE *f = fopen(dump, "ab")) {
        const uint64_t hdr[6] = {cand_begin, n, q_first, q_end, (uint64_t)kind, (uint64_t)ntasks};
        fwrite(hdr, 8, 6, f);
        fwrite(hs.p, kind == kScorePairs ? 4 : sizeof(kern::ScoreTask), ntasks, f);
        fwrite(counts.data() + q_first, 4, q_end - q_first, f);
        fwrite(offsets.data() + q_first, 8, q_end - q_first, f);
        fclose(f);
      }
    }
    const size_t tb = ntasks * (kind == kScorePairs ? 4 : sizeof(kern::ScoreTask));
    I.task_buf[buf].Reserve(tb);
    HIP_CHECK(hipMemcpyAsync(I.task_buf[buf].p, hs.p, tb, hipMemcpyHostToDevice, S(stream_)));
    TraceMark("tasks_up", ntasks);
  }
  I.task_turn = 1 - buf;
  const bool unit = kind == kScoreUnit, pairs = kind == kScorePairs, sparse = kind == kScoreRowsSparse;
  const Layout slay = SparseLayout(q->L);
  if (pairs && q->fcodes_lpad != lay.Lpad) {  // the query chunk's forward row codes, once
    q->fcodes.Reserve((size_t)q->nseq * lay.Lpad + 16);
    const size_t words = (size_t)q->nseq * (lay.Lpad / 4);
    if (words)
      hipLaunchKernelGGL(kern::k_fwd_codes, dim3((uint32_t)((words + 255) / 256)), dim3(256), 0, S(stream_),
                         q->seq.as<uint8_t>(), q->nseq, q->L, lay.Lpad, q->fcodes.as<uint32_t>());
    q->fcodes_lpad = lay.Lpad;
  }
  I.score_out.Reserve(n * 4);
  I.end_out.Reserve(n * 4);
  kern::ScoreArgs a{};
  a.qseq = q->seq.as<uint8_t>();
  a.L = q->L;
  a.Lpad = lay.Lpad;
  a.pad = lay.Lpad - q->L;
  a.G = lay.G;
  a.gpw = lay.gpw;
  a.db = d->Residues();
  a.dblen = d->len;
  a.mat = I.mat_k2.as<int>();
  a.cand_qid = I.cand_qid.as<uint32_t>();
  a.cand_start = I.cand_start.as<uint32_t>();
  a.tasks = I.task_buf[buf].as<kern::ScoreTask>();
  a.base = base;
  a.extend = gap.extend;
  a.open = gap.open;
  a.ext = gap.ext;
  a.score_out = I.score_out.as<uint32_t>();
  a.end_out = I.end_out.as<uint32_t>();
  a.out_base = cand_begin;
  a.swar_low = (uint32_t)swar_low;
  a.swar_restart = (uint32_t)swar_restart;
  a.swar_step = levels ? (uint32_t)swar_step : 0u;
  a.swar_cap = levels ? (uint32_t)swar_cap : 0u;
  if (pairs) {
    a.pairs = I.task_buf[buf].as<uint32_t>();
    a.npairs = (uint32_t)ntasks;
    a.fcodes = q->fcodes.as<uint32_t>();
  }
  if (sparse) {  // 16 rows per lane, kScoreQmaxSparse profiles of kProfRowsSparse code rows
    a.Lpad = slay.Lpad;
    a.pad = slay.Lpad - q->L;
    a.G = slay.G;
    a.gpw = slay.gpw;
    a.prof_slots = kern::SparseSlots();
    a.prof_rows = kern::kProfRowsSparse;
  }
  // counters: [0] cells (u64), [2] guard count (u32)
  I.counters.Reserve(32);
  HIP_CHECK(hipMemsetAsync(I.counters.p, 0, 32, S(stream_)));
  a.cells = I.counters.as<unsigned long long>();
  if (half && guard) {
    I.guard_list.Reserve((size_t)n * 8);
    a.guard = guard;
    a.guard_count = reinterpret_cast<uint32_t *>(I.counters.as<unsigned long long>() + 2);
    a.guard_list = I.guard_list.as<uint32_t>();
  }
  // packed: the profiles, then the 32 x 32 code table they are built from
  // (UNIT: 32-bit words, rows padded by 4 words, a 32 x 32 word code table)
  const size_t lds = unit     ? (size_t)kern::kScoreQmaxUnit * kern::kProfRows16 * (lay.Lpad + 4) * 4 + 32 * 32 * 4
                     : sparse ? (size_t)kern::SparseSlots() * kern::kProfRowsSparse * (slay.Lpad + 8) * 2 + 32 * 32 * 2
                     : packed ? (size_t)kern::kScoreQmax * kern::kProfRows16 * (lay.Lpad + 8) * 2 + 32 * 32 * 2
                              : (size_t)kern::kScoreQmax * kern::kProfRows * (lay.Lpad + 4) * 4;
  HIP_CHECK(hipEventRecord(I.ev0, S(stream_)));
  const dim3 grid((uint32_t)ntasks), block(kern::kScoreBlock);
  if (pairs) {
    // persistent: one 768-thread workgroup per CU (the 96 KB pair table), looping
    // over the pairs. At most 16 rows per lane: with 32 (the profile kernels'
    // layout at L > 64) K2 took 3.57 against 3.40 ms per cfg2 step, same box
    // (profiles/r5k/); GHOSTM_K2_PAIR_S=8|16|32 forces the rows per lane (A/B).
    // The kernel is bound by the table's LDS bank conflicts: two workgroups per CU
    // (a 78.7 KB table) or 1024-thread workgroups measured slower (profiles/r5i, r5j).
    uint32_t ps = std::min<uint32_t>((uint32_t)lay.S, 16);
    if (const char *e = getenv("GHOSTM_K2_PAIR_S")) ps = (uint32_t)atoi(e);
    const uint32_t pg = ps == 8 || ps == 16 || ps == 32 ? lay.Lpad / ps : 0;
    const Layout play = pg >= 1 && pg <= 16 && pg * ps == lay.Lpad ? Layout{(int)ps, pg, lay.Lpad, 64 / pg} : lay;
    a.G = play.G;
    a.gpw = play.gpw;
    const uint32_t per_wg = (kern::kPairBlock / 64) * play.gpw;
    const dim3 pgrid(std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)I.cus, (uint32_t)((ntasks + per_wg - 1) / per_wg))));
    const dim3 pblock(kern::kPairBlock);
    const size_t plds = (size_t)kern::kPairK2Words * 4;
    switch (play.S) {
      case 32: hipLaunchKernelGGL((kern::k_score_pair<32>), pgrid, pblock, plds, S(stream_), a); break;
      case 16: hipLaunchKernelGGL((kern::k_score_pair<16>), pgrid, pblock, plds, S(stream_), a); break;
      default: hipLaunchKernelGGL((kern::k_score_pair<8>), pgrid, pblock, plds, S(stream_), a); break;
    }
  } else if (sparse) {
    if (levels) hipLaunchKernelGGL((kern::k_score16f<16, true, false, true>), grid, block, lds, S(stream_), a);
    else hipLaunchKernelGGL((kern::k_score16f<16, true>), grid, block, lds, S(stream_), a);
  } else if (packed) {
    switch (lay.S) {
      case 32:
        if (unit) hipLaunchKernelGGL((kern::k_score16f<32, true, true>), grid, block, lds, S(stream_), a);
        else if (levels) hipLaunchKernelGGL((kern::k_score16f<32, true, false, true>), grid, block, lds, S(stream_), a);
        else if (swar) hipLaunchKernelGGL((kern::k_score16f<32, true>), grid, block, lds, S(stream_), a);
        else if (framed) hipLaunchKernelGGL((kern::k_score16f<32>), grid, block, lds, S(stream_), a);
        else if (half) hipLaunchKernelGGL((kern::k_score16<32, true>), grid, block, lds, S(stream_), a);
        else hipLaunchKernelGGL((kern::k_score16<32, false>), grid, block, lds, S(stream_), a);
        break;
      case 16:
        if (unit) hipLaunchKernelGGL((kern::k_score16f<16, true, true>), grid, block, lds, S(stream_), a);
        else if (levels) hipLaunchKernelGGL((kern::k_score16f<16, true, false, true>), grid, block, lds, S(stream_), a);
        else if (swar) hipLaunchKernelGGL((kern::k_score16f<16, true>), grid, block, lds, S(stream_), a);
        else if (framed) hipLaunchKernelGGL((kern::k_score16f<16>), grid, block, lds, S(stream_), a);
        else if (half) hipLaunchKernelGGL((kern::k_score16<16, true>), grid, block, lds, S(stream_), a);
        else hipLaunchKernelGGL((kern::k_score16<16, false>), grid, block, lds, S(stream_), a);
        break;
      default:
        if (unit) hipLaunchKernelGGL((kern::k_score16f<8, true, true>), grid, block, lds, S(stream_), a);
        else if (levels) hipLaunchKernelGGL((kern::k_score16f<8, true, false, true>), grid, block, lds, S(stream_), a);
        else if (swar) hipLaunchKernelGGL((kern::k_score16f<8, true>), grid, block, lds, S(stream_), a);
        else if (framed) hipLaunchKernelGGL((kern::k_score16f<8>), grid, block, lds, S(stream_), a);
        else if (half) hipLaunchKernelGGL((kern::k_score16<8, true>), grid, block, lds, S(stream_), a);
        else hipLaunchKernelGGL((kern::k_score16<8, false>), grid, block, lds, S(stream_), a);
        break;
    }
  } else {
    switch (lay.S) {
      case 32: hipLaunchKernelGGL(kern::k_score<32>, grid, block, lds, S(stream_), a); break;
      case 16: hipLaunchKernelGGL(kern::k_score<16>, grid, block, lds, S(stream_), a); break;
      default: hipLaunchKernelGGL(kern::k_score<8>, grid, block, lds, S(stream_), a); break;
    }
  }
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipEventRecord(I.ev1, S(stream_)));
  times_.score_launches += 1;
  times_.score_launches_packed += packed ? 1 : 0;
  times_.score_launches_half += half ? 1 : 0;
  times_.score_launches_framed += framed ? 1 : 0;
  times_.score_launches_swar += swar ? 1 : 0;
  times_.score_launches_unit += unit ? 1 : 0;
  times_.score_launches_pair += pairs ? 1 : 0;
  times_.score_launches_sparse += sparse ? 1 : 0;
  times_.score_launches_levels += levels && (sparse || (packed && !unit && !pairs)) ? 1 : 0;
  P.active = true;
  P.guarded = half && guard;
  P.cand_begin = cand_begin;
  P.n = n;
  P.lds = lds;
  P.S = lay.S;
  P.args = a;
  // the next segment's tasks, built on the host while K2 runs and uploaded on
  // the copy stream into the other buffer (its last reader, the previous K2,
  // has finished: ScoreFinish waited for it)
  // (the pipelined caller defers it, ScoreDeferNext, and builds it with
  // ScorePrepareNext after it has enqueued this segment's K4/K3, so the build
  // overlaps them too)
  I.deferred = Impl::DeferredNext{};
  if (next && next->n) {
    I.deferred = Impl::DeferredNext{true, *next, swar, guard == 0, per_block,
                                    task_bytes(next->n, next->q_first, next->q_end), sparse_pb};
    if (!defer_next_) ScorePrepareNext(counts, offsets);
  }
}

void DeviceModule::ScorePrepareNext(const std::vector<uint32_t> &counts, const std::vector<uint64_t> &offsets) {
  Impl &I = *impl_;
  if (!I.deferred.valid) return;
  const Impl::DeferredNext dn = I.deferred;
  I.deferred.valid = false;
  const ScoreSegment *next = &dn.seg;
  const int nb = I.task_turn;
  PinnedBuf &hs = I.h_tasks[nb];
  int nkind = kScoreRows;
  hs.Reserve(dn.bytes);
  const size_t nt = BuildTasks(dn.swar, next->cand_begin, next->n, next->q_first, next->q_end, counts, offsets,
                               dn.per_block, hs.as<kern::ScoreTask>(), &nkind, dn.pairs_ok, nullptr,
                               dn.sparse_per_block);
  const size_t nbytes = nt * (nkind == kScorePairs ? 4 : sizeof(kern::ScoreTask));
  I.task_buf[nb].Reserve(nbytes);
  HIP_CHECK(hipMemcpyAsync(I.task_buf[nb].p, hs.p, nbytes, hipMemcpyHostToDevice, S(copy_stream_)));
  HIP_CHECK(hipEventRecord(I.ev_tasks, S(copy_stream_)));
  I.prepared = Impl::Prepared{true, next->cand_begin, next->n, (uint32_t)nt, dn.per_block, dn.swar, nkind, nb};
}

bool DeviceModule::ScoreGuarded() const { return impl_ && impl_->score_state.active && impl_->score_state.guarded; }

void DeviceModule::ScoreFinish() {
  Use();
  Impl &I = *impl_;
  Impl::ScoreState &P = I.score_state;
  if (!P.active) return;
  P.active = false;
  SettleSeedTime();
  // the counters on the copy stream: the main stream may already hold K4/K3
  unsigned long long cells = 0;
  uint32_t nguard = 0;
  HIP_CHECK(hipStreamWaitEvent(S(copy_stream_), I.ev1, 0));
  HIP_CHECK(hipMemcpyAsync(&cells, I.counters.p, 8, hipMemcpyDeviceToHost, S(copy_stream_)));
  HIP_CHECK(hipMemcpyAsync(&nguard, I.counters.as<unsigned long long>() + 2, 4, hipMemcpyDeviceToHost,
                           S(copy_stream_)));
  HIP_CHECK(hipStreamSynchronize(S(copy_stream_)));
  times_.score += ElapsedMs(I.ev0, I.ev1) * 1e-3;
  times_.score_cells += cells;
  if (P.guarded && nguard) {
    // exact re-score of the guarded candidates with the int16 kernel, one
    // candidate per work item (nothing of this segment is queued behind K2:
    // the pipeline waits for ScoreFinish when the launch is guarded)
    std::vector<uint32_t> list((size_t)nguard * 2);
    HIP_CHECK(hipMemcpy(list.data(), I.guard_list.p, list.size() * 4, hipMemcpyDeviceToHost));
    std::vector<kern::ScoreTask> redo(nguard);
    for (uint32_t k = 0; k < nguard; ++k)
      redo[k] = kern::ScoreTask{P.cand_begin + list[2 * k], 1u, list[2 * k + 1], 1u, 1u,
                                P.cand_begin + list[2 * k] + 1, list[2 * k + 1] + 1, 0u};
    I.tasks_redo.Reserve(redo.size() * sizeof(kern::ScoreTask));
    HIP_CHECK(hipMemcpy(I.tasks_redo.p, redo.data(), redo.size() * sizeof(kern::ScoreTask), hipMemcpyHostToDevice));
    kern::ScoreArgs r = P.args;
    r.tasks = I.tasks_redo.as<kern::ScoreTask>();
    r.guard = 0;
    r.cells = I.counters.as<unsigned long long>() + 3;  // not counted twice
    const dim3 rgrid(nguard), block(kern::kScoreBlock);
    switch (P.S) {
      case 32: hipLaunchKernelGGL((kern::k_score16<32, false>), rgrid, block, P.lds, S(stream_), r); break;
      case 16: hipLaunchKernelGGL((kern::k_score16<16, false>), rgrid, block, P.lds, S(stream_), r); break;
      default: hipLaunchKernelGGL((kern::k_score16<8, false>), rgrid, block, P.lds, S(stream_), r); break;
    }
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(S(stream_)));
    times_.score_rechecks += nguard;
  }
}

void DeviceModule::Score(DevQuery *q, DevDb *d, uint64_t cand_begin, uint64_t n, uint32_t q_first,
                         uint32_t q_end, const std::vector<uint32_t> &counts,
                         const std::vector<uint64_t> &offsets, uint32_t base,
                         const GapConfig &gap, uint32_t *score, uint32_t *end, const ScoreSegment *next) {
  if (n == 0) return;
  ScoreLaunch(q, d, cand_begin, n, q_first, q_end, counts, offsets, base, gap, next);
  ScoreFinish();
  Impl &I = *impl_;
  if (score) HIP_CHECK(hipMemcpyAsync(score, I.score_out.p, n * 4, hipMemcpyDeviceToHost, S(stream_)));
  if (end) HIP_CHECK(hipMemcpyAsync(end, I.end_out.p, n * 4, hipMemcpyDeviceToHost, S(stream_)));
  if (score || end) HIP_CHECK(hipStreamSynchronize(S(stream_)));
}

// K3 launch: the key formulation when its field widths hold (len < 511,
// matches < 128, |h| < 8192), else the int32 kernel. GHOSTM_K3=int32 forces it.
void DeviceModule::LaunchTraceback(kern::TbArgs a, DevQuery *q, uint32_t n, const DevDb *d, uint32_t pair_span) {
  const uint32_t rows = q->L;
  Impl &I = *impl_;
  I.tk_recorded = false;
  const Layout lay = ChooseLayout(rows, a.base);
  a.Lpad = lay.Lpad;
  a.G = lay.G;
  a.gpw = lay.gpw;
  int max_abs = 0;
  for (int v : I.h_matrix) max_abs = std::max(max_abs, v < 0 ? -v : v);
  // path length <= rows + columns; ml = len << 7 | matches (matches <= L <= 127)
  const char *force = getenv("GHOSTM_K3");
  const bool allow = !(force && strcmp(force, "int32") == 0) && a.L <= 127 && a.open <= 0 && a.ext <= 0;
  const uint64_t span = (uint64_t)lay.Lpad + a.base;
  const int64_t hmax = (int64_t)a.L * max_abs;
  // h, E, F stay in [open + ext, hmax]; the field must hold that and the padding
  // rows' h + pad must stay negative
  const bool key16 = allow && span < 500 && hmax < 8000 && -a.open < 4000 && -a.ext < 4000;
  const bool key17 = !key16 && allow && span < 1000 && hmax < 4000 && -a.open < 2000 && -a.ext < 2000;
  const bool key = key16 || key17;
  if (key) a.mat_tb = I.mat_tbk.as<int>() + (key17 ? 32 * 32 : 0);
  a.order = nullptr;
  a.ncols = nullptr;
  a.best_h = nullptr;
  // Two-pass traceback (kernels.h K3a): a scores-only reverse scan finds each
  // hit's first maximal column j*, then the traceback DP runs columns 0..j*
  // only, hits sorted by that count. Needs the packed encodings' value range
  // (as K2): f16 below 2048, int16 below 30000. GHOSTM_K3_SCAN=0 turns it off,
  // =int16 forces the int16 scan.
  const char *scan_env = getenv("GHOSTM_K3_SCAN");
  const bool scan_off = scan_env && strcmp(scan_env, "0") == 0;
  const bool scan_gaps = a.open <= 0 && a.ext <= 0 && -a.open < 2000 && -a.ext < 2000;
  const bool scan = !scan_off && n > 0 && scan_gaps && hmax < 30000 && a.base < 65536;
  if (scan) {
    const bool half = hmax < 2048 && !(scan_env && strcmp(scan_env, "int16") == 0);
    // the column-framed f16 scan: values up to best + (window + 2G) * ext_pen
    // must stay exact (GHOSTM_K3_SCAN=f16plain keeps the unframed one)
    const int64_t scan_sigma = (int64_t)(a.base + 2 * lay.G) * (-a.ext);
    const bool framed = half && hmax + scan_sigma < 2048 && !(scan_env && strcmp(scan_env, "f16plain") == 0);
    // the framed scan over 16-bit integer patterns (the default): exact while
    // every value stays below the f16 infinity pattern; GHOSTM_K3_SCAN=f16frame
    // / f16plain / int16 keep the others
    const int64_t swar_low = 1024 + 64 + (-(int64_t)a.open) + (-(int64_t)a.ext);
    const bool swar = !(scan_env && (strcmp(scan_env, "f16frame") == 0 || strcmp(scan_env, "f16plain") == 0 ||
                                     strcmp(scan_env, "int16") == 0)) &&
                      swar_low + scan_sigma + hmax + std::abs((int64_t)a.open - a.ext) + 64 < 0x7C00;
    const uint32_t NB = kern::kSortBins;
    I.tb_width.Reserve((size_t)n * 4);
    I.tb_ncols.Reserve((size_t)n * 4);
    I.tb_key.Reserve((size_t)n * 4);
    I.tb_order1.Reserve((size_t)n * 4);
    I.tb_order2.Reserve((size_t)n * 4);
    I.tb_pair_a.Reserve((size_t)n * 4);
    I.tb_pair_b.Reserve((size_t)n * 4);
    I.tb_best.Reserve((size_t)n * 4);
    I.tb_skey.Reserve((size_t)n * 4);
    // two histograms + totals, two cursor arrays, the key DP's strip-class offsets
    constexpr uint32_t kClassWords = kern::kTbStripClasses + 1;
    I.tb_sort.Reserve((size_t)(4 * NB + 2 + kClassWords) * 4);
    uint32_t *hist1 = I.tb_sort.as<uint32_t>(), *hist2 = hist1 + NB + 1;
    uint32_t *cur1 = hist2 + NB + 1, *cur2 = cur1 + NB, *class_off = cur2 + NB;
    HIP_CHECK(hipMemsetAsync(I.tb_sort.p, 0, (size_t)(4 * NB + 2 + kClassWords) * 4, S(stream_)));
    // strip classes for the key DP when a group has at most kTbStripClasses
    // lanes (GHOSTM_K3_STRIPS=0 keeps every hit on all of them)
    const char *strips_env = getenv("GHOSTM_K3_STRIPS");
    const bool strips = lay.G <= kern::kTbStripClasses && !(strips_env && strcmp(strips_env, "0") == 0);
    const dim3 g256((n + 255) / 256), b256(256);
    const uint32_t *subj = d && d->nsubj ? d->subj.as<uint32_t>() : nullptr;
    hipLaunchKernelGGL(kern::k_tb_prep, g256, b256, 0, S(stream_), a.qid, a.end, n, a.base, subj,
                       subj ? d->nsubj : 0u, subj ? d->subj_bucket.as<uint32_t>() : nullptr, d ? d->len : 0u,
                       I.tb_width.as<uint32_t>(),
                       I.tb_ncols.as<uint32_t>(), I.tb_skey.as<uint32_t>(), hist2);  // empty slots -> hist2[0]
    const uint32_t ps = std::max<uint32_t>(pair_span, 1);
    const uint32_t runs_per_span = (ps + kern::kPairRun - 1) / kern::kPairRun;
    const uint64_t runs = (uint64_t)((n + ps - 1) / ps) * runs_per_span;
    // (diagnostics: GHOSTM_K3_SCAN_ORDER=query runs the scan's pairs in query
    // order, as a per-query-profile scan would have to, instead of by width)
    const char *order_env = getenv("GHOSTM_K3_SCAN_ORDER");
    const bool query_order = order_env && strcmp(order_env, "query") == 0;
    hipLaunchKernelGGL(kern::k_tb_pairs, dim3((uint32_t)((runs + 255) / 256)), b256, 0, S(stream_), a.qid,
                       I.tb_width.as<uint32_t>(), n, ps, I.tb_pair_a.as<uint32_t>(), I.tb_pair_b.as<uint32_t>(),
                       I.tb_key.as<uint32_t>(), hist1, query_order);
    const dim3 gsort((n + kern::kCsortTile - 1) / kern::kCsortTile);
    hipLaunchKernelGGL(kern::k_csort_scatter, gsort, b256, 0, S(stream_), I.tb_key.as<uint32_t>(), n, true,
                       hist1, cur1, I.tb_order1.as<uint32_t>());
    kern::TbScanArgs sa{};
    // the scan's rows per lane: GHOSTM_K3_SCAN_S=16 halves them (twice the lanes
    // per hit; its strips map onto the key DP's by a shift)
    Layout slay = lay;
    if (const char *e = getenv("GHOSTM_K3_SCAN_S")) {
      const uint32_t ss = (uint32_t)atoi(e);
      const uint32_t sg = ss == 8 || ss == 16 || ss == 32 ? lay.Lpad / ss : 0;
      if (sg >= lay.G && sg <= 16 && sg * ss == lay.Lpad) slay = Layout{(int)ss, sg, lay.Lpad, 64 / sg};
    }
    uint32_t shift = 0;
    while ((lay.G << shift) < slay.G) ++shift;
    sa.strip_shift = shift;
    sa.qseq = a.qseq;
    sa.L = a.L;
    sa.Lpad = slay.Lpad;
    sa.G = slay.G;
    sa.gpw = slay.gpw;
    sa.db = a.db;
    sa.mat = I.mat_raw.as<int>();
    sa.qid = a.qid;
    sa.end = a.end;
    sa.width = I.tb_width.as<uint32_t>();
    sa.pair_a = I.tb_pair_a.as<uint32_t>();
    sa.pair_b = I.tb_pair_b.as<uint32_t>();
    sa.key = I.tb_key.as<uint32_t>();
    if (q->rcodes_lpad != lay.Lpad) {
      q->rcodes.Reserve((size_t)q->nseq * lay.Lpad + 16);
      const size_t words = (size_t)q->nseq * (lay.Lpad / 4);
      if (words)
        hipLaunchKernelGGL(kern::k_rev_codes, dim3((uint32_t)((words + 255) / 256)), b256, 0, S(stream_),
                           q->seq.as<uint8_t>(), q->nseq, q->L, lay.Lpad, q->rcodes.as<uint32_t>());
      q->rcodes_lpad = lay.Lpad;
    }
    sa.rcodes = q->rcodes.as<uint32_t>();
    sa.n = n;
    sa.base = a.base;
    sa.items = I.tb_order1.as<uint32_t>();
    sa.item_total = hist1 + NB;
    sa.query_order = query_order ? 1u : 0u;
    sa.open = a.open;
    sa.ext = a.ext;
    sa.ncols = I.tb_ncols.as<uint32_t>();
    sa.hist = hist2;
    sa.cells = a.cells ? a.cells + 1 : nullptr;
    // every CU one workgroup (kScanBlock threads), looping over the sorted pairs
    const uint32_t pairs_per_block = (kern::kScanBlock / 64) * slay.gpw;
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)I.cus,
                                                                     (n + pairs_per_block - 1) / pairs_per_block));
    // exact windows (cut at the subject's start) need the DB's subject table
    const bool exact = subj != nullptr;
    sa.best_out = I.tb_best.as<uint32_t>();
    sa.swar_low = (uint32_t)swar_low;
    sa.skey = I.tb_skey.as<uint32_t>();
    sa.strips = strips ? 1u : 0u;
#define GHOSTM_SCAN1(SS, HH, EE, FF)                                                                          \
  hipLaunchKernelGGL((kern::k_tb_scan<SS, HH, EE, FF>), dim3(blocks), dim3(kern::kScanBlock), kScanLds, S(stream_), \
                     sa)
#define GHOSTM_SCANW(SS, EE)                                                                                  \
  hipLaunchKernelGGL((kern::k_tb_scan<SS, true, EE, true, true>), dim3(blocks), dim3(kern::kScanBlock), kScanLds, \
                     S(stream_), sa)
#define GHOSTM_SCANP(SS, EE)                                                                                      \
  hipLaunchKernelGGL((kern::k_tb_scan<SS, true, EE, true, true, true>), dim3(blocks), dim3(kern::kScanBlock), \
                     kScanLdsPriv, S(stream_), sa)
    // GHOSTM_K3_SCAN=priv: the bank-private table (A/B)
    const bool priv = swar && scan_env && strcmp(scan_env, "priv") == 0;
#define GHOSTM_SCAN(SS)                                          \
  if (priv && exact) GHOSTM_SCANP(SS, true);                     \
  else if (priv) GHOSTM_SCANP(SS, false);                        \
  else if (swar && exact) GHOSTM_SCANW(SS, true);                \
  else if (swar) GHOSTM_SCANW(SS, false);                        \
  else if (framed && exact) GHOSTM_SCAN1(SS, true, true, true);  \
  else if (framed) GHOSTM_SCAN1(SS, true, false, true);          \
  else if (half && exact) GHOSTM_SCAN1(SS, true, true, false);   \
  else if (half) GHOSTM_SCAN1(SS, true, false, false);           \
  else if (exact) GHOSTM_SCAN1(SS, false, true, false);          \
  else GHOSTM_SCAN1(SS, false, false, false);
    switch (slay.S) {
      case 32: GHOSTM_SCAN(32); break;
      case 16: GHOSTM_SCAN(16); break;
      default: GHOSTM_SCAN(8); break;
    }
#undef GHOSTM_SCAN
#undef GHOSTM_SCANP
#undef GHOSTM_SCANW
#undef GHOSTM_SCAN1
    hipLaunchKernelGGL(kern::k_csort_scatter, gsort, b256, 0, S(stream_), I.tb_skey.as<uint32_t>(), n, false,
                       hist2, cur2, I.tb_order2.as<uint32_t>(), strips ? class_off : nullptr);
    a.class_off = strips ? class_off : nullptr;
    times_.traceback_launches_strips += strips ? 1 : 0;
    HIP_CHECK(hipGetLastError());
    // the scan phase (prep, pairs, sorts, K3a) ends here; the key DP follows
    HIP_CHECK(hipEventRecord(I.ev_tk, S(stream_)));
    I.tk_recorded = true;
    a.order = I.tb_order2.as<uint32_t>();
    a.ncols = I.tb_ncols.as<uint32_t>();
    a.best_h = I.tb_best.as<uint32_t>();
    a.rcodes = q->rcodes.as<uint32_t>();  // built for this Lpad just above
    times_.traceback_launches_scan += 1;
    times_.traceback_launches_scan_swar += swar ? 1 : 0;
  }
  const uint32_t per_block = (kern::kTbBlock / 64) * lay.gpw;
  // strip classes: each class rounds its last wave up, so one more block covers
  // the (at most kTbStripClasses) extra waves
  const dim3 grid((n + per_block - 1) / per_block + (a.class_off ? 1 : 0)), block(kern::kTbBlock);
  const bool fin = a.best_h != nullptr;  // the scan's maxima: no running maximum in the key DP
  // the framed key DP (kernels.h k_traceback_key FRAME): h + every column's
  // frame, (span + 1) * ext_pen, must still fit the field; GHOSTM_K3_KEYFRAME=0
  // keeps the unframed one
  const char *kf_env = getenv("GHOSTM_K3_KEYFRAME");
  const int64_t kframe = hmax + (int64_t)(span + 1) * (-(int64_t)a.ext);
  const bool frame = fin && !(kf_env && strcmp(kf_env, "0") == 0) && (key16 ? kframe < 8000 : kframe < 4000);
#define GHOSTM_TB(SS)                                                                                                 \
  if (key16 && frame) hipLaunchKernelGGL((kern::k_traceback_key<SS, 16, true, true>), grid, block, 0, S(stream_), a); \
  else if (key16 && fin) hipLaunchKernelGGL((kern::k_traceback_key<SS, 16, true>), grid, block, 0, S(stream_), a);    \
  else if (key16) hipLaunchKernelGGL((kern::k_traceback_key<SS, 16, false>), grid, block, 0, S(stream_), a);          \
  else if (key17 && frame)                                                                                            \
    hipLaunchKernelGGL((kern::k_traceback_key<SS, 17, true, true>), grid, block, 0, S(stream_), a);                   \
  else if (key17 && fin) hipLaunchKernelGGL((kern::k_traceback_key<SS, 17, true>), grid, block, 0, S(stream_), a);    \
  else if (key17) hipLaunchKernelGGL((kern::k_traceback_key<SS, 17, false>), grid, block, 0, S(stream_), a);          \
  else hipLaunchKernelGGL(kern::k_traceback<SS>, grid, block, 0, S(stream_), a);
  switch (lay.S) {
    case 32: GHOSTM_TB(32); break;
    case 16: GHOSTM_TB(16); break;
    default: GHOSTM_TB(8); break;
  }
#undef GHOSTM_TB
  HIP_CHECK(hipGetLastError());
  times_.traceback_launches += 1;
  times_.traceback_launches_key += key ? 1 : 0;
  times_.traceback_launches_keyframe += key && frame ? 1 : 0;
}

void DeviceModule::ResetCarry(DevQuery *q, uint32_t cap) {
  Use();
  Impl &I = *impl_;
  const size_t ng = q->ngroups;
  I.carry_hits.Reserve(ng * cap * sizeof(kern::SlotHit) + 8);
  I.carry_count.Reserve(ng * 4 + 4);
  if (ng) HIP_CHECK(hipMemsetAsync(I.carry_count.p, 0, ng * 4, S(stream_)));
  // every chunk starts its K2 task buffers at the same one, so a repeated run
  // gives each segment the buffer pair it had before: with an odd number of
  // segments the turns alternated between runs, and the second run grew the
  // other staging buffer (a 35 MB hipHostMalloc, 6.4 ms, in the 125 K-query
  // shard's second run, profiles/r5u/)
  if (!I.prepared.valid) I.task_turn = 0;
}

void DeviceModule::SetChunkBases(const uint32_t *bases, uint32_t n) {
  Use();
  Impl &I = *impl_;
  I.chunk_base.Reserve((size_t)n * 4 + 4);
  if (n) HIP_CHECK(hipMemcpy(I.chunk_base.p, bases, (size_t)n * 4, hipMemcpyHostToDevice));
}

void DeviceModule::CarryToHost(DevQuery *q, uint32_t g0, uint32_t g1, uint32_t cap, std::vector<uint32_t> *counts,
                               HostHits *hits) {
  Use();
  Impl &I = *impl_;
  if (g1 > q->ngroups || g0 > g1) throw Error("group range outside the chunk");
  const size_t ng = g1 - g0;
  counts->assign(ng, 0);
  AcquireHostHits(ng * cap, hits);
  if (ng == 0) return;
  HIP_CHECK(hipMemcpyAsync(counts->data(), I.carry_count.as<uint32_t>() + g0, ng * 4, hipMemcpyDeviceToHost,
                           S(stream_)));
  HIP_CHECK(hipMemcpyAsync(hits->data, I.carry_hits.as<kern::SlotHit>() + (size_t)g0 * cap,
                           ng * cap * sizeof(SelectedHit), hipMemcpyDeviceToHost, S(stream_)));
  HIP_CHECK(hipStreamSynchronize(S(stream_)));
}

// K4 + K3 + finalize enqueued behind the segment's K2, no host wait (ev_done
// marks the end); MergeCollect copies the selection back on the copy stream.
void DeviceModule::MergeLaunch(DevQuery *q, DevDb *d, uint32_t g0, uint32_t g1, uint64_t cand_begin, uint64_t n,
                               uint32_t best, uint32_t tb_base, int open, int ext, const MergePass &pass) {
  Use();
  Impl &I = *impl_;
  Impl::MergeState &P = I.merge_state;
  if (P.active) throw Error("MergeLaunch: the previous selection was not collected");
  if (g1 > q->ngroups || g0 > g1) throw Error("group range outside the chunk");
  const uint32_t ng = g1 - g0;
  const uint32_t cap = std::max<uint32_t>(best, 1);
  P = Impl::MergeState();
  P.ng = ng;
  P.slots = (size_t)ng * cap;
  if (ng == 0) return;
  if (d->nsubj == 0) throw Error("DB subjects not set for the device merge");
  const size_t slots = (size_t)ng * cap;
  if (slots >= (1ull << 32)) throw Error("too many result slots in one segment (groups x -b >= 2^32)");
  const bool carry_in = pass.carry_in, carry_out = pass.carry_out;
  if ((carry_in || carry_out) && I.carry_count.bytes < (size_t)q->ngroups * 4)
    throw Error("ResetCarry was not called for this query chunk");
  I.keys.Reserve((n + slots) * 8 + 8);  // per group: its candidates and cap carried keys
  I.sel_from.Reserve(slots * 4);
  I.sel_count.Reserve((size_t)ng * 4);
  I.sel_score.Reserve(slots * 4);
  I.sel_sid.Reserve(slots * 4);
  I.tb_qid.Reserve(slots * 4);
  I.tb_end.Reserve(slots * 4);
  I.tb_start.Reserve(slots * 4);
  I.tb_ml.Reserve(slots * 4);
  I.slot_hits.Reserve(slots * sizeof(kern::SlotHit));
  kern::MergeArgs m{};
  m.group_first = q->group_first.as<uint32_t>() + g0;
  m.group_last = q->group_last.as<uint32_t>() + g0;
  m.ng = ng;
  m.offsets = I.offsets.as<unsigned long long>();
  m.counts = I.counts.as<uint32_t>();
  m.out_base = cand_begin;
  m.score = I.score_out.as<uint32_t>();
  m.end = I.end_out.as<uint32_t>();
  m.cand_qid = I.cand_qid.as<uint32_t>();
  m.subj_start = d->subj.as<uint32_t>();
  m.subj_bucket = d->subj_bucket.as<uint32_t>();
  m.nsubj = d->nsubj;
  m.sid_bits = 0;
  while (m.sid_bits < 32 && (d->nsubj - 1) >> m.sid_bits) ++m.sid_bits;
  m.dblen = d->len;
  m.keys = I.keys.as<unsigned long long>();
  m.best = best;
  m.cap = cap;
  m.sel_count = I.sel_count.as<uint32_t>();
  m.sel_score = I.sel_score.as<uint32_t>();
  m.sel_sid = I.sel_sid.as<uint32_t>();
  m.tb_qid = I.tb_qid.as<uint32_t>();
  m.tb_end = I.tb_end.as<uint32_t>();
  m.cand_lo = pass.cand_lo;
  m.cand_hi = std::min<uint64_t>(pass.cand_hi, I.ncand);
  m.carry_count = carry_in ? I.carry_count.as<uint32_t>() + g0 : nullptr;
  m.carry = carry_in ? I.carry_hits.as<kern::SlotHit>() + (size_t)g0 * cap : nullptr;
  m.sel_from = carry_in ? I.sel_from.as<uint32_t>() : nullptr;
  HIP_CHECK(hipEventRecord(I.ev_m0, S(stream_)));
  // K4: one wave per name group (keys in LDS) for -b up to kMergeBest, else
  // one thread per group; GHOSTM_K4=thread|wave forces one (tests)
  bool wave = best >= 1 && best <= kern::kMergeBest;
  if (const char *force = getenv("GHOSTM_K4")) {
    if (!strcmp(force, "thread")) wave = false;
    else if (!strcmp(force, "wave") && best >= 1 && best <= kern::kMergeBest) wave = true;
  }
  m.wave_cap = kern::kMergeCap;
  if (const char *c = getenv("GHOSTM_K4_CAP"))  // tests: send smaller groups to the one-lane fallback
    m.wave_cap = std::min<uint32_t>((uint32_t)strtoul(c, nullptr, 10), kern::kMergeCap);
  if (wave) {
    // persistent: groups of up to 512 keys in 29 KB workgroups (five per CU),
    // then the larger ones in 53 KB workgroups (three per CU)
    m.wave_small = std::min<uint32_t>(kern::kMergeSmall, m.wave_cap);
    const uint32_t want = (ng + kern::kMergeWaves - 1) / kern::kMergeWaves;
    const uint32_t small = std::max<uint32_t>(1, std::min<uint32_t>(want, (uint32_t)I.cus * 5));
    const uint32_t large = std::max<uint32_t>(1, std::min<uint32_t>(want, (uint32_t)I.cus * 3));
    hipLaunchKernelGGL((kern::k_merge_wave<kern::kMergeSmall, true>), dim3(small), dim3(64 * kern::kMergeWaves), 0,
                       S(stream_), m);
    hipLaunchKernelGGL((kern::k_merge_wave<kern::kMergeCap, false>), dim3(large), dim3(64 * kern::kMergeWaves), 0,
                       S(stream_), m);
  }
  else
    hipLaunchKernelGGL(kern::k_merge, dim3((ng + 255) / 256), dim3(256), 0, S(stream_), m);
  times_.merge_launches += 1;
  times_.merge_launches_wave += wave ? 1 : 0;
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipEventRecord(I.ev_m1, S(stream_)));

  // K3 over the slots (empty slots carry qid 0xFFFFFFFF and are skipped)
  kern::TbArgs a{};
  a.qseq = q->seq.as<uint8_t>();
  a.L = q->L;
  a.db = d->Residues();
  a.mat_tb = I.mat_tb.as<int>();
  a.qid = I.tb_qid.as<uint32_t>();
  a.end = I.tb_end.as<uint32_t>();
  a.n = (uint32_t)slots;
  a.base = tb_base;
  a.open = open;
  a.ext = ext;
  a.out_start = I.tb_start.as<uint32_t>();
  a.out_ml = I.tb_ml.as<uint32_t>();
  // K3 counters: [0] traceback cells, [1] K3a scan cells
  I.tb_counters.Reserve(24);
  HIP_CHECK(hipMemsetAsync(I.tb_counters.p, 0, 24, S(stream_)));
  a.cells = I.tb_counters.as<unsigned long long>();
  HIP_CHECK(hipEventRecord(I.ev_t0, S(stream_)));
  LaunchTraceback(a, q, (uint32_t)slots, d, cap);
  HIP_CHECK(hipEventRecord(I.ev_t1, S(stream_)));
  hipLaunchKernelGGL(kern::k_finalize, dim3((uint32_t)((slots + 255) / 256)), dim3(256), 0, S(stream_),
                     I.sel_count.as<uint32_t>(), I.sel_score.as<uint32_t>(), I.sel_sid.as<uint32_t>(),
                     I.tb_end.as<uint32_t>(), I.tb_start.as<uint32_t>(),
                     I.tb_ml.as<uint32_t>(), d->subj.as<uint32_t>(), ng, cap, pass.chunk,
                     m.sel_from, m.carry, I.slot_hits.as<kern::SlotHit>(),
                     I.tb_counters.as<unsigned long long>() + 2);
  HIP_CHECK(hipGetLastError());
  static_assert(sizeof(kern::SlotHit) == sizeof(SelectedHit), "record layout");
  if (carry_out) {  // the groups' new result lists are the next pass's carry
    HIP_CHECK(hipMemcpyAsync(I.carry_count.as<uint32_t>() + g0, I.sel_count.p, (size_t)ng * 4,
                             hipMemcpyDeviceToDevice, S(stream_)));
    HIP_CHECK(hipMemcpyAsync(I.carry_hits.as<kern::SlotHit>() + (size_t)g0 * cap, I.slot_hits.p,
                             slots * sizeof(kern::SlotHit), hipMemcpyDeviceToDevice, S(stream_)));
  }
  HIP_CHECK(hipEventRecord(I.ev_done, S(stream_)));
  P.active = true;
}

// Waits for the launched K4/K3 and copies counts[ng] (and, unless hits is null,
// the ng * cap selected hits) back on the copy stream, so the main stream can
// already run the next segment's K2. The device buffers are not reused before
// this returns: the next MergeLaunch is issued after it.
void DeviceModule::MergeCollect(std::vector<uint32_t> *counts, HostHits *hits) {
  Use();
  Impl &I = *impl_;
  Impl::MergeState &P = I.merge_state;
  counts->assign(P.ng, 0);
  if (hits) *hits = HostHits();
  if (!P.active) return;
  P.active = false;
  unsigned long long cells[3] = {0, 0, 0};
  HIP_CHECK(hipStreamWaitEvent(S(copy_stream_), I.ev_done, 0));
  HIP_CHECK(hipMemcpyAsync(counts->data(), I.sel_count.p, (size_t)P.ng * 4, hipMemcpyDeviceToHost,
                           S(copy_stream_)));
  if (hits) {  // null: the selection stays on the device (a carried pass)
    AcquireHostHits(P.slots, hits);
    HIP_CHECK(hipMemcpyAsync(hits->data, I.slot_hits.p, P.slots * sizeof(SelectedHit), hipMemcpyDeviceToHost,
                             S(copy_stream_)));
  }
  HIP_CHECK(hipMemcpyAsync(cells, I.tb_counters.p, 24, hipMemcpyDeviceToHost, S(copy_stream_)));
  HIP_CHECK(hipStreamSynchronize(S(copy_stream_)));
  times_.merge += ElapsedMs(I.ev_m0, I.ev_m1) * 1e-3;
  times_.traceback += ElapsedMs(I.ev_t0, I.ev_t1) * 1e-3;
  if (I.tk_recorded) times_.traceback_scan += ElapsedMs(I.ev_t0, I.ev_tk) * 1e-3;
  times_.traceback_cells += cells[0];
  times_.traceback_scan_cells += cells[1];
  times_.traced_hits += cells[2];
}

void DeviceModule::MergeSelect(DevQuery *q, DevDb *d, uint32_t g0, uint32_t g1, uint64_t cand_begin, uint64_t n,
                               uint32_t best, uint32_t tb_base, int open, int ext, std::vector<uint32_t> *counts,
                               HostHits *hits, const MergePass &pass) {
  MergeLaunch(q, d, g0, g1, cand_begin, n, best, tb_base, open, ext, pass);
  MergeCollect(counts, hits);
}

static void GrowRecords(DevBuf &buf, uint64_t records, uint64_t want, hipStream_t st) {
  const size_t need = (size_t)want * sizeof(kern::HitRecord32);
  if (need <= buf.bytes) return;
  DevBuf bigger;
  bigger.Reserve(std::max(need, buf.bytes * 2));
  if (records) HIP_CHECK(hipMemcpyAsync(bigger.p, buf.p, (size_t)records * sizeof(kern::HitRecord32),
                                        hipMemcpyDeviceToDevice, st));
  HIP_CHECK(hipStreamSynchronize(st));
  buf.Release();
  buf = bigger;
  bigger.p = nullptr;
  bigger.bytes = 0;
}

static constexpr uint64_t kRecordReserveMax = 8ull << 30;

void DeviceModule::ResetRecords(uint64_t expect) {
  records_ = 0;
  if (!impl_ || !expect) return;
  Use();
  expect = std::min<uint64_t>(expect, kRecordReserveMax / sizeof(kern::HitRecord32));
  GrowRecords(impl_->records, 0, expect, S(stream_));
}

void DeviceModule::AppendRecords(DevQuery *q, uint32_t g0, const std::vector<uint32_t> &counts, uint32_t cap,
                                 uint32_t q_base, bool from_carry) {
  Use();
  Impl &I = *impl_;
  const uint32_t ng = (uint32_t)counts.size();
  if (ng == 0) return;
  std::vector<uint32_t> &prefix = I.h_rec_prefix;  // kept alive for the async copy
  prefix.resize(ng);
  uint64_t total = 0;
  for (uint32_t g = 0; g < ng; ++g) {
    prefix[g] = (uint32_t)total;
    total += counts[g];
  }
  if (total == 0) return;
  GrowRecords(I.records, records_, records_ + total, S(stream_));
  I.rec_prefix.Reserve((size_t)ng * 4);
  HIP_CHECK(hipMemcpyAsync(I.rec_prefix.p, prefix.data(), (size_t)ng * 4, hipMemcpyHostToDevice, S(stream_)));
  const uint32_t *cnt = from_carry ? I.carry_count.as<uint32_t>() + g0 : I.sel_count.as<uint32_t>();
  const kern::SlotHit *sh = from_carry ? I.carry_hits.as<kern::SlotHit>() + (size_t)g0 * cap
                                       : I.slot_hits.as<kern::SlotHit>();
  hipLaunchKernelGGL(kern::k_records, dim3((ng + 255) / 256), dim3(256), 0, S(stream_), cnt, sh,
                     I.rec_prefix.as<uint32_t>(),
                     q->group_last.as<uint32_t>() + g0, ng, cap, q_base, I.chunk_base.as<uint32_t>(),
                     I.records.as<kern::HitRecord32>() + records_);
  HIP_CHECK(hipGetLastError());
  records_ += total;
}

void DeviceModule::UploadRecords(const void *recs, uint64_t n) {
  Use();
  Impl &I = *impl_;
  records_ = 0;
  if (n == 0) return;
  GrowRecords(I.records, 0, n, S(stream_));
  HIP_CHECK(hipMemcpy(I.records.p, recs, (size_t)n * sizeof(kern::HitRecord32), hipMemcpyHostToDevice));
  records_ = n;
}

void DeviceModule::CopyRecords(void *dst, uint64_t n) {
  Use();
  Impl &I = *impl_;
  n = std::min(n, records_);
  if (n == 0) return;
  HIP_CHECK(hipMemcpyAsync(dst, I.records.p, (size_t)n * sizeof(kern::HitRecord32), hipMemcpyDeviceToDevice,
                           S(stream_)));
  HIP_CHECK(hipStreamSynchronize(S(stream_)));
}

void DeviceModule::TraceBack(DevQuery *q, DevDb *d, uint32_t n, const uint32_t *qid,
                             const uint32_t *db_end, uint32_t base, int open, int ext,
                             uint32_t *db_start, uint32_t *aln_len, uint32_t *aln_match,
                             float *seq_id) {
  Use();
  Impl &I = *impl_;
  if (n == 0) return;
  I.tb_qid.Reserve((size_t)n * 4);
  I.tb_end.Reserve((size_t)n * 4);
  I.tb_start.Reserve((size_t)n * 4);
  I.tb_ml.Reserve((size_t)n * 4);
  HIP_CHECK(hipMemcpyAsync(I.tb_qid.p, qid, (size_t)n * 4, hipMemcpyHostToDevice, S(stream_)));
  HIP_CHECK(hipMemcpyAsync(I.tb_end.p, db_end, (size_t)n * 4, hipMemcpyHostToDevice, S(stream_)));
  kern::TbArgs a{};
  a.qseq = q->seq.as<uint8_t>();
  a.L = q->L;
  a.db = d->Residues();
  a.mat_tb = I.mat_tb.as<int>();
  a.qid = I.tb_qid.as<uint32_t>();
  a.end = I.tb_end.as<uint32_t>();
  a.n = n;
  a.base = base;
  a.open = open;
  a.ext = ext;
  a.out_start = I.tb_start.as<uint32_t>();
  a.out_ml = I.tb_ml.as<uint32_t>();
  I.tb_counters.Reserve(16);
  HIP_CHECK(hipMemsetAsync(I.tb_counters.p, 0, 16, S(stream_)));
  a.cells = I.tb_counters.as<unsigned long long>();
  HIP_CHECK(hipEventRecord(I.ev0, S(stream_)));
  LaunchTraceback(a, q, n, d, kern::kPairRun);
  HIP_CHECK(hipEventRecord(I.ev1, S(stream_)));
  std::vector<uint32_t> ml(n);
  HIP_CHECK(hipMemcpyAsync(db_start, I.tb_start.p, (size_t)n * 4, hipMemcpyDeviceToHost, S(stream_)));
  HIP_CHECK(hipMemcpyAsync(ml.data(), I.tb_ml.p, (size_t)n * 4, hipMemcpyDeviceToHost, S(stream_)));
  unsigned long long cells = 0;
  unsigned long long scan_cells = 0;
  HIP_CHECK(hipMemcpyAsync(&cells, I.tb_counters.p, 8, hipMemcpyDeviceToHost, S(stream_)));
  HIP_CHECK(hipMemcpyAsync(&scan_cells, I.tb_counters.as<unsigned long long>() + 1, 8, hipMemcpyDeviceToHost,
                           S(stream_)));
  HIP_CHECK(hipStreamSynchronize(S(stream_)));
  times_.traceback += ElapsedMs(I.ev0, I.ev1) * 1e-3;
  if (I.tk_recorded) times_.traceback_scan += ElapsedMs(I.ev0, I.ev_tk) * 1e-3;
  times_.traceback_cells += cells;
  times_.traceback_scan_cells += scan_cells;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t len = ml[i] >> 8, match = ml[i] & 0xFFu;
    if (aln_len) aln_len[i] = len;
    if (aln_match) aln_match[i] = match;
    // seq_id as the reference computes it on the host (aligner.cpp:945)
    if (seq_id) seq_id[i] = (float)match / (float)len;
  }
}

const char *SourceHash();  // build_hash.cpp, generated by the Makefile (ghostm_amd/srchash.py)

const char *DeviceBuildInfo() {
  static const std::string info =
      std::string("ghostm_hip gfx950: K1 k_seed_lists/k_seed_filter/k_seed_hash/k_seed, K2 k_score16f/k_score16/"
                  "k_score, K3 k_tb_scan/k_traceback_key/k_traceback, K4 k_merge_wave/k_merge"
#ifdef GHOSTM_LDS_POISON
                  "; LDS poison build"
#endif
#ifdef GHOSTM_ALT_TAG
                  "; A/B build " GHOSTM_ALT_TAG
#endif
                  ) +
      "; src " + SourceHash();
  return info.c_str();
}

// ============================================================ reference C ABI
namespace {

struct RefState {
  std::mutex mu;
  uint32_t max_list_length = 0;
  DevQuery *query = nullptr;
  DevDb *db = nullptr;
  bool seeded = false;
  std::vector<uint32_t> counts;
  std::vector<uint64_t> offsets;
  // last batch (SearchNextGpu)
  uint32_t batch_first = 0, batch_count = 0;
  uint64_t batch_begin = 0, batch_n = 0;
};

RefState &Ref() {
  static RefState *s = new RefState();
  return *s;
}

void SetError(const std::string &m) { g_last_error = m; }

}  // namespace

void SetLastErrorMessage(const std::string &m) { g_last_error = m; }

}  // namespace ghostm

using namespace ghostm;

extern "C" {

const char *GhostmGetLastError(void) { return g_last_error.c_str(); }

const char *GhostmBuildInfo(void) { return DeviceBuildInfo(); }

uint64_t GhostmDevicePoolTrim(void) { return DevPool::Get().Trim(); }

int GhostmDevicePoolInfo(uint64_t *cached_bytes, uint64_t *oom_retries) {
  if (cached_bytes) *cached_bytes = DevPool::Get().Cached();
  if (oom_retries) *oom_retries = DevPool::Get().OomRetries();
  return 0;
}

int InitGpu(void) {
  RefState &r = Ref();
  std::lock_guard<std::mutex> lk(r.mu);
  DeviceModule &m = DeviceModule::Get();
  if (r.query) m.Free(r.query);
  if (r.db) m.Free(r.db);
  r.query = nullptr;
  r.db = nullptr;
  r.seeded = false;
  r.counts.clear();
  r.offsets.clear();
  g_last_error.clear();
  return 0;
}

size_t GetNeededGPUMemorySize(uint32_t seed, uint32_t shift_size, uint32_t max_list_length,
                              uint32_t max_query_length, uint32_t max_number_queries,
                              uint32_t max_db_length) {
  const uint32_t w = SeedWeight(seed);
  uint64_t kcl = 1;
  for (uint32_t i = 0; i < w; ++i) kcl *= 32;
  kcl += 1;
  const uint32_t seed_len = SeedLength(seed);
  const uint64_t nq = max_number_queries;
  const uint64_t lists = max_query_length >= seed_len && shift_size
                             ? (max_query_length - seed_len) / shift_size + 1
                             : 0;
  (void)lists;
  size_t b = 0;
  b += (size_t)nq * max_query_length;             // query records
  b += (size_t)nq * (4 + 4 + 8 + 256 * 4);          // counts, nelem, offsets, slots
  b += (size_t)max_list_length * 16;                // start, qid, score, end
  b += (size_t)max_db_length * (1 + 4);             // sequence + positions
  b += (size_t)kcl * 4;                             // CSR offsets
  b += 2 * 32 * 32 * 4;                             // score tables
  return b;
}

int CheckGpuMemory(uint32_t seed, uint32_t shift_size, uint32_t max_list_length,
                   uint32_t max_query_length, uint32_t max_number_queries, uint32_t max_db_length) {
  try {
    size_t free_b = 0, total_b = 0;
    int dev = DeviceModule::Get().device();
    if (dev < 0) HIP_CHECK(hipSetDevice(0));
    HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    return GetNeededGPUMemorySize(seed, shift_size, max_list_length, max_query_length,
                                  max_number_queries, max_db_length) > total_b ? 1 : 0;
  } catch (std::exception &e) {
    SetError(e.what());
    return 1;
  }
}

int SetOptionGpu(uint32_t max_list_length, int score_matrix[], int device) {
  try {
    RefState &r = Ref();
    std::lock_guard<std::mutex> lk(r.mu);
    DeviceModule &m = DeviceModule::Get();
    m.Bind(device);
    m.SetMatrix(score_matrix);
    r.max_list_length = max_list_length;
    return 0;
  } catch (std::exception &e) {
    SetError(e.what());
    return 1;
  }
}

void printGpuInfo(int device) {
  try {
    hipDeviceProp_t p;
    HIP_CHECK(hipGetDeviceProperties(&p, device));
    fprintf(stdout, "  [GPU] device: \"%s\"\n", p.name);
    fprintf(stdout, "  [GPU] global memory size: %lu bytes (%gMB)\n", (unsigned long)p.totalGlobalMem,
            p.totalGlobalMem / 1048576.0);
  } catch (std::exception &e) {
    SetError(e.what());
  }
}

int SetQueryGpu(uint8_t sequences[], uint32_t number_sequences, uint32_t sequence_length) {
  try {
    RefState &r = Ref();
    std::lock_guard<std::mutex> lk(r.mu);
    DeviceModule &m = DeviceModule::Get();
    if (r.query) m.Free(r.query);
    r.query = m.UploadQuery(sequences, number_sequences, sequence_length);
    r.seeded = false;
    return 0;
  } catch (std::exception &e) {
    SetError(e.what());
    return 1;
  }
}

int SetDbGpu(uint8_t sequences[], uint32_t sequences_legnth, uint32_t keys_count[],
             uint32_t keys_count_length, uint32_t positions[], uint32_t positions_length) {
  try {
    RefState &r = Ref();
    std::lock_guard<std::mutex> lk(r.mu);
    DeviceModule &m = DeviceModule::Get();
    if (r.db) m.Free(r.db);
    r.db = m.UploadDb(sequences, sequences_legnth, keys_count, keys_count_length, positions,
                      positions_length);
    r.seeded = false;
    return 0;
  } catch (std::exception &e) {
    SetError(e.what());
    return 1;
  }
}

uint32_t SearchNextGpu(uint32_t query_sequence_length, uint32_t number_query_sequences,
                       uint32_t seed, uint32_t threshold, uint32_t shift_size,
                       uint32_t log_region_size, uint32_t max_number_alignments,
                       uint32_t start_query_id, uint32_t *alignment_count_list, uint32_t *starts) {
  try {
    RefState &r = Ref();
    std::lock_guard<std::mutex> lk(r.mu);
    if (!r.query || !r.db) throw Error("SetQueryGpu/SetDbGpu not called");
    if (start_query_id >= number_query_sequences) return 0;
    if (query_sequence_length != r.query->L || number_query_sequences != r.query->nseq)
      throw Error("query shape differs from SetQueryGpu");
    DeviceModule &m = DeviceModule::Get();
    if (!r.seeded || start_query_id == 0) {
      SeedConfig cfg;
      cfg.seed_mask = seed;
      cfg.threshold = threshold;
      cfg.shift = shift_size;
      cfg.log_region = log_region_size;
      m.Seed(r.query, r.db, cfg, &r.counts, &r.offsets);
      r.seeded = true;
    }
    // reference GPU batching rule (aligner_gpu.cu:911-920)
    uint64_t total = 0;
    uint32_t j = 1;
    alignment_count_list[0] = 0;
    for (uint32_t i = start_query_id; i < number_query_sequences; ++i, ++j) {
      if (total + r.counts[i] >= max_number_alignments) break;
      total += r.counts[i];
      alignment_count_list[j] = (uint32_t)total;
    }
    const uint32_t qcount = j - 1;
    r.batch_first = start_query_id;
    r.batch_count = qcount;
    r.batch_begin = r.offsets[start_query_id];
    r.batch_n = total;
    m.CopyStarts(r.batch_begin, total, starts);
    return qcount;
  } catch (std::exception &e) {
    SetError(e.what());
    fprintf(stderr, "[ghostm_hip] SearchNextGpu: %s\n", e.what());
    return 0;
  }
}

void CalculateScoreGpu(uint32_t db_length, uint32_t query_sequence_length,
                       uint32_t number_alignment_list, uint32_t scores[], uint32_t ends[],
                       uint32_t base_search_length, uint32_t offset, int open_gap, int extend_gap) {
  try {
    RefState &r = Ref();
    std::lock_guard<std::mutex> lk(r.mu);
    if (!r.seeded) throw Error("SearchNextGpu not called");
    (void)db_length;
    (void)query_sequence_length;
    GapConfig gap;
    gap.extend = offset;
    gap.open = open_gap;
    gap.ext = extend_gap;
    const uint64_t n = std::min<uint64_t>(number_alignment_list, r.batch_n);
    DeviceModule::Get().Score(r.query, r.db, r.batch_begin, n, r.batch_first,
                              r.batch_first + r.batch_count, r.counts, r.offsets,
                              base_search_length, gap, scores, ends);
  } catch (std::exception &e) {
    SetError(e.what());
    fprintf(stderr, "[ghostm_hip] CalculateScoreGpu: %s\n", e.what());
  }
}

int FreeGpu(void) {
  try {
    RefState &r = Ref();
    std::lock_guard<std::mutex> lk(r.mu);
    DeviceModule &m = DeviceModule::Get();
    if (r.query) m.Free(r.query);
    if (r.db) m.Free(r.db);
    r.query = nullptr;
    r.db = nullptr;
    r.seeded = false;
    return 0;
  } catch (std::exception &e) {
    SetError(e.what());
    return 1;
  }
}

int CountCandidatesGpu(uint32_t query_sequence_length, uint32_t number_query_sequences,
                       uint32_t seed, uint32_t threshold, uint32_t shift_size,
                       uint32_t log_region_size, uint32_t counts[]) {
  try {
    RefState &r = Ref();
    std::lock_guard<std::mutex> lk(r.mu);
    if (!r.query || !r.db) throw Error("SetQueryGpu/SetDbGpu not called");
    if (query_sequence_length != r.query->L || number_query_sequences != r.query->nseq)
      throw Error("query shape differs from SetQueryGpu");
    SeedConfig cfg;
    cfg.seed_mask = seed;
    cfg.threshold = threshold;
    cfg.shift = shift_size;
    cfg.log_region = log_region_size;
    DeviceModule::Get().Seed(r.query, r.db, cfg, &r.counts, &r.offsets);
    r.seeded = true;
    std::copy(r.counts.begin(), r.counts.end(), counts);
    return 0;
  } catch (std::exception &e) {
    SetError(e.what());
    return 1;
  }
}

int TraceBackGpu(uint32_t nhits, const uint32_t query_ids[], const uint32_t db_ends[],
                 uint32_t query_sequence_length, uint32_t base_search_length, int open_gap,
                 int extend_gap, uint32_t db_starts[], uint32_t aln_lens[],
                 uint32_t aln_matches[], float seq_ids[]) {
  try {
    RefState &r = Ref();
    std::lock_guard<std::mutex> lk(r.mu);
    if (!r.query || !r.db) throw Error("SetQueryGpu/SetDbGpu not called");
    if (query_sequence_length != r.query->L) throw Error("query shape differs from SetQueryGpu");
    DeviceModule::Get().TraceBack(r.query, r.db, nhits, query_ids, db_ends, base_search_length,
                                  open_gap, extend_gap, db_starts, aln_lens, aln_matches, seq_ids);
    return 0;
  } catch (std::exception &e) {
    SetError(e.what());
    return 1;
  }
}

}  // extern "C"
