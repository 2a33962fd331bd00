// aligner.cpp — see aligner.h.
#include "aligner.h"

#include <fcntl.h>
#include <getopt.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <fstream>
#include <iostream>
#include <stdexcept>
#include <thread>

#include "common.h"
#include "worker_pool.h"

namespace ghostm {

// ------------------------------------------------------------------ trace
namespace {
struct TraceEvent {
  double t;
  const char *label;
  uint64_t value;
  std::thread::id thread;
};
std::mutex g_trace_mu;
std::vector<TraceEvent> g_trace;
}  // namespace

double ThreadCpuSeconds() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

bool TraceOn() {
  static const bool on = [] {
    const char *e = getenv("GHOSTM_TRACE");
    return e && *e && strcmp(e, "0") != 0;
  }();
  return on;
}

void TraceMark(const char *label, uint64_t value) {
  if (!TraceOn()) return;
  const double t = NowSeconds();
  std::lock_guard<std::mutex> lk(g_trace_mu);
  g_trace.push_back(TraceEvent{t, label, value, std::this_thread::get_id()});
}

void TraceDump() {
  if (!TraceOn()) return;
  std::lock_guard<std::mutex> lk(g_trace_mu);
  if (g_trace.empty()) return;
  const double t0 = g_trace.front().t;
  const std::thread::id main = g_trace.front().thread;
  for (const TraceEvent &e : g_trace)
    fprintf(stderr, "trace %9.3f %s %-18s %llu\n", (e.t - t0) * 1e3, e.thread == main ? "M" : "F", e.label,
            (unsigned long long)e.value);
  g_trace.clear();
}

unsigned HostThreads() {
  if (const char *e = getenv("GHOSTM_THREADS")) {
    const int v = atoi(e);
    if (v > 0) return (unsigned)v;
  }
  // the CPUs this process may run on: its affinity mask, capped by a cgroup v2
  // CPU quota ("<quota> <period>" in cpu.max; "max" = none)
  unsigned cpus = std::thread::hardware_concurrency();
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = (unsigned)CPU_COUNT(&set);
  {
    std::ifstream f("/sys/fs/cgroup/cpu.max");
    std::string quota;
    uint64_t period = 0;
    if (f >> quota >> period && quota != "max" && period > 0) {
      const uint64_t q = strtoull(quota.c_str(), nullptr, 10);
      if (q > 0) cpus = std::min<unsigned>(cpus, (unsigned)std::max<uint64_t>(1, (q + period - 1) / period));
    }
  }
  // shared among the ranks of this node (torchrun sets LOCAL_WORLD_SIZE)
  unsigned ranks = 1;
  if (const char *e = getenv("LOCAL_WORLD_SIZE")) ranks = (unsigned)std::max(1, atoi(e));
  const unsigned share = std::max(1u, cpus) / ranks;
  return std::max(1u, std::min(share, 16u));
}


void ParallelFor(size_t n, unsigned threads,
                 const std::function<void(size_t, size_t, unsigned)> &fn) {
  if (n == 0) return;
  threads = (unsigned)std::max<size_t>(1, std::min<size_t>(threads, n));
  if (threads == 1) {
    fn(0, n, 0);
    return;
  }
  const size_t per = (n + threads - 1) / threads;
  const unsigned pieces = (unsigned)((n + per - 1) / per);
  WorkerPool::Get().Run(pieces, [&](unsigned t) { fn(t * per, std::min(n, (size_t)t * per + per), t); });
}

size_t PieceCount(size_t n, size_t pieces) {
  if (n == 0) return 0;
  const size_t per = (n + std::max<size_t>(1, std::min(pieces, n)) - 1) / std::max<size_t>(1, std::min(pieces, n));
  return (n + per - 1) / per;
}

void ParallelForPieces(size_t n, size_t pieces, unsigned threads,
                       const std::function<void(size_t, size_t, unsigned)> &fn) {
  const size_t np = PieceCount(n, pieces);
  if (np == 0) return;
  const size_t per = (n + np - 1) / np;
  if (threads <= 1 || np == 1) {
    for (size_t t = 0; t < np; ++t) fn(t * per, std::min(n, t * per + per), (unsigned)t);
    return;
  }
  WorkerPool::Get().Run((unsigned)np, [&](unsigned t) { fn(t * per, std::min(n, (size_t)t * per + per), t); },
                        threads);
}

// ------------------------------------------------------------------ TaskQueue
TaskQueue::TaskQueue() : worker_([this] { Loop(); }) {}

TaskQueue::~TaskQueue() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  worker_.join();
}

void TaskQueue::Submit(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    tasks_.push_back(std::move(fn));
  }
  cv_.notify_one();
}

void TaskQueue::Drain() {
  std::unique_lock<std::mutex> lk(mu_);
  idle_.wait(lk, [this] { return tasks_.empty() && !busy_; });
  if (error_) {
    std::exception_ptr e = error_;
    error_ = nullptr;
    std::rethrow_exception(e);
  }
}

void TaskQueue::Loop() {
  for (;;) {
    std::function<void()> fn;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return stop_ || !tasks_.empty(); });
      if (tasks_.empty()) return;
      fn = std::move(tasks_.front());
      tasks_.pop_front();
      busy_ = true;
    }
    try {
      fn();
    } catch (...) {
      std::lock_guard<std::mutex> lk(mu_);
      if (!error_) error_ = std::current_exception();
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      busy_ = false;
    }
    idle_.notify_all();
  }
}

// ------------------------------------------------------------------ options
AlignerOptions ParseAlignerOptions(int argc, char **argv) {
  AlignerOptions o;
  std::string matrix_file = "BLOSUM62";
  optind = 1;
  opterr = 1;
  int c;
  while ((c = getopt(argc, argv, "b:d:D:e:E:G:i:l:M:o:r:s:t:S:L:y:v")) >= 0) {
    switch (c) {
      case 'b': o.best = atoi(optarg); break;
      case 'd': o.db_prefix = optarg; break;
      case 'D': o.device = atoi(optarg); break;
      case 'e': o.extend = atoi(optarg); break;
      case 'E': o.extend_gap = -atoi(optarg); break;
      case 'G': o.open_gap = -atoi(optarg); break;
      case 'i': o.query_prefix = optarg; break;
      case 'S': o.start_query_chunk = atoi(optarg); break;
      case 'L': o.end_query_chunk = atoi(optarg); break;
      case 'l': o.max_list_length = atoi(optarg) * (1 << 20); break;
      case 'M': matrix_file = optarg; break;
      case 'o': o.output_file = optarg; break;
      case 'r': {
        const int lr = (int)log2(atoi(optarg));
        o.log_region = lr < 1 ? 1 : lr;
        break;
      }
      case 's': o.shift = atoi(optarg); break;
      case 't': o.threshold = atoi(optarg); break;
      case 'y': o.output_style = atoi(optarg); break;
      case 'v': o.verbose = true; break;
      default: throw std::invalid_argument("");
    }
  }
  // test hook: -l in candidates instead of MiB units (exercises batch cuts on
  // small inputs); the oracle honours the same variable
  if (const char *e = getenv("GHOSTM_MAX_LIST_OVERRIDE")) o.max_list_length = (uint32_t)strtoul(e, nullptr, 10);
  o.matrix = ReadScoreMatrix(matrix_file);
  if (o.output_style == 0) {
    // extension: GHOSTM_KARLIN=ungapped prices combinations the
    // reference's table lacks with the matrix's ungapped ideal parameters
    // (karlin_params.cpp); unset, they throw as the reference does
    const char *kp = getenv("GHOSTM_KARLIN");
    if (kp && std::string(kp) == "ungapped") {
      try {
        o.karlin = GappedKarlinParams(o.matrix, o.open_gap, o.extend_gap);
      } catch (std::invalid_argument &) {
        o.karlin = UngappedKarlinParams(o.matrix);
      }
    } else {
      o.karlin = GappedKarlinParams(o.matrix, o.open_gap, o.extend_gap);
    }
  }
  return o;
}

// ------------------------------------------------------------------ shards
void ShardCuts(uint64_t n, const uint32_t *weight, const uint8_t *group_start, uint32_t world, uint64_t *cuts) {
  if (world == 0) throw std::invalid_argument("world must be >= 1");
  std::vector<uint64_t> prefix(n + 1, 0);
  for (uint64_t i = 0; i < n; ++i) prefix[i + 1] = prefix[i] + weight[i];
  const unsigned __int128 total = prefix[n];
  cuts[0] = 0;
  for (uint32_t r = 1; r < world; ++r) {
    // first group start at or after the previous cut whose prefix weight
    // reaches total * r / world (exact integer comparison)
    uint64_t c = cuts[r - 1];
    while (c < n && !((c == 0 || group_start[c]) && (unsigned __int128)prefix[c] * world >= total * r)) ++c;
    cuts[r] = c;
  }
  cuts[world] = n;
}

// The CPU path's batch cuts (aligner.cpp:383-521 driven by Execute's loop at
// 131-171): a query whose candidates push the running total above -l is carried
// into the next batch; the loop stops at the first empty batch, so a carried last
// query is dropped, exactly as the reference does.
std::vector<Batch> CpuBatches(const std::vector<uint32_t> &counts, uint64_t max_list) {
  std::vector<Batch> out;
  const uint32_t n = (uint32_t)counts.size();
  uint32_t next = 0;
  int64_t carry = -1;
  for (;;) {
    if (next == n) break;
    uint32_t first = next;
    uint64_t total = 0;
    if (carry >= 0) {
      first = (uint32_t)carry;
      total = counts[carry];
    }
    carry = -1;
    uint32_t i = next;
    bool cut = false;
    for (; i < n; ++i) {
      total += counts[i];
      if (total > max_list) { cut = true; break; }
    }
    const uint64_t cands = cut ? total - counts[i] : total;
    const uint32_t stop = cut ? i : n;
    if (cut) { next = i + 1; carry = i; } else { next = n; }
    if (cands == 0) break;
    out.push_back(Batch{first, stop});
  }
  return out;
}

namespace {
// FNV-1a over a slice's candidate counts: a shard's runs must see the counts
// its batch plan was made from
uint64_t CountsHash(const uint32_t *c, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) {
    h ^= c[i];
    h *= 1099511628211ull;
  }
  return h;
}
}  // namespace

// Name groups (consecutive equal names, merged into one result list:
// aligner.cpp:697-700) and (qlen) WriteOutput's query lengths of one query chunk.
void Session::PrepareQueryChunk(QueryData *qd, bool qlen) {
  QueryData &q = *qd;
  const uint32_t n = q.chunk.nseq, L = q.chunk.L;
  q.group_end.assign(n, 0);
  q.group_first.clear();
  q.group_last.clear();
  for (uint32_t i = n; i-- > 0;) {
    q.group_end[i] = (i + 1 < n && q.chunk.names[i + 1] == q.chunk.names[i]) ? q.group_end[i + 1] : i + 1;
  }
  for (uint32_t i = 0; i < n; i = q.group_end[i]) {
    q.group_first.push_back(i);
    q.group_last.push_back(q.group_end[i] - 1);
  }
  if (!qlen) return;
  q.qlen.assign(n, 1);
  for (uint32_t i = 0; i < n; ++i) q.qlen[i] = QueryResidues(&q.chunk.seq[(size_t)i * L], L);
}

// WriteOutput's query lengths of every loaded chunk on the worker pool, in
// blocks of rows (a row's last byte per 127: ~9 ms per 500 K-query chunk on one
// thread, the largest part of reading a chunk once its names are a NameTable).
void Session::QueryLengths(std::vector<QueryData *> chunks) {
  constexpr uint32_t kRows = 1u << 12;
  std::vector<std::pair<QueryData *, uint32_t>> blocks;
  for (QueryData *q : chunks) {
    q->qlen.assign(q->chunk.nseq, 1);
    for (uint32_t r = 0; r < q->chunk.nseq; r += kRows) blocks.emplace_back(q, r);
  }
  ParallelFor(blocks.size(), std::max(1u, threads_), [&](size_t b, size_t e, unsigned) {
    for (size_t k = b; k < e; ++k) {
      QueryData &q = *blocks[k].first;
      const uint32_t L = q.chunk.L, r1 = std::min(q.chunk.nseq, blocks[k].second + kRows);
      for (uint32_t i = blocks[k].second; i < r1; ++i) q.qlen[i] = QueryResidues(&q.chunk.seq[(size_t)i * L], L);
    }
  });
}

// The batch plan of a slice against DB chunk di, from the counts of its WHOLE
// chunk: the unsharded run's batches (aligner.cpp:131-171, 511-514), which every
// shard replays on its own queries (see Passes).
void Session::PlanFromCounts(QueryData &q, size_t di, const std::vector<uint32_t> &chunk_counts, uint32_t n) {
  if (q.plan.size() <= di) {
    q.plan.resize(di + 1);
    q.plan_sum.resize(di + 1);
    q.plan_hash.resize(di + 1);
  }
  q.plan[di] = CpuBatches(chunk_counts, opt_.max_list_length);
  uint64_t sum = 0;
  for (uint32_t i = 0; i < n; ++i) sum += chunk_counts[q.slice_lo + i];
  q.plan_sum[di] = sum;
  q.plan_hash[di] = CountsHash(chunk_counts.data() + q.slice_lo, n);
  q.planned = true;
}

// Without a collective: the shard counts every query of each chunk it touches
// itself (K1 on the whole chunk, once), then keeps only its own range. The
// chunks' queries are cut into `world` contiguous ranges of about equal
// residues, at name-group starts (groups never span chunks: the reference
// merges per chunk, aligner.cpp:697-700).
void Session::ApplyShard(uint32_t rank, uint32_t world) {
  DeviceModule &dev = DeviceModule::Get();
  std::vector<uint32_t> weight;
  std::vector<uint8_t> start;
  for (const QueryData &q : queries_) {
    const QueryChunk &c = q.chunk;
    for (uint32_t i = 0; i < c.nseq; ++i) {
      weight.push_back(q.qlen[i]);
      start.push_back(i == 0 || c.names[i] != c.names[i - 1]);
    }
  }
  std::vector<uint64_t> cuts(world + 1);
  ShardCuts(weight.size(), weight.data(), start.data(), world, cuts.data());
  const uint64_t lo = cuts[rank], hi = cuts[rank + 1];
  shard_begin_ = lo;
  shard_end_ = hi;
  SeedConfig sc;
  sc.threshold = opt_.threshold;
  sc.shift = opt_.shift;
  sc.log_region = opt_.log_region;
  std::vector<QueryData> kept;
  uint64_t at = 0;  // index of the chunk's first query over the loaded chunks
  for (QueryData &q : queries_) {
    QueryChunk &c = q.chunk;
    const uint64_t chunk_end = at + c.nseq;
    const uint64_t b = std::max<uint64_t>(lo, at), e = std::min<uint64_t>(hi, chunk_end);
    if (b < e) {
      const uint32_t i0 = (uint32_t)(b - at), n = (uint32_t)(e - b);
      // the whole chunk's counts against every DB chunk -> its batch plan
      q.slice_lo = i0;
      q.chunk_nseq = c.nseq;
      {
        // the whole chunk on the device while it is counted; freed on every exit
        std::unique_ptr<DevQuery, std::function<void(DevQuery *)>> full(
            dev.UploadQuery(c.seq.data(), c.nseq, c.L), [&dev](DevQuery *p) { dev.Free(p); });
        std::vector<uint32_t> counts;
        std::vector<uint64_t> offsets;
        for (size_t di = 0; di < dbs_.size(); ++di) {
          sc.seed_mask = dbs_[di].chunk.seed;
          dev.Seed(full.get(), dbs_[di].dev, sc, &counts, &offsets);
          PlanFromCounts(q, di, counts, n);
        }
      }
      c.seq.Own(std::vector<uint8_t>(c.seq.begin() + (size_t)i0 * c.L, c.seq.begin() + (size_t)(i0 + n) * c.L));
      c.names = c.names.Slice(i0, n);
      c.nseq = n;
      q.global_base += i0;
      PrepareQueryChunk(&q);
      kept.push_back(std::move(q));
    }
    at = chunk_end;
  }
  queries_.swap(kept);
}

// With a collective: every rank has counted its own slices; the ranks
// all-gather their candidate totals per (query chunk, DB chunk). A chunk whose
// total fits -l is one batch, as in the unsharded run; otherwise the ranks
// all-gather the chunk's per-query counts and cut it with the CPU rule.
// chunk_nseq[c] = queries of chunk c, rank_lo[c][r] = rank r's first query in
// chunk c (rank_lo[c][world] = chunk_nseq[c]).
void Session::PlanExchange(uint32_t rank, uint32_t world, const ShardExchange &ex,
                           const std::vector<uint32_t> &chunk_nseq,
                           const std::vector<std::vector<uint64_t>> &rank_lo) {
  DeviceModule &dev = DeviceModule::Get();
  const size_t nc = chunk_nseq.size(), nd = dbs_.size();
  SeedConfig sc;
  sc.threshold = opt_.threshold;
  sc.shift = opt_.shift;
  sc.log_region = opt_.log_region;
  // this rank's counts per (chunk, DB chunk); queries_ holds its slices in chunk order
  std::vector<QueryData *> slice(nc, nullptr);
  {
    size_t k = 0;
    for (size_t c = 0; c < nc; ++c)
      if (rank_lo[c][rank] < rank_lo[c][rank + 1]) slice[c] = &queries_.at(k++);
    if (k != queries_.size()) throw Error("shard slices out of order");
  }
  std::vector<std::vector<uint32_t>> mine(nc * nd);
  // the candidate totals per (chunk, DB chunk), then this rank's ok flag: a
  // rank whose counting fails still takes part in the gather, and every rank
  // then fails
  const size_t np = nc * nd;
  std::vector<uint64_t> sums(np + 1, 0);
  std::string err;
  try {
    for (size_t c = 0; c < nc; ++c) {
      if (!slice[c]) continue;
      std::vector<uint64_t> offsets;
      for (size_t di = 0; di < nd; ++di) {
        sc.seed_mask = dbs_[di].chunk.seed;
        sums[c * nd + di] = dev.Seed(slice[c]->dev, dbs_[di].dev, sc, &mine[c * nd + di], &offsets);
      }
    }
  } catch (std::exception &e) {
    err = e.what();
    if (err.empty()) err = "shard session: counting failed";
  }
  sums[np] = err.empty() ? 1 : 0;
  auto gather = [&](const void *send, uint64_t bytes, void *recv, const std::vector<uint64_t> &sizes) {
    if (ex.fn(ex.ctx, send, bytes, recv, sizes.data()) != 0) throw Error("shard exchange (all-gather) failed");
  };
  std::vector<uint64_t> all(world * (np + 1));
  gather(sums.data(), sums.size() * 8, all.data(), std::vector<uint64_t>(world, sums.size() * 8));
  if (!err.empty()) throw Error(err);
  for (uint32_t r = 0; r < world; ++r)
    if (all[r * (np + 1) + np] != 1)
      throw Error("shard session: rank " + std::to_string(r) + " failed counting its queries");
  std::vector<uint64_t> total(np, 0);
  for (uint32_t r = 0; r < world; ++r)
    for (size_t p = 0; p < np; ++p) total[p] += all[r * (np + 1) + p];
  // pairs that need the whole chunk's counts: more than one batch
  std::vector<size_t> wide;
  for (size_t p = 0; p < nc * nd; ++p)
    if (total[p] > opt_.max_list_length) wide.push_back(p);
  std::vector<std::vector<uint32_t>> chunk_counts(nc * nd);
  if (!wide.empty()) {
    std::vector<uint64_t> sizes(world, 0);
    for (uint32_t r = 0; r < world; ++r)
      for (size_t p : wide) sizes[r] += (rank_lo[p / nd][r + 1] - rank_lo[p / nd][r]) * 4;
    std::vector<uint32_t> send;
    for (size_t p : wide) send.insert(send.end(), mine[p].begin(), mine[p].end());
    if (send.size() * 4 != sizes[rank]) throw Error("shard exchange: slice sizes disagree");
    uint64_t recv_total = 0;
    for (uint64_t s : sizes) recv_total += s;
    std::vector<uint32_t> recv(recv_total / 4);
    gather(send.data(), send.size() * 4, recv.data(), sizes);
    // rank r's block holds its part of every wide pair in order
    uint64_t block = 0;
    for (uint32_t r = 0; r < world; ++r) {
      uint64_t at = block;
      for (size_t p : wide) {
        const uint64_t n = rank_lo[p / nd][r + 1] - rank_lo[p / nd][r];
        chunk_counts[p].insert(chunk_counts[p].end(), recv.begin() + at, recv.begin() + at + n);
        at += n;
      }
      block += sizes[r] / 4;
    }
  }
  for (size_t c = 0; c < nc; ++c) {
    QueryData *q = slice[c];
    if (!q) continue;
    for (size_t di = 0; di < nd; ++di) {
      const size_t p = c * nd + di;
      if (q->plan.size() <= di) {
        q->plan.resize(di + 1);
        q->plan_sum.resize(di + 1);
        q->plan_hash.resize(di + 1);
      }
      if (total[p] > opt_.max_list_length) {
        if (chunk_counts[p].size() != chunk_nseq[c]) throw Error("shard exchange: chunk counts incomplete");
        q->plan[di] = CpuBatches(chunk_counts[p], opt_.max_list_length);
      } else if (total[p] > 0) {
        q->plan[di] = {Batch{0, chunk_nseq[c]}};  // CpuBatches of a chunk within -l
      } else {
        q->plan[di].clear();
      }
      q->plan_sum[di] = sums[p];
      q->plan_hash[di] = CountsHash(mine[p].data(), mine[p].size());
    }
    q->planned = true;
  }
}

std::vector<Batch> Session::Passes(QueryData &q, size_t di, const std::vector<uint32_t> &counts,
                                   uint64_t total) const {
  if (!q.planned) {
    // within -l the rule makes one batch (none without candidates): no scan
    if (total <= opt_.max_list_length)
      return total ? std::vector<Batch>{Batch{0, (uint32_t)counts.size()}} : std::vector<Batch>{};
    return CpuBatches(counts, opt_.max_list_length);
  }
  uint64_t sum = 0;
  for (uint32_t c : counts) sum += c;
  if (di >= q.plan.size() || sum != q.plan_sum[di] || CountsHash(counts.data(), counts.size()) != q.plan_hash[di])
    throw Error("shard session: candidate counts differ from its batch plan");
  const uint32_t lo = q.slice_lo, hi = lo + q.chunk.nseq;
  std::vector<Batch> out;
  for (const Batch &b : q.plan[di])
    out.push_back(Batch{std::clamp(b.q0, lo, hi) - lo, std::clamp(b.q1, lo, hi) - lo});
  return out;
}

// ------------------------------------------------------------------ session
Session::Session(const AlignerOptions &opt, uint32_t shard_rank, uint32_t shard_world, const ShardExchange *ex)
    : opt_(opt) {
  threads_ = HostThreads();
  if (shard_world == 0 || shard_rank >= shard_world) throw std::invalid_argument("shard rank outside the world");
  try {
    Create(shard_rank, shard_world, ex);
  } catch (...) {
    // a throwing constructor runs no destructor: free the resident chunks here
    DeviceModule &dev = DeviceModule::Get();
    for (QueryData &q : queries_) dev.Free(q.dev);
    for (DbData &d : dbs_) dev.Free(d.dev);
    queries_.clear();
    dbs_.clear();
    throw;
  }
}

void Session::Create(uint32_t shard_rank, uint32_t shard_world, const ShardExchange *ex) {
  shard_world_ = shard_world;
  const bool local = shard_world > 1 && ex && ex->fn;  // rank-local reads + exchange
  std::vector<uint32_t> chunk_nseq;
  std::vector<std::vector<uint64_t>> rank_lo;
  if (!local) {
    Load(shard_rank, shard_world, false, &chunk_nseq, &rank_lo);
  } else {
    // a rank whose loading fails still joins the creation header exchange with
    // its error flag set, so every rank fails together instead of its peers
    // waiting in the plan's all-gather for a rank that never comes
    std::string err;
    try {
      Load(shard_rank, shard_world, true, &chunk_nseq, &rank_lo);
    } catch (std::exception &e) {
      err = e.what();
      if (err.empty()) err = "shard session creation failed";
    }
    AgreeOnCreate(shard_rank, shard_world, *ex, err, chunk_nseq, rank_lo);
    PlanExchange(shard_rank, shard_world, *ex, chunk_nseq, rank_lo);
  }
  TraceMark("create_sync");
  DeviceModule::Get().Synchronize();
  TraceMark("uploaded");
  formatter_.reset(new TaskQueue());
}

// Every rank's view of the job must be the same before the plan's all-gather
// sizes its buffers from it: a fixed-size header per rank (ok flag, query
// chunks, DB chunks, queries, a hash of every chunk's size and of the shard
// cuts) is all-gathered first. Any rank's failure or any disagreement throws on
// every rank.
void Session::AgreeOnCreate(uint32_t rank, uint32_t world, const ShardExchange &ex, const std::string &err,
                            const std::vector<uint32_t> &chunk_nseq,
                            const std::vector<std::vector<uint64_t>> &rank_lo) {
  constexpr size_t kWords = 8;
  uint64_t mine[kWords] = {0};
  mine[0] = err.empty() ? 1 : 0;
  if (err.empty()) {
    mine[1] = chunk_nseq.size();
    mine[2] = dbs_.size();
    for (uint32_t n : chunk_nseq) mine[3] += n;
    mine[4] = CountsHash(chunk_nseq.data(), chunk_nseq.size());
    std::vector<uint32_t> cuts;
    for (const std::vector<uint64_t> &lo : rank_lo)
      for (uint64_t x : lo) cuts.push_back((uint32_t)x);
    mine[5] = CountsHash(cuts.data(), cuts.size());
    mine[6] = db_sum_u32_;
    mine[7] = world;
  }
  std::vector<uint64_t> all(world * kWords);
  const std::vector<uint64_t> sizes(world, sizeof(mine));
  if (ex.fn(ex.ctx, mine, sizeof(mine), all.data(), sizes.data()) != 0)
    throw Error("shard exchange (creation header all-gather) failed");
  if (!err.empty()) throw Error(err);
  for (uint32_t r = 0; r < world; ++r) {
    const uint64_t *h = &all[r * kWords];
    if (h[0] != 1) throw Error("shard session: rank " + std::to_string(r) + " failed at creation");
    for (size_t k = 1; k < kWords; ++k)
      if (h[k] != mine[k])
        throw Error("shard session: rank " + std::to_string(r) + " sees a different query/DB set than rank " +
                    std::to_string(rank));
  }
}

// Reads and uploads the query and DB chunks (a rank-local shard: only its own
// slice of the queries) and, for a rank-local shard, returns the chunks' sizes
// and every rank's first query per chunk.
void Session::Load(uint32_t shard_rank, uint32_t shard_world, bool local, std::vector<uint32_t> *chunk_nseq_out,
                   std::vector<std::vector<uint64_t>> *rank_lo_out) {
  std::vector<uint32_t> &chunk_nseq = *chunk_nseq_out;
  std::vector<std::vector<uint64_t>> &rank_lo = *rank_lo_out;
  DeviceModule &dev = DeviceModule::Get();
  TraceMark("create");
  dev.Bind(opt_.device);
  TraceMark("bound");
  // the staged uploads' host copies on the worker pool, 1 MB per piece
  const unsigned copiers = std::max(1u, std::min(threads_, 8u));
  dev.SetHostCopy([copiers](void *dst, const void *src, size_t n) {
    const size_t piece = 1u << 20, pieces = (n + piece - 1) / piece;
    ParallelFor(pieces, copiers, [&](size_t b, size_t e, unsigned) {
      const size_t lo = b * piece, hi = std::min(n, e * piece);
      std::memcpy(static_cast<char *>(dst) + lo, static_cast<const char *>(src) + lo, hi - lo);
    });
  });
  dev.SetHostParallel([copiers](size_t parts, const std::function<void(size_t)> &fn) {
    ParallelFor(parts, copiers, [&](size_t b, size_t e, unsigned) {
      for (size_t k = b; k < e; ++k) fn(k);
    });
  });
  dev.SetMatrix(opt_.matrix.m.data());

  // query chunks: -S start (or 0) .. -L end, as Execute walks them
  // (aligner.cpp:98-204), and every DB chunk; the chunk files are read on
  // parallel threads, then the chunks up to the first missing one are kept
  QueryFile qf(opt_.query_prefix);
  uint32_t id = opt_.start_query_chunk == UINT32_MAX ? 0 : opt_.start_query_chunk;
  uint32_t base = 0;
  for (uint32_t k = 0; k < id && k < qf.division; ++k) {
    std::ifstream f((qf.prefix + "_" + std::to_string(k) + ".inf").c_str(), std::ios::binary);
    uint32_t n = 0;
    if (f) f.read(reinterpret_cast<char *>(&n), 4);
    base += n;
  }
  // chunk `id`, then the following ones up to -L (at least `id` itself)
  uint32_t nq_chunks = 0;
  if ((int64_t)id < (int64_t)qf.division) {
    const uint64_t last = std::min<uint64_t>(opt_.end_query_chunk, (uint64_t)qf.division - 1);
    nq_chunks = (uint32_t)(last >= id ? last - id + 1 : 1);
  }
  DbFile df(opt_.db_prefix);
  const uint32_t nd_chunks = (int64_t)df.division > 0 ? (uint32_t)df.division : 0u;
  std::vector<QueryData> qread(nq_chunks);
  std::vector<QueryChunkIndex> qidx(local ? nq_chunks : 0);
  std::vector<DbData> dread(nd_chunks);
  std::vector<char> qok(nq_chunks, 0), dok(nd_chunks, 0);
  // chunks uploaded here but not (yet) handed to queries_/dbs_ are freed on every
  // exit, the error exits included (a chunk handed over has its handle nulled
  // here; the constructor frees queries_/dbs_ if creation fails later)
  struct Unadopted {
    std::vector<QueryData> &q;
    std::vector<DbData> &d;
    ~Unadopted() {
      DeviceModule &m = DeviceModule::Get();
      for (QueryData &x : q)
        if (x.dev) m.Free(x.dev);
      for (DbData &x : d)
        if (x.dev) m.Free(x.dev);
    }
  } unadopted{qread, dread};
  // (each query chunk's name groups and WriteOutput lengths are derived on its
  // reading thread too; a rank-local shard only indexes the query chunks here).
  // A DB chunk is uploaded by its reading thread as soon as it is read, one
  // upload at a time (the staging buffers are shared), while the query chunks
  // are still being read (cfg3: the 34 MB DB and index upload took 1.5 ms of a
  // 4.1 ms session create after every read, profiles/r5ad/)
  std::mutex upload_mu;
  // host copies resident on the device are dropped on a thread of their own
  // after creation (unmapping ~40 MB of chunk files took ~0.3 ms per 12.7 MB
  // on the critical path, and under the upload lock)
  std::mutex drop_mu;
  std::vector<std::shared_ptr<const void>> drop;
  auto drop_later = [&](std::shared_ptr<const void> h) {
    std::lock_guard<std::mutex> lock(drop_mu);
    drop.push_back(std::move(h));
  };
  struct DropInBackground {
    std::vector<std::shared_ptr<const void>> &d;
    ~DropInBackground() {
      if (d.empty()) return;
      try {
        std::thread([h = std::move(d)]() mutable { h.clear(); }).detach();
      } catch (...) {
        d.clear();  // no thread: drop them here
      }
    }
  } drop_in_background{drop};
  auto upload_db = [&](DbData &d) {
    {
      std::lock_guard<std::mutex> lock(upload_mu);
      const DbChunk &c = d.chunk;
      d.dev = dev.UploadDb(c.seq.data(), c.len, c.keys_count.data(), c.kcl, c.positions.data(), c.npos);
      if (c.nseq) dev.SetDbSubjects(d.dev, c.starts.data(), c.nseq);
    }
    // resident on the device from here; the host keeps names and starts
    drop_later(d.chunk.seq.Detach());
    drop_later(d.chunk.keys_count.Detach());
    drop_later(d.chunk.positions.Detach());
  };
  auto upload_query = [&](QueryData &q) {
    std::lock_guard<std::mutex> lock(upload_mu);
    q.dev = dev.UploadQuery(q.chunk.seq.data(), q.chunk.nseq, q.chunk.L);
    dev.SetQueryGroups(q.dev, q.group_first.data(), q.group_last.data(), (uint32_t)q.group_first.size());
  };
  ParallelFor(nq_chunks + nd_chunks, std::max<unsigned>(1u, std::min(threads_, 8u)),
              [&](size_t b0, size_t e0, unsigned) {
                // DB chunks first (they are listed after the query chunks)
                for (size_t j = b0; j < e0; ++j) {
                  const size_t k = nq_chunks + nd_chunks - 1 - j;
                  if (k < nq_chunks && local) {
                    qok[k] = qf.IndexChunk(id + (uint32_t)k, &qidx[k]);
                  } else if (k < nq_chunks) {
                    qok[k] = qf.ReadChunk(id + (uint32_t)k, &qread[k].chunk);
                    if (qok[k]) PrepareQueryChunk(&qread[k], false);
                    TraceMark("q_chunk_read", k);
                    // an unsharded session uploads the chunk here too (a sharded
                    // one keeps only its slice, below)
                    if (qok[k] && shard_world == 1) {
                      upload_query(qread[k]);
                      TraceMark("q_chunk_up", k);
                    }
                  } else {
                    DbData &d = dread[k - nq_chunks];
                    dok[k - nq_chunks] = df.ReadChunk((uint32_t)(k - nq_chunks), &d.chunk);
                    TraceMark("db_chunk_read", k - nq_chunks);
                    if (dok[k - nq_chunks]) upload_db(d);
                    TraceMark("db_chunk_up", k - nq_chunks);
                  }
                }
              });
  uint32_t nchunks = 0;
  while (nchunks < nq_chunks && qok[nchunks]) ++nchunks;
  if (nchunks == 0) throw std::runtime_error("[Aligner] error: don't find query file.");
  if (!local) {
    std::vector<QueryData *> chunks;
    for (uint32_t k = 0; k < nchunks; ++k) chunks.push_back(&qread[k]);
    QueryLengths(chunks);
  }
  TraceMark("queries_read", nchunks);

  db_sum_u32_ = (uint32_t)df.sum_length;
  uint32_t dbase = 0;
  uint32_t nd_kept = 0;
  for (; nd_kept < nd_chunks && dok[nd_kept]; ++nd_kept) {
    dread[nd_kept].global_base = dbase;
    dbase += dread[nd_kept].chunk.nseq;
    dbs_.push_back(std::move(dread[nd_kept]));
    dread[nd_kept].dev = nullptr;
  }
  // chunks read past a missing one are not used (freed by `unadopted`)
  if (dbs_.empty()) throw std::runtime_error("[Aligner] error: don't find db file.");
  TraceMark("db_read", dbs_.size());
  {
    std::vector<uint32_t> bases;
    for (const DbData &d : dbs_) bases.push_back(d.global_base);
    // DB chunk ids are the indices into dbs_ (chunks are read from 0 in order)
    for (size_t k = 0; k < dbs_.size(); ++k)
      if (dbs_[k].chunk.id != k) throw Error("DB chunk ids out of order");
    dev.SetChunkBases(bases.data(), (uint32_t)bases.size());
    TraceMark("bases_set");
  }

  if (local) {
    // the cut over every selected query from the chunk indices, then only this
    // rank's rows and names are read
    std::vector<uint32_t> weight;
    std::vector<uint8_t> start;
    for (uint32_t k = 0; k < nchunks; ++k) {
      weight.insert(weight.end(), qidx[k].qlen.begin(), qidx[k].qlen.end());
      start.insert(start.end(), qidx[k].group_start.begin(), qidx[k].group_start.end());
    }
    std::vector<uint64_t> cuts(shard_world + 1);
    ShardCuts(weight.size(), weight.data(), start.data(), shard_world, cuts.data());
    shard_begin_ = cuts[shard_rank];
    shard_end_ = cuts[shard_rank + 1];
    std::vector<uint32_t> read;  // chunks holding queries of this rank
    uint64_t at = 0;
    uint32_t cbase = base;
    chunk_nseq.resize(nchunks);
    rank_lo.resize(nchunks);
    for (uint32_t k = 0; k < nchunks; ++k) {
      const uint32_t n = qidx[k].nseq;
      chunk_nseq[k] = n;
      for (uint32_t r = 0; r <= shard_world; ++r)
        rank_lo[k].push_back(std::min<uint64_t>(n, cuts[r] > at ? cuts[r] - at : 0));
      if (rank_lo[k][shard_rank] < rank_lo[k][shard_rank + 1]) {
        qread[k].slice_lo = (uint32_t)rank_lo[k][shard_rank];
        qread[k].chunk_nseq = n;
        qread[k].global_base = cbase + qread[k].slice_lo;
        read.push_back(k);
      }
      at += n;
      cbase += n;
    }
    ParallelFor(read.size(), std::max<unsigned>(1u, std::min(threads_, 8u)), [&](size_t b, size_t e, unsigned) {
      for (size_t j = b; j < e; ++j) {
        const uint32_t k = read[j];
        qidx[k].ReadSlice(qread[k].slice_lo, (uint32_t)(rank_lo[k][shard_rank + 1] - qread[k].slice_lo),
                          &qread[k].chunk);
        PrepareQueryChunk(&qread[k], false);
      }
    });
    {
      std::vector<QueryData *> chunks;
      for (uint32_t k : read) chunks.push_back(&qread[k]);
      QueryLengths(chunks);
    }
    for (uint32_t k : read) {
      queries_.push_back(std::move(qread[k]));
      qread[k].dev = nullptr;
    }
    TraceMark("slices_read", queries_.size());
  } else {
    for (uint32_t k = 0; k < nchunks; ++k) {
      qread[k].global_base = base;
      base += qread[k].chunk.nseq;
      queries_.push_back(std::move(qread[k]));
      qread[k].dev = nullptr;
    }
    if (shard_world > 1) ApplyShard(shard_rank, shard_world);  // may leave no queries
  }

  for (QueryData &q : queries_) {
    if (!q.dev) upload_query(q);  // (uploaded while reading when unsharded)
    drop_later(q.chunk.seq.Detach());  // resident on the device (qlen and names stay on the host)
  }
  TraceMark("queries_released");
  // query chunks read past a missing one are not used (freed by `unadopted`)
}

namespace {
struct MergeItem {
  uint32_t score;
  uint32_t end;       // absolute db end (new) / unused (resolved)
  uint32_t query;     // candidate's own query (frame)
  int32_t from;       // -1: new candidate; else position in the group's old results
};
struct ScoreDesc {
  bool operator()(const MergeItem &a, const MergeItem &b) const { return a.score > b.score; }
};
}  // namespace

// reference Merge (aligner.cpp:687-769): per name group, the batch's candidates
// of each query then its kept results, std::sort by score (unstable), first hit
// per subject traced back, stop at -b. Groups are independent -> host threads.
// Used when a chunk needs several batches or several DB chunks.
void Session::HostMergeBatch(QueryData &q, DbData &d, uint32_t bq0, uint32_t bq1,
                             uint64_t cand_begin, const uint32_t *score, const uint32_t *end,
                             const std::vector<uint32_t> &counts, const std::vector<uint64_t> &offsets,
                             Results *results) {
  const uint32_t ng = (uint32_t)q.group_first.size();
  const uint64_t epoch = ++merge_epoch_;
  const uint32_t nsubj = d.chunk.nseq;
  struct Pending {
    uint32_t id, pos;
  };
  std::vector<std::vector<Pending>> pending(threads_);
  ParallelFor(ng, threads_, [&](size_t gb, size_t ge, unsigned t) {
    std::vector<uint64_t> owner(nsubj, ~0ull);
    std::vector<MergeItem> l;
    std::vector<HitRecord> old;
    for (size_t g = gb; g < ge; ++g) {
      const uint32_t gs = q.group_first[g], gend = q.group_last[g] + 1, id = gend - 1;
      l.clear();
      old.clear();
      for (uint32_t i = gs; i < gend; ++i) {
        if (i >= bq0 && i < bq1) {
          const uint64_t b = offsets[i] - cand_begin;
          for (uint32_t k = 0; k < counts[i]; ++k)
            l.push_back(MergeItem{score[b + k], end[b + k], i, -1});
        }
        for (HitRecord &h : (*results)[i]) {
          l.push_back(MergeItem{h.score, 0, h.query, (int32_t)old.size()});
          old.push_back(h);
        }
        (*results)[i].clear();
      }
      if (l.empty()) continue;
      std::sort(l.begin(), l.end(), ScoreDesc());
      std::vector<HitRecord> &out = (*results)[id];
      const uint64_t tag = (epoch << 32) | id;
      for (const MergeItem &it : l) {
        if (it.from >= 0) {
          out.push_back(old[it.from]);
        } else {
          const uint32_t sid = d.chunk.SubjectOf(it.end);
          if (sid >= nsubj) throw Error("candidate end outside the database");
          if (owner[sid] != tag) {
            owner[sid] = tag;
            HitRecord h;
            h.query = it.query;
            h.db_chunk = d.chunk.id;
            h.subject = sid;
            h.score = it.score;
            h.end = it.end;          // absolute until the traceback
            h.start = UINT32_MAX;
            pending[t].push_back(Pending{id, (uint32_t)out.size()});
            out.push_back(h);
          }
        }
        if (out.size() >= opt_.best) break;
      }
    }
  });

  // K3 for every newly selected hit of this batch, then rebase to the subject
  std::vector<Pending> all;
  for (auto &p : pending) all.insert(all.end(), p.begin(), p.end());
  const uint32_t nh = (uint32_t)all.size();
  if (nh == 0) return;
  std::vector<uint32_t> qid(nh), e(nh), st(nh), len(nh), mt(nh);
  std::vector<float> sid(nh);
  for (uint32_t k = 0; k < nh; ++k) {
    const HitRecord &h = (*results)[all[k].id][all[k].pos];
    qid[k] = h.query;
    e[k] = h.end;
  }
  const uint32_t tb_base = q.chunk.L + 2 * opt_.extend * 2 * (1u << opt_.log_region);
  DeviceModule::Get().TraceBack(q.dev, d.dev, nh, qid.data(), e.data(), tb_base, opt_.open_gap,
                                opt_.extend_gap, st.data(), len.data(), mt.data(), sid.data());
  stats_.tracebacks += nh;
  for (uint32_t k = 0; k < nh; ++k) {
    HitRecord &h = (*results)[all[k].id][all[k].pos];
    const uint32_t pos = d.chunk.starts[h.subject];
    h.start = st[k] - pos;
    h.end = h.end - pos;
    h.aln_len = len[k];
    h.aln_match = mt[k];
    h.seq_id = sid[k];
  }
}

// Device path, one pass per (DB chunk, batch): the chunk's groups are cut into
// segments of ~kSegmentCands of the batch's candidates (at group boundaries, so
// every group's candidates stay together as in the reference batch); per
// segment K2 -> K4 -> K3 run on the GPU. K4 merges each group's candidates with
// the result list carried from the earlier passes (the reference Merge over
// result_list, aligner.cpp:687-769, called for every batch of every DB chunk,
// aligner.cpp:118-174); in the final pass the segment's text is formatted by the
// background worker while the GPU works on the next one.
void Session::DevicePass(QueryData &q, DbData &d, const std::vector<uint32_t> &counts,
                         const std::vector<uint64_t> &offsets, uint32_t bq0, uint32_t bq1, uint64_t c_lo,
                         uint64_t c_hi, bool carry_in, bool final_pass) {
  DeviceModule &dev = DeviceModule::Get();
  GapConfig gap;
  gap.extend = opt_.extend;
  gap.log_region = opt_.log_region;
  gap.open = opt_.open_gap;
  gap.ext = opt_.extend_gap;
  const uint32_t base = q.chunk.L + 2 * opt_.extend + 2 * (1u << opt_.log_region);
  const uint32_t tb_base = q.chunk.L + 2 * opt_.extend * 2 * (1u << opt_.log_region);
  const uint32_t cap = std::max<uint32_t>(opt_.best, 1);
  // segments of ~16M candidates (fewer host round trips per step);
  // GHOSTM_SEGMENT_CANDS / GHOSTM_TAIL_CANDS shrink them so that small test
  // datasets run the many-segment pipeline of the full-size workloads
  // The tail floor is 1 M candidates, or a quarter of a smaller batch, so a
  // batch of under ~2 M candidates is still cut into three segments whose
  // formatting overlaps the next one's K2 (cfg2's 0.9 M: 10.2 -> 8.7 ms per
  // step; at cfg3 and the 125 K shard a smaller floor only adds launches,
  // profiles/r4_tail_sweep.txt)
  // The floor's cap counts the last segment's formatting, which grows with its
  // queries, not its candidates: 1 M candidates or 16 K queries' worth,
  // whichever is more (dense batches, 127 per query: ~2 M; cfg4 351.1 -> 350.5
  // ms, the 125 K shard 46.7 -> 46.4 ms; cfg3's 63 per query keeps ~1 M: 2 M
  // lost 0.5 ms there, profiles/r5aj/, profiles/r5ai/)
  const uint64_t batch_q = bq1 > bq0 ? bq1 - bq0 : 1;
  const uint64_t tail_cap = std::max<uint64_t>(1ull << 20, (c_hi - c_lo) / batch_q * 16384);
  uint64_t kSegmentCands = 16ull << 20;
  uint64_t kTailCands = std::min<uint64_t>(tail_cap, std::max<uint64_t>(1ull << 17, (c_hi - c_lo) / 4));
  if (const char *e = getenv("GHOSTM_SEGMENT_CANDS")) kSegmentCands = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
  if (const char *e = getenv("GHOSTM_TAIL_CANDS")) kTailCands = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
  // the first segment's K2 tasks are built while the GPU waits (the later
  // ones during the previous K2): a head of at most kHeadCands shortens that
  // wait (GHOSTM_HEAD_CANDS; 0 = no head cap). At >= 96 candidates per query the
  // unit kernel's consecutive tasks need no count pass (score_tasks.h) and the
  // build is short (0.04 ms for the 125 K-query shard's first 1 M): no head
  // there, one segment fewer (shard 46.5-46.8 against 46.7-47.5 ms with it,
  // profiles/r5t/)
  uint64_t kHeadCands = (c_hi - c_lo) / batch_q >= 96 ? 0 : kTailCands;
  if (const char *e = getenv("GHOSTM_HEAD_CANDS")) kHeadCands = strtoull(e, nullptr, 10);
  const uint32_t ng = (uint32_t)q.group_first.size();
  // a group's first candidate of this batch (groups outside it have none)
  auto group_begin = [&](uint32_t g) { return std::min(std::max(offsets[q.group_first[g]], c_lo), c_hi); };
  auto group_of = [&](uint32_t qi) {
    return (uint32_t)(std::upper_bound(q.group_first.begin(), q.group_first.end(), qi) - q.group_first.begin()) - 1;
  };
  // the batch's groups [gb0, gb1) (a batch may cut a name group); the groups
  // before and after it have no new candidates
  const uint32_t gb0 = bq1 > bq0 ? group_of(bq0) : 0, gb1 = bq1 > bq0 ? group_of(bq1 - 1) + 1 : 0;
  // segment cuts (group ranges) first, so each segment's K2 tasks can be built
  // on the host while the previous segment's K2 runs
  std::vector<std::pair<uint32_t, uint32_t>> cuts;
  const uint32_t kIdleGroups = 1u << 17;  // groups per segment without candidates
  auto idle = [&](uint32_t from, uint32_t to) {
    for (uint32_t g = from; g < to; g += kIdleGroups) cuts.emplace_back(g, std::min(to, g + kIdleGroups));
  };
  idle(0, gb0);
  for (uint32_t g0 = gb0; g0 < gb1;) {
    const uint64_t rem = c_hi - group_begin(g0);  // candidates from g0 to the batch's end
    // full segments, then shrinking ones (3/5 of what is left, down to
    // kTailCands): each segment's GPU time (~3.5 ms per 1 M candidates) covers
    // the text formatting of the one before it (~1.4 ms per 1 M), so little of
    // the formatting is left when the GPU finishes
    // (a carried pass formats nothing: full segments only)
    uint64_t target = rem > 2 * kSegmentCands || !final_pass ? kSegmentCands
                                                              : std::max<uint64_t>(kTailCands, rem * 3 / 5);
    if (g0 == gb0 && kHeadCands && rem > 2 * kHeadCands) target = std::min(target, kHeadCands);
    // the first group g1 > g0 at least `target` candidates on (group_begin
    // does not decrease with g: a binary search, not a walk over the groups)
    const uint64_t from = group_begin(g0);
    uint32_t lo = g0 + 1, hi = gb1;
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo) / 2;
      if (group_begin(mid) - from < target) lo = mid + 1;
      else hi = mid;
    }
    const uint32_t g1 = lo;
    cuts.emplace_back(g0, g1);
    g0 = g1;
  }
  idle(gb1, ng);
  TraceMark("cuts", cuts.size());
  std::vector<DeviceModule::ScoreSegment> segs;
  for (const auto &c : cuts) {
    const uint64_t c0 = group_begin(c.first), c1 = c.second < ng ? group_begin(c.second) : c_hi;
    segs.push_back({c0, c1 - c0, q.group_first[c.first], q.group_last[c.second - 1] + 1});
  }
  MergePass pass;
  pass.cand_lo = c_lo;
  pass.cand_hi = c_hi;
  pass.carry_in = carry_in;
  pass.carry_out = !final_pass;
  pass.chunk = d.chunk.id;
  // Pipeline, per segment k: K2(k) is enqueued first; then segment k-1's
  // selection (its K4/K3 finished before K2(k) started) is copied back on the
  // copy stream, turned into records and handed to the formatter while K2(k)
  // runs; then K4/K3(k) are enqueued behind K2(k) (after K2 finishes when its
  // guard list needs re-scoring first). The GPU never waits for the host
  // between segments.
  struct Pending {
    uint32_t g0 = 0, g1 = 0;
    bool active = false, identity = false;
  } pending;
  auto finish_pending = [&] {
    if (!pending.active) return;
    pending.active = false;
    const uint32_t g0 = pending.g0;
    auto sel_counts = std::make_shared<std::vector<uint32_t>>();
    auto sel_hits = std::make_shared<HostHits>();
    const double t0 = NowSeconds();
    dev.MergeCollect(sel_counts.get(), final_pass ? sel_hits.get() : nullptr);
    stats_.seconds_merge += NowSeconds() - t0;
    TraceMark("merge_done", pending.g1 - g0);
    if (!final_pass) return;
    dev.AppendRecords(q.dev, g0, *sel_counts, cap, q.global_base, false);
    Part *part = NewPart();
    const QueryData *qp = &q;
    TraceMark("records", g0);
    formatter_->Submit([this, qp, g0, sel_counts, sel_hits, cap, part] {
      const double t = NowSeconds();
      TraceMark("fmt_begin", g0);
      FormatSelected(*qp, g0, *sel_counts, *sel_hits, cap, part);
      stats_.seconds_output += NowSeconds() - t;
      TraceMark("fmt_end", g0);
      PartDone(part);
    });
  };
  struct DeferNext {  // ScorePrepareNext below builds each next segment's tasks
    DeviceModule &dev;
    explicit DeferNext(DeviceModule &d) : dev(d) { dev.ScoreDeferNext(true); }
    ~DeferNext() { dev.ScoreDeferNext(false); }
  } defer_next{dev};
  for (size_t k = 0; k < cuts.size(); ++k) {
    const uint32_t g0 = cuts[k].first, g1 = cuts[k].second;
    const uint64_t c0 = segs[k].cand_begin, c1 = c0 + segs[k].n;
    // nothing to merge: no candidates and nothing carried (the carry of these
    // groups is still the empty list ResetCarry left). Groups without new
    // candidates keep their carried list as it is when -b <= 16: it is sorted
    // by score, std::sort of <= 16 elements is a stable insertion sort, and
    // carried entries are all taken (aligner.cpp:719-721); in the final pass
    // their lists are printed straight from the carry
    const bool identity = c1 == c0 && carry_in && opt_.best <= 16;
    const bool work = c1 > c0 || (carry_in && !identity);
    TraceMark("seg", k);
    if (c1 > c0)
      dev.ScoreLaunch(q.dev, d.dev, c0, c1 - c0, segs[k].q_first, segs[k].q_end, counts, offsets, base, gap,
                      k + 1 < segs.size() ? &segs[k + 1] : nullptr);
    finish_pending();  // segment k - 1, while K2(k) runs
    const bool guarded = dev.ScoreGuarded();
    if (work && !guarded) {
      dev.MergeLaunch(q.dev, d.dev, g0, g1, c0, c1 - c0, opt_.best, tb_base, opt_.open_gap, opt_.extend_gap, pass);
      pending = Pending{g0, g1, true, false};
    }
    // segment k + 1's K2 tasks, while K2(k) and K4/K3(k) run
    dev.ScorePrepareNext(counts, offsets);
    dev.ScoreFinish();
    TraceMark("score_done", c1 - c0);
    if (work && guarded) {
      dev.MergeLaunch(q.dev, d.dev, g0, g1, c0, c1 - c0, opt_.best, tb_base, opt_.open_gap, opt_.extend_gap, pass);
      pending = Pending{g0, g1, true, false};
    }
    stats_.segments += 1;
    if (work || !final_pass) continue;
    // no K4 for these groups: their lists come straight from the carry (or are
    // empty), formatted in order behind the pending segment's
    finish_pending();
    auto sel_counts = std::make_shared<std::vector<uint32_t>>();
    auto sel_hits = std::make_shared<HostHits>();
    if (identity) {
      dev.CarryToHost(q.dev, g0, g1, cap, sel_counts.get(), sel_hits.get());
      dev.AppendRecords(q.dev, g0, *sel_counts, cap, q.global_base, true);
    } else {
      sel_counts->assign(g1 - g0, 0);
    }
    Part *part = NewPart();
    const QueryData *qp = &q;
    formatter_->Submit([this, qp, g0, sel_counts, sel_hits, cap, part] {
      const double t = NowSeconds();
      FormatSelected(*qp, g0, *sel_counts, *sel_hits, cap, part);
      stats_.seconds_output += NowSeconds() - t;
      PartDone(part);
    });
  }
  finish_pending();
}

void Session::RunQueryChunk(QueryData &q) {
  DeviceModule &dev = DeviceModule::Get();
  SeedConfig sc;
  sc.threshold = opt_.threshold;
  sc.shift = opt_.shift;
  sc.log_region = opt_.log_region;
  // K1's per-query counts and offsets: session buffers, reused by every chunk
  // and run (a fresh vector's zero-fill and first-touch faults sat before K1's
  // first kernel: 6 MB per cfg4 chunk)
  std::vector<uint32_t> &counts = seed_counts_;
  std::vector<uint64_t> &offsets = seed_offsets_;
  // the device merge needs every DB chunk's subject table; GHOSTM_MERGE=host
  // keeps the host merge (tests)
  bool device_merge = true;
  for (const DbData &d : dbs_) device_merge = device_merge && d.chunk.nseq > 0;
  if (const char *e = getenv("GHOSTM_MERGE")) device_merge = device_merge && strcmp(e, "host") != 0;
  if (!device_merge) {
    RunQueryChunkHostMerge(q);
    return;
  }
  const uint32_t cap = std::max<uint32_t>(opt_.best, 1);
  dev.ResetCarry(q.dev, cap);
  if (run_sync_) dev.Synchronize();  // (see Run)
  TraceMark("carry_idle");
  bool carry = false, formatted = false;
  for (size_t di = 0; di < dbs_.size(); ++di) {
    DbData &d = dbs_[di];
    sc.seed_mask = d.chunk.seed;
    TraceMark("seed", q.chunk.nseq);
    const uint64_t total = dev.Seed(q.dev, d.dev, sc, &counts, &offsets);
    stats_.candidates += total;
    TraceMark("seed_done", total);
    // (a shard replays the unsharded run's batches; those that miss its
    // queries are passes without candidates over its carried lists)
    const std::vector<Batch> batches = Passes(q, di, counts, total);
    TraceMark("batches", batches.size());
    for (size_t bi = 0; bi < batches.size(); ++bi) {
      const Batch &b = batches[bi];
      const uint64_t c0 = b.q0 < counts.size() ? offsets[b.q0] : total;
      const uint64_t c1 = b.q1 < counts.size() ? offsets[b.q1] : total;
      const bool final_pass = di + 1 == dbs_.size() && bi + 1 == batches.size();
      DevicePass(q, d, counts, offsets, b.q0, b.q1, c0, c1, carry, final_pass);
      carry = true;
      formatted = final_pass;
      stats_.batches += 1;
    }
  }
  if (!formatted) {
    // the last DB chunk had no batch: the carried lists are the results
    auto sel_counts = std::make_shared<std::vector<uint32_t>>();
    auto sel_hits = std::make_shared<HostHits>();
    dev.CarryToHost(q.dev, 0, (uint32_t)q.group_first.size(), cap, sel_counts.get(), sel_hits.get());
    records_on_device_ = false;  // records are uploaded from the host on demand
    Part *part = NewPart();
    const QueryData *qp = &q;
    formatter_->Submit([this, qp, sel_counts, sel_hits, cap, part] {
      const double t = NowSeconds();
      FormatSelected(*qp, 0, *sel_counts, *sel_hits, cap, part);
      stats_.seconds_output += NowSeconds() - t;
      PartDone(part);
    });
  }
}

// Host merge (GHOSTM_MERGE=host, or a DB chunk without subjects): every batch's
// scores come back to the host and HostMergeBatch applies the reference Merge.
void Session::RunQueryChunkHostMerge(QueryData &q) {
  DeviceModule &dev = DeviceModule::Get();
  SeedConfig sc;
  sc.threshold = opt_.threshold;
  sc.shift = opt_.shift;
  sc.log_region = opt_.log_region;
  GapConfig gap;
  gap.extend = opt_.extend;
  gap.log_region = opt_.log_region;
  gap.open = opt_.open_gap;
  gap.ext = opt_.extend_gap;
  const uint32_t base = q.chunk.L + 2 * opt_.extend + 2 * (1u << opt_.log_region);
  std::vector<uint32_t> counts;
  std::vector<uint64_t> offsets;
  std::vector<uint32_t> score, end;
  Results results(q.chunk.nseq);
  records_on_device_ = false;  // host merge: records are uploaded on demand
  for (size_t di = 0; di < dbs_.size(); ++di) {
    DbData &d = dbs_[di];
    sc.seed_mask = d.chunk.seed;
    const uint64_t total = dev.Seed(q.dev, d.dev, sc, &counts, &offsets);
    stats_.candidates += total;
    const std::vector<Batch> batches = Passes(q, di, counts);
    TraceMark("batches", batches.size());
    for (const Batch &b : batches) {
      const uint64_t c0 = b.q0 < counts.size() ? offsets[b.q0] : total;
      const uint64_t c1 = b.q1 < counts.size() ? offsets[b.q1] : total;
      const uint64_t nc = c1 - c0;
      score.resize(nc);
      end.resize(nc);
      if (nc) dev.Score(q.dev, d.dev, c0, nc, b.q0, b.q1, counts, offsets, base, gap, score.data(), end.data());
      const double t0 = NowSeconds();
      HostMergeBatch(q, d, b.q0, b.q1, c0, score.data(), end.data(), counts, offsets, &results);
      stats_.seconds_merge += NowSeconds() - t0;
      stats_.batches += 1;
    }
  }
  formatter_->Drain();
  const double t1 = NowSeconds();
  Part *part = NewPart();
  FormatResults(q, results, part);
  PartDone(part);
  stats_.seconds_output += NowSeconds() - t1;
}

// ------------------------------------------------------------------ output
namespace {
// two-digit table for integer formatting
struct Digits {
  char d[200];
  Digits() {
    for (int i = 0; i < 100; ++i) { d[2 * i] = (char)('0' + i / 10); d[2 * i + 1] = (char)('0' + i % 10); }
  }
};
const Digits kDigits;

inline char *PutU32(char *p, uint32_t v) {
  char buf[12];
  char *e = buf + sizeof(buf), *b = e;
  while (v >= 100) {
    const uint32_t r = v % 100;
    v /= 100;
    b -= 2;
    std::memcpy(b, kDigits.d + 2 * r, 2);
  }
  if (v >= 10) {
    b -= 2;
    std::memcpy(b, kDigits.d + 2 * v, 2);
  } else {
    *--b = (char)('0' + v);
  }
  std::memcpy(p, b, (size_t)(e - b));
  return p + (e - b);
}
// ostream << float == printf("%g") == to_chars(general, 6) (checked on 6e8 bit
// patterns incl. NaN/inf/denormals), and to_chars is ~5x faster than snprintf.
inline char *PutFloat(char *p, float f) {
  return std::to_chars(p, p + 48, f, std::chars_format::general, 6).ptr;
}
inline char *PutStr(char *p, std::string_view s) {
  std::memcpy(p, s.data(), s.size());
  return p + s.size();
}
// %g text of at most 15 bytes (every float's fits: "-1.17549e-38" is 12)
inline char *PutFloat15(char *p, float f) {
  return std::to_chars(p, p + 15, f, std::chars_format::general, 6).ptr;
}
constexpr uint32_t kIdLen = 512, kIdMatch = 128;
}  // namespace

// A table of short texts (at most 15 bytes) filled on first use: entry = bytes
// 0..14 the text, byte 15 its length (0: not yet), in two 64-bit atomics (the
// second, holding the length, published last); racing writers store the same
// bytes. A hit copies the 16 bytes straight from the two loaded words into the
// line (which has kFixed bytes of room) and steps on by the length: no reload
// from a stack buffer at an odd offset, which stalled on store forwarding. The
// storage comes zeroed from calloc (the OS's zero pages), so a table costs
// nothing until entries are used: the session's create -> run path no longer
// formats 60 K identity strings up front.
struct TextCache {
  struct Entry {
    std::atomic<uint64_t> a, b;
  };
  Entry *e = nullptr;
  size_t n = 0;
  explicit TextCache(size_t entries) : e(static_cast<Entry *>(std::calloc(entries, sizeof(Entry)))), n(entries) {
    if (!e) throw std::bad_alloc();
  }
  ~TextCache() { std::free(e); }
  TextCache(const TextCache &) = delete;
  TextCache &operator=(const TextCache &) = delete;
  // the text of entry k, made by make(buf) (writes at most 15 bytes, returns its end) on first use
  template <class F>
  char *Put(char *p, size_t k, F make) const {
    Entry &c = e[k];
    uint64_t w[2];
    w[1] = c.b.load(std::memory_order_acquire);
    if ((w[1] >> 56) == 0) {
      char buf[16] = {0};
      buf[15] = (char)(make(buf) - buf);
      std::memcpy(w, buf, 16);
      c.a.store(w[0], std::memory_order_relaxed);
      c.b.store(w[1], std::memory_order_release);
    } else {
      w[0] = c.a.load(std::memory_order_relaxed);
    }
    std::memcpy(p, w, 16);
    return p + (w[1] >> 56);
  }
};

// One output line, WriteOutput / V1 / V2 (aligner.cpp:951-1012). Everything that
// depends only on the score (bits, exp(-lambda*s)), only on (len, matches) (the
// identity) or only on (query length, score) (the E-value: search space = qlen x
// the DB's residue sum) is formatted once per session, by whichever formatter
// thread needs it first (TextCache); the arithmetic is the reference's float /
// double steps.
struct LineFormat {
  int style = 0;
  EvalueCalculator ev;
  std::vector<double> expd;           // per score: exp(-1.0 * s * lambda)
  static constexpr uint32_t kEvScores = 4096;
  std::unique_ptr<TextCache> bits_txt;  // per score
  std::unique_ptr<TextCache> id_txt;    // per (len, match): 100*id (style 0) or id (style 2)
  std::unique_ptr<TextCache> ev_txt;    // per (query length, score)

  LineFormat(int st, const KarlinParams &k, uint32_t max_score) : style(st), ev(k) {
    if (style == 0) {
      expd.resize(max_score + 1);
      for (uint32_t sc = 0; sc <= max_score; ++sc) expd[sc] = exp(static_cast<double>(-1.0 * (int)sc * ev.p.lambda));
      bits_txt.reset(new TextCache(max_score + 1));
      ev_txt.reset(new TextCache((size_t)(kMaxQueryLength + 1) * kEvScores));
    }
    if (style != 1) id_txt.reset(new TextCache((size_t)kIdLen * kIdMatch));
  }
  float Id(uint32_t len, uint32_t m) const {
    const float id = (float)m / (float)len;  // aligner.cpp:945
    return style == 0 ? id * 100 : id;
  }
  char *PutId(char *p, uint32_t len, uint32_t m) const {
    if (len < kIdLen && m < kIdMatch && m <= len && len > 0)
      return id_txt->Put(p, (size_t)len * kIdMatch + m, [&](char *b) { return PutFloat15(b, Id(len, m)); });
    return PutFloat(p, Id(len, m));
  }
  // the E-value (float)((double)scaled * exp(-lambda * score)), as %g text
  char *PutEvalue(char *p, uint32_t qlen, uint32_t score, float scaled) const {
    const double e = score < expd.size() ? expd[score] : exp(static_cast<double>(-1.0 * (int)score * ev.p.lambda));
    if (qlen > kMaxQueryLength || score >= kEvScores || !ev_txt) return PutFloat(p, (float)((double)scaled * e));
    return ev_txt->Put(p, (size_t)qlen * kEvScores + score, [&](char *b) { return PutFloat15(b, (float)((double)scaled * e)); });
  }
  char *PutBits(char *p, uint32_t score) const {
    if (bits_txt && score < bits_txt->n)
      return bits_txt->Put(p, score, [&](char *b) { return PutFloat15(b, ev.Bits((int)score)); });
    return PutFloat(p, ev.Bits((int)score));
  }
  // bytes a line can take beyond the two names
  static constexpr size_t kFixed = 160;
  // scaled = (float)search_space * K, per query of non-X length qlen
  char *Write(char *p, std::string_view qname, std::string_view sname, uint32_t score, uint32_t start,
              uint32_t end, uint32_t len, uint32_t match, float scaled, uint32_t qlen) const {
    p = PutStr(p, qname);
    *p++ = '\t';
    p = PutStr(p, sname);
    *p++ = '\t';
    if (style == 1) {
      p = PutU32(p, score); *p++ = '\t';
      p = PutU32(p, start + 1); *p++ = '\t';
      p = PutU32(p, end + 1);
    } else if (style == 2) {
      p = PutU32(p, score); *p++ = '\t';
      p = PutU32(p, start + 1); *p++ = '\t';
      p = PutU32(p, end + 1); *p++ = '\t';
      p = PutId(p, len, match); *p++ = '\t';
      p = PutU32(p, len); *p++ = '\t';
      p = PutU32(p, match);
    } else {
      p = PutId(p, len, match); *p++ = '\t';
      p = PutU32(p, len); *p++ = '\t';
      p = PutU32(p, match); *p++ = '\t';
      p = PutU32(p, start + 1); *p++ = '\t';
      p = PutU32(p, end + 1); *p++ = '\t';
      p = PutEvalue(p, qlen, score, scaled); *p++ = '\t';
      p = PutBits(p, score); *p++ = '\t';
    }
    *p++ = '\n';
    return p;
  }
};

namespace {
// Appends lines through a raw cursor into a std::string that grows in chunks.
struct TextCursor {
  std::string &s;
  size_t used;
  explicit TextCursor(std::string &str) : s(str), used(str.size()) {}
  char *Reserve(size_t need) {
    if (s.size() < used + need) s.resize(std::max(used + need, s.size() * 2 + 4096));
    return &s[used];
  }
  void Commit(char *end) { used = (size_t)(end - s.data()); }
  ~TextCursor() { s.resize(used); }
};
}  // namespace

// pieces per formatting worker in a streamed run (GHOSTM_STREAM_PIECES, A/B;
// 1 = the part's pieces as in a run without a file)
static size_t StreamPiecesPerWorker() {
  static const size_t v = [] {
    const char *e = getenv("GHOSTM_STREAM_PIECES");
    return e ? (size_t)std::max(1, atoi(e)) : (size_t)4;
  }();
  return v;
}

const LineFormat &Session::Format() {
  if (!format_) format_.reset(new LineFormat(opt_.output_style, opt_.karlin, 4095));
  return *format_;
}

void Session::Part::Reset(size_t pieces) {
  text.resize(pieces);
  hits.resize(pieces);
  for (std::string &t : text) t.clear();
  for (std::vector<GhostmHit> &h : hits) h.clear();
  std::lock_guard<std::mutex> lk(mu);
  done.assign(pieces, 0);
  abandoned = false;
  streaming = false;
}

void Session::Part::MarkDone(size_t k) {
  {
    std::lock_guard<std::mutex> lk(mu);
    done[k] = 1;
  }
  cv.notify_all();
}

void Session::Part::Abandon() {
  {
    std::lock_guard<std::mutex> lk(mu);
    abandoned = true;
  }
  cv.notify_all();
}

bool Session::Part::Wait(size_t k) {
  std::unique_lock<std::mutex> lk(mu);
  cv.wait(lk, [&] { return done[k] || abandoned; });
  return done[k] != 0;
}

Session::Part *Session::NewPart() {
  if (used_parts_ == parts_.size()) parts_.emplace_back();
  return &parts_[used_parts_++];
}

void Session::FormatResults(const QueryData &q, const Results &results, Part *out) {
  const uint32_t n = q.chunk.nseq;
  out->Reset(threads_);
  const LineFormat &w = Format();
  ParallelFor(n, threads_, [&](size_t b, size_t e, unsigned t) {
    TextCursor text(out->text[t]);
    std::vector<GhostmHit> &hits = out->hits[t];
    for (size_t i = b; i < e; ++i) {
      const uint64_t space = (uint64_t)q.qlen[i] * (uint64_t)db_sum_u32_;
      const float scaled = (float)space * w.ev.p.K;
      const std::string_view qname = q.chunk.names[i];
      for (const HitRecord &h : results[i]) {
        const DbData &d = dbs_[h.db_chunk];
        const std::string_view sname = d.chunk.names[h.subject];
        char *p = text.Reserve(qname.size() + sname.size() + LineFormat::kFixed);
        text.Commit(w.Write(p, qname, sname, h.score, h.start, h.end, h.aln_len, h.aln_match, scaled, q.qlen[i]));
        hits.push_back(GhostmHit{q.global_base + (uint32_t)i, d.global_base + h.subject, h.score, h.start,
                                 h.end, h.aln_len, h.aln_match, h.seq_id});
      }
    }
  });
}

// Same text from the device-selected hits: a name group's lines are printed
// under its last query (the reference's result_list[last]).
void Session::FormatSelected(const QueryData &q, uint32_t g0, const std::vector<uint32_t> &counts,
                             const HostHits &hits, uint32_t cap, Part *out) {
  const uint32_t ng = (uint32_t)counts.size();
  const unsigned workers = std::max(1u, threads_ > 1 ? threads_ - 1 : 1u);
  // a streamed run cuts the part into four pieces per worker, formatted in
  // order, and the writer writes each as soon as it and those before it are
  // done (the file then trails the formatting by a piece, not by the part)
  const bool stream = stream_fd_ >= 0;
  const size_t pieces = PieceCount(ng, stream ? (size_t)workers * StreamPiecesPerWorker() : workers);
  out->Reset(pieces);
  struct AbandonOnError {  // a failed formatting releases the writer waiting for its pieces
    Part *p;
    bool armed = true;
    ~AbandonOnError() {
      if (armed) p->Abandon();
    }
  } abandon{out};
  if (stream) StreamPart(out);
  const LineFormat &w = Format();
  // timeline diagnostics: each worker's wall and on-CPU time (a thread that
  // waits for a CPU, e.g. under a cgroup quota, shows wall >> CPU)
  const bool trace = TraceOn();
  std::vector<double> wall(trace ? pieces : 0), cpu(trace ? pieces : 0);  // per piece
  ParallelForPieces(ng, pieces, workers, [&](size_t b, size_t e, unsigned t) {
    const double w0 = trace ? NowSeconds() : 0.0, c0 = trace ? ThreadCpuSeconds() : 0.0;
    struct Done {
      bool on;
      double w0, c0, *wall, *cpu;
      ~Done() {
        if (on) *wall = NowSeconds() - w0, *cpu = ThreadCpuSeconds() - c0;
      }
    } done{trace, w0, c0, trace ? &wall[t] : nullptr, trace ? &cpu[t] : nullptr};
    std::vector<GhostmHit> &ph = out->hits[t];
    size_t nh = 0;
    for (size_t g = b; g < e; ++g) nh += counts[g];
    out->text[t].reserve(nh * 96);
    ph.reserve(nh);
    {
    TextCursor text(out->text[t]);
    for (size_t g = b; g < e; ++g) {
      const uint32_t i = q.group_last[g0 + g];
      const std::string_view name = q.chunk.names[i];
      const uint64_t space = (uint64_t)q.qlen[i] * (uint64_t)db_sum_u32_;
      const float scaled = (float)space * w.ev.p.K;
      for (uint32_t k = 0; k < counts[g]; ++k) {
        const SelectedHit &h = hits[(size_t)g * cap + k];
        const DbData &d = dbs_[h.chunk];
        const uint32_t len = h.ml >> 8, match = h.ml & 0xFFu;
        const float seq_id = (float)match / (float)len;  // aligner.cpp:945
        const std::string_view sname = d.chunk.names[h.sid];
        char *p = text.Reserve(name.size() + sname.size() + LineFormat::kFixed);
        text.Commit(w.Write(p, name, sname, h.score, h.start, h.end, len, match, scaled, q.qlen[i]));
        ph.push_back(GhostmHit{q.global_base + i, d.global_base + h.sid, h.score, h.start, h.end, len, match,
                               seq_id});
      }
    }
    }  // the piece's text is final here (TextCursor trims it)
    if (stream) out->MarkDone(t);
  });
  abandon.armed = false;
  if (trace) {
    double ws = 0, cs = 0, wm = 0;
    for (size_t t = 0; t < pieces; ++t) ws += wall[t], cs += cpu[t], wm = std::max(wm, wall[t]);
    TraceMark("fmt_wall_max_us", (uint64_t)(wm * 1e6));
    TraceMark("fmt_wall_sum_us", (uint64_t)(ws * 1e6));
    TraceMark("fmt_cpu_sum_us", (uint64_t)(cs * 1e6));
  }
}

void Session::Run(bool stream_to_file) {
  DeviceModule &dev = DeviceModule::Get();
  formatter_->Drain();
  if (writer_) writer_->Drain();
  streamed_ = false;
  stream_failed_ = false;
  stream_off_ = 0;
  if (stream_to_file) {
    if (!writer_) writer_ = std::make_unique<TaskQueue>();
    // an unwritable path writes nothing, as the reference's unchecked ofstream
    stream_fd_ = open(opt_.output_file.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  }
  struct CloseStream {  // also on an error: the formatter, then the writer drained, the file closed
    Session *s;
    ~CloseStream() {
      if (s->stream_fd_ < 0) return;
      // a formatting task still running may hand a part to the writer, which
      // must not reach a closed (or reused) descriptor
      try {
        s->formatter_->Drain();
      } catch (...) {
        s->stream_failed_ = true;
      }
      try {
        s->writer_->Drain();
      } catch (...) {
        s->stream_failed_ = true;
      }
      close(s->stream_fd_);
      s->stream_fd_ = -1;
    }
  } close_stream{this};
  dev.ResetTimes();
  stats_ = GhostmStats{};
  merge_epoch_ = 0;
  used_parts_ = 0;
  joined_.clear();
  joined_valid_ = false;
  hits_.clear();
  hits_valid_ = false;
  Format();  // built here, before any formatting task can need it
  dev.ResetRecords(HitCapacity());  // the most records the run can append
  records_on_device_ = true;
  const double t0 = NowSeconds();
  TraceMark("run");
  // Both streams drained at the start of a run and after each chunk's carry
  // reset: without these waits (which find the streams idle, < 0.03 ms) a
  // session's second run waited 10-28 ms before its first K1 kernel
  // (profiles/r5i/). GHOSTM_RUN_SYNC=0 leaves them out (A/B).
  const char *rs = getenv("GHOSTM_RUN_SYNC");
  run_sync_ = !(rs && strcmp(rs, "0") == 0);
  if (run_sync_) dev.Synchronize();
  TraceMark("run_idle");
  for (QueryData &q : queries_) {
    RunQueryChunk(q);
    stats_.queries += q.chunk.nseq;
    for (uint32_t v : q.qlen) stats_.query_residues += v;
  }
  TraceMark("drain");
  formatter_->Drain();
  if (stream_fd_ >= 0) {
    writer_->Drain();
    TraceMark("streamed", stream_off_);
    if (stream_failed_) throw Error("writing " + opt_.output_file + " failed");
    streamed_ = true;
  }
  stats_.seconds_total = NowSeconds() - t0;
  TraceMark("run_end");
  TraceDump();
  const DeviceTimes &dt = dev.times();
  stats_.seconds_seed = dt.seed;
  stats_.seconds_score = dt.score;
  stats_.seconds_traceback = dt.traceback;
  stats_.seconds_traceback_scan = dt.traceback_scan;
  stats_.score_launches = dt.score_launches;
  stats_.score_launches_packed = dt.score_launches_packed;
  stats_.score_launches_half = dt.score_launches_half;
  stats_.traceback_launches = dt.traceback_launches;
  stats_.traceback_launches_key = dt.traceback_launches_key;
  stats_.seed_runs_hash = dt.seed_launches_hash;
  stats_.score_rechecks = dt.score_rechecks;
  stats_.seed_bytes = dt.seed_bytes;
  stats_.seed_list_entries = dt.seed_list_entries;
  stats_.score_cells = dt.score_cells;
  stats_.traceback_cells = dt.traceback_cells;
  stats_.traceback_launches_scan = dt.traceback_launches_scan;
  stats_.traceback_scan_cells = dt.traceback_scan_cells;
  stats_.merge_launches = dt.merge_launches;
  stats_.merge_launches_wave = dt.merge_launches_wave;
  stats_.score_launches_framed = dt.score_launches_framed;
  for (int c = 0; c < 4; ++c) stats_.seed_queries_class[c] = dt.seed_queries_class[c];
  stats_.seed_queries_wide = dt.seed_queries_wide;
  stats_.seed_runs_filter = dt.seed_launches_filter;
  stats_.seed_filter_overflows = dt.seed_filter_overflows;
  stats_.seed_table_full = dt.seed_table_full;
  stats_.seed_compact_redo = dt.seed_compact_redo;
  stats_.score_launches_sparse = dt.score_launches_sparse;
  stats_.traceback_launches_keyframe = dt.traceback_launches_keyframe;
  stats_.score_launches_levels = dt.score_launches_levels;
  stats_.score_launches_swar = dt.score_launches_swar;
  stats_.score_launches_unit = dt.score_launches_unit;
  stats_.score_launches_pair = dt.score_launches_pair;
  stats_.traceback_launches_strips = dt.traceback_launches_strips;
  stats_.traceback_launches_scan_swar = dt.traceback_launches_scan_swar;
  stats_.tracebacks += dt.traced_hits;  // device merge (the host merge counts its own)
  for (size_t k = 0; k < used_parts_; ++k)
    for (const auto &h : parts_[k].hits) stats_.hits += h.size();
}

const std::string &Session::Output() {
  if (!joined_valid_) {
    size_t n = 0;
    for (size_t k = 0; k < used_parts_; ++k)
      for (const std::string &t : parts_[k].text) n += t.size();
    joined_.clear();
    joined_.reserve(n);
    for (size_t k = 0; k < used_parts_; ++k)
      for (const std::string &t : parts_[k].text) joined_.append(t);
    joined_valid_ = true;
  }
  return joined_;
}

const std::vector<GhostmHit> &Session::Hits() {
  if (!hits_valid_) {
    hits_.clear();
    for (size_t k = 0; k < used_parts_; ++k)
      for (const auto &h : parts_[k].hits) hits_.insert(hits_.end(), h.begin(), h.end());
    hits_valid_ = true;
  }
  return hits_;
}

uint64_t Session::HitCapacity() const {
  uint64_t n = 0;  // each name group keeps at most -b hits
  for (const QueryData &q : queries_) n += (uint64_t)q.group_first.size() * std::max<uint32_t>(opt_.best, 1);
  return n;
}

size_t Session::DeviceHits(void *dst, size_t cap) {
  DeviceModule &dev = DeviceModule::Get();
  if (!records_on_device_) {
    const std::vector<GhostmHit> &h = Hits();
    dev.UploadRecords(h.data(), h.size());
    records_on_device_ = true;
  }
  const size_t n = (size_t)dev.RecordCount();
  if (dst && cap) dev.CopyRecords(dst, std::min(n, cap));
  return n;
}

// The writer's task for a streamed part: piece k is written once it is
// formatted (Part::Wait), in order; submitted before the formatting starts, so
// the writer's tasks stay in part order.
void Session::StreamPart(Part *part) {
  part->streaming = true;
  writer_->Submit([this, part] {
    TraceMark("w_begin", stream_off_);
    struct Done {
      const uint64_t &off;
      ~Done() { TraceMark("w_end", off); }
    } done{stream_off_};
    for (size_t k = 0; k < part->text.size(); ++k) {
      if (!part->Wait(k)) return;  // formatting failed: the run throws from the formatter
      const char *p = part->text[k].data();
      size_t left = part->text[k].size();
      while (left && !stream_failed_) {
        const ssize_t w = pwrite(stream_fd_, p, left, (off_t)stream_off_);
        if (w <= 0) {
          stream_failed_ = true;
          break;
        }
        p += w;
        left -= (size_t)w;
        stream_off_ += (uint64_t)w;
      }
    }
  });
}

void Session::PartDone(const Part *part) {
  if (stream_fd_ < 0 || part->streaming) return;  // (a streamed part is written by StreamPart's task)
  writer_->Submit([this, part] {
    TraceMark("w_begin", stream_off_);
    struct Done {
      const uint64_t &off;
      ~Done() { TraceMark("w_end", off); }
    } done{stream_off_};
    for (const std::string &t : part->text) {
      const char *p = t.data();
      size_t left = t.size();
      while (left && !stream_failed_) {
        const ssize_t w = pwrite(stream_fd_, p, left, (off_t)stream_off_);
        if (w <= 0) {
          stream_failed_ = true;
          break;
        }
        p += w;
        left -= (size_t)w;
        stream_off_ += (uint64_t)w;
      }
    }
  });
}

void Session::WriteOutputFile() {
  if (streamed_) return;  // Run(true) wrote it while searching
  TraceMark("write");
  struct Done {
    ~Done() {
      TraceMark("written");
      TraceDump();
    }
  } done;
  // the pieces in output order, written at their offsets by parallel threads
  // (an unwritable path writes nothing, as the reference's unchecked ofstream)
  std::vector<const std::string *> pieces;
  std::vector<uint64_t> at;
  uint64_t total = 0;
  for (size_t k = 0; k < used_parts_; ++k)
    for (const std::string &t : parts_[k].text) {
      if (t.empty()) continue;
      pieces.push_back(&t);
      at.push_back(total);
      total += t.size();
    }
  const int fd = open(opt_.output_file.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return;
  std::vector<char> failed(pieces.size(), 0);
  ParallelFor(pieces.size(), std::max<unsigned>(1u, std::min(threads_, 8u)), [&](size_t b, size_t e, unsigned) {
    for (size_t k = b; k < e; ++k) {
      const char *p = pieces[k]->data();
      size_t left = pieces[k]->size();
      off_t off = (off_t)at[k];
      while (left) {
        const ssize_t w = pwrite(fd, p, left, off);
        if (w <= 0) {
          failed[k] = 1;
          break;
        }
        p += w;
        off += w;
        left -= (size_t)w;
      }
    }
  });
  close(fd);
  for (char f : failed)
    if (f) throw Error("writing " + opt_.output_file + " failed");
}

// defined after LineFormat (a complete type for format_)
Session::~Session() {
  formatter_.reset();
  DeviceModule &dev = DeviceModule::Get();
  for (QueryData &q : queries_) dev.Free(q.dev);
  for (DbData &d : dbs_) dev.Free(d.dev);
}

}  // namespace ghostm
