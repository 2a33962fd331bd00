// index.hip — the `db` formatter's k-mer index built on the GPU.
//
// Reference: DBCreator::ConstructIndex (db_creator.cpp:167-241). For every
// subject longer than the seed span, every window [j, j + span) inside the
// subject without an X gets key = the seed positions' 5-bit codes, first residue
// most significant (Index::GetKey); keys_count is the CSR prefix of the key
// counts (kcl = 32^weight + 1 entries, keys_count[0] = 0) and positions lists
// each key's windows in ascending j (the reference fills them in j order).
//
// On the device, per chunk of len residues (HBM-bound, one pass over the bytes):
//   k_index_keys    one thread per position j: the window test and the key
//                   (sentinel 32^weight = no key), key counts by atomics
//   k_scan_*        in-place inclusive scan of the counts -> keys_count
//   k_rs_*          stable LSD radix sort of the (key, j) pairs, 8-bit digits
//                   over 5*weight + 1 bits: per 4096-element tile a digit
//                   histogram, one scan of the (digit, tile) counts, then each
//                   tile scatters its elements in order (ranks within a wave by
//                   ballot matching of the digit bits, across waves by an LDS
//                   prefix). j ascending within each key, the keyless windows
//                   (sentinel) last, so positions = the first npos values.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <utility>

#include "../../include/ghostm_hip.h"
#include "common.h"
#include "formats.h"

namespace ghostm {

void SetLastErrorMessage(const std::string &m);

namespace {

#define IDX_CHECK(expr)                                                                  \
  do {                                                                                   \
    hipError_t err_ = (expr);                                                            \
    if (err_ != hipSuccess)                                                              \
      throw Error(std::string("HIP error '") + hipGetErrorString(err_) + "' at " #expr); \
  } while (0)

constexpr uint32_t kIdxBlock = 256;
constexpr uint32_t kScanItems = 4;                       // counts per thread in the block scan
constexpr uint32_t kScanTile = kIdxBlock * kScanItems;   // counts per block

// One thread per position j. A window is keyed when it lies inside one subject
// (no END in [j, j + span)), holds no X, and its subject is longer than the span
// (db_creator.cpp:197: a subject of exactly `span` residues contributes nothing,
// i.e. a window that starts the subject and is followed by its END).
__global__ __launch_bounds__(kIdxBlock) void k_index_keys(const uint8_t *seq, uint32_t len, uint32_t seed,
                                                           uint32_t span, uint32_t sentinel, uint32_t *key_at,
                                                           uint32_t *val, uint32_t *counts) {
  const uint32_t j = blockIdx.x * kIdxBlock + threadIdx.x;
  if (j >= len) return;
  val[j] = j;
  uint32_t key = sentinel;
  // the last byte of a chunk is an END, so a keyed window has j + span < len
  if ((uint64_t)j + span < len) {
    bool ok = true;
    uint32_t k = 0, s = seed;
    for (uint32_t t = 0; t < span; ++t, s >>= 1) {
      const uint32_t c = seq[j + t];
      ok = ok && c != kSeqEnd && c != kBaseX;
      if (s & 1u) k = (k << kCharBits) | c;
    }
    if (ok && (j == 0 || seq[j - 1] == kSeqEnd) && seq[j + span] == kSeqEnd) ok = false;
    if (ok) {
      key = k;
      atomicAdd(&counts[k + 1], 1u);
    }
  }
  key_at[j] = key;
}

// Inclusive scan of n counts in place: tiles of kScanTile per block (their sums
// to tile_sum), one block scanning the tile sums, then each tile adds its prefix.
__device__ inline uint32_t BlockInclusiveScan(uint32_t v, uint32_t *s_part) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(v, d);
    if (lane >= d) v += o;
  }
  if (lane == 63) s_part[wave] = v;
  __syncthreads();
  uint32_t add = 0;
  for (uint32_t w = 0; w < wave; ++w) add += s_part[w];
  __syncthreads();
  return v + add;
}

__global__ __launch_bounds__(kIdxBlock) void k_scan_tiles(uint32_t *x, uint32_t n, uint32_t *tile_sum) {
  __shared__ uint32_t s_part[kIdxBlock / 64];
  const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  uint32_t v[kScanItems], sum = 0;
#pragma unroll
  for (uint32_t u = 0; u < kScanItems; ++u) {
    v[u] = base + u < n ? x[base + u] : 0u;
    sum += v[u];
  }
  const uint32_t incl = BlockInclusiveScan(sum, s_part);
  uint32_t run = incl - sum;
#pragma unroll
  for (uint32_t u = 0; u < kScanItems; ++u) {
    run += v[u];
    if (base + u < n) x[base + u] = run;
  }
  if (threadIdx.x == kIdxBlock - 1) tile_sum[blockIdx.x] = incl;
}

// exclusive prefix of the tile sums, in place (one block, any count)
__global__ __launch_bounds__(kIdxBlock) void k_scan_sums(uint32_t *tile_sum, uint32_t ntiles) {
  __shared__ uint32_t s_part[kIdxBlock / 64];
  __shared__ uint32_t s_carry;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (uint32_t b = 0; b < ntiles; b += kIdxBlock) {
    const uint32_t i = b + threadIdx.x;
    const uint32_t v = i < ntiles ? tile_sum[i] : 0u;
    const uint32_t incl = BlockInclusiveScan(v, s_part);
    const uint32_t carry = s_carry;
    if (i < ntiles) tile_sum[i] = carry + incl - v;
    __syncthreads();
    if (threadIdx.x == kIdxBlock - 1) s_carry = carry + incl;
    __syncthreads();
  }
}

__global__ __launch_bounds__(kIdxBlock) void k_scan_add(uint32_t *x, uint32_t n, const uint32_t *tile_prefix) {
  const uint32_t i = blockIdx.x * kIdxBlock + threadIdx.x;
  if (i < n) x[i] += tile_prefix[i / kScanTile];
}

// ---- stable LSD radix sort (key, value), 8-bit digits
constexpr uint32_t kRsBits = 8, kRsDigits = 1u << kRsBits;
constexpr uint32_t kRsWaves = 4, kRsItems = 16;                 // 256 threads, 16 elements each
constexpr uint32_t kRsTile = 64 * kRsItems * kRsWaves;          // elements per tile (block)
static_assert(kIdxBlock == 64 * kRsWaves && kIdxBlock == kRsDigits, "one thread per digit");

// Digit counts of tile t, digit-major: hist[d * ntiles + t].
__global__ __launch_bounds__(kIdxBlock) void k_rs_hist(const uint32_t *key, uint32_t n, uint32_t shift,
                                                        uint32_t ntiles, uint32_t *hist) {
  __shared__ uint32_t s_h[kRsDigits];
  s_h[threadIdx.x] = 0;
  __syncthreads();
  const size_t t0 = (size_t)blockIdx.x * kRsTile;
  for (uint32_t k = threadIdx.x; k < kRsTile; k += kIdxBlock) {
    const size_t i = t0 + k;
    if (i < n) atomicAdd(&s_h[(key[i] >> shift) & (kRsDigits - 1)], 1u);
  }
  __syncthreads();
  hist[(size_t)threadIdx.x * ntiles + blockIdx.x] = s_h[threadIdx.x];
}

// Scatter of tile t in element order. incl = inclusive scan of hist (digit-major),
// so the tile's first slot for digit d is incl[d * ntiles + t] - (tile's count of
// d). Wave w owns elements [t*kRsTile + w*1024, +1024), batch u = 64 consecutive
// ones; a lane's rank among same-digit lanes of a batch comes from the ballots of
// the eight digit bits, the counts of earlier batches from the wave's LDS row.
__global__ __launch_bounds__(kIdxBlock) void k_rs_scatter(const uint32_t *key_in, const uint32_t *val_in, uint32_t n,
                                                           uint32_t shift, uint32_t ntiles, const uint32_t *incl,
                                                           uint32_t *key_out, uint32_t *val_out, bool write_keys) {
  __shared__ uint32_t s_cnt[kRsWaves][kRsDigits];
  __shared__ uint32_t s_base[kRsDigits];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (uint32_t v = 0; v < kRsWaves; ++v) s_cnt[v][threadIdx.x] = 0;
  __syncthreads();
  const size_t first = (size_t)blockIdx.x * kRsTile + (size_t)w * (64 * kRsItems);
  const unsigned long long lt = (1ull << lane) - 1;
  uint32_t keys[kRsItems], vals[kRsItems], rank[kRsItems];
#pragma unroll
  for (uint32_t u = 0; u < kRsItems; ++u) {
    const size_t i = first + u * 64 + lane;
    const bool valid = i < n;
    keys[u] = valid ? key_in[i] : 0u;
    vals[u] = valid ? val_in[i] : 0u;
    const uint32_t d = (keys[u] >> shift) & (kRsDigits - 1);
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (uint32_t b = 0; b < kRsBits; ++b) {
      const unsigned long long bal = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? bal : ~bal;
    }
    // all lanes read the count before the leaders (lowest lane of each digit)
    // write it back: LDS operations of one wave complete in program order
    const uint32_t before = valid ? s_cnt[w][d] : 0u;
    rank[u] = before + (uint32_t)__popcll(peers & lt);
    __builtin_amdgcn_wave_barrier();
    if (valid && (peers & lt) == 0) s_cnt[w][d] = before + (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  {  // per digit: exclusive prefix over the waves, and the tile's global base
    const uint32_t d = threadIdx.x;
    uint32_t pre = 0;
#pragma unroll
    for (uint32_t v = 0; v < kRsWaves; ++v) {
      const uint32_t c = s_cnt[v][d];
      s_cnt[v][d] = pre;
      pre += c;
    }
    s_base[d] = incl[(size_t)d * ntiles + blockIdx.x] - pre;
  }
  __syncthreads();
#pragma unroll
  for (uint32_t u = 0; u < kRsItems; ++u) {
    const size_t i = first + u * 64 + lane;
    if (i < n) {
      const uint32_t d = (keys[u] >> shift) & (kRsDigits - 1);
      const uint32_t at = s_base[d] + s_cnt[w][d] + rank[u];
      if (write_keys) key_out[at] = keys[u];
      val_out[at] = vals[u];
    }
  }
}

struct Buf {
  void *p = nullptr;
  explicit Buf(size_t bytes) { IDX_CHECK(hipMalloc(&p, bytes < 256 ? 256 : bytes)); }
  ~Buf() {
    if (p) (void)hipFree(p);
  }
  Buf(const Buf &) = delete;
  Buf &operator=(const Buf &) = delete;
  template <class T> T *as() const { return static_cast<T *>(p); }
};

uint32_t Bits(uint32_t v) {
  uint32_t b = 0;
  while ((1ull << b) <= v) ++b;
  return b;
}

}  // namespace

void BuildIndexDevice(const uint8_t *seq, uint32_t len, uint32_t seed, uint32_t kcl, uint32_t *keys_count,
                      uint32_t *positions, uint32_t *npos, int device, float *device_ms) {
  if (seed == 0) throw Error("index: empty seed");
  const uint32_t span = SeedLength(seed), weight = SeedWeight(seed);
  if (weight > 6) throw Error("index: seed weight above 6");
  const uint32_t sentinel = 1u << (kCharBits * weight);
  if (kcl != sentinel + 1) throw Error("index: keys_count length must be 32^weight + 1");
  int ndev = 0;
  IDX_CHECK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) throw Error("index: no such device");
  IDX_CHECK(hipSetDevice(device));
  *npos = 0;
  if (len == 0) {
    for (uint32_t k = 0; k < kcl; ++k) keys_count[k] = 0;
    if (device_ms) *device_ms = 0.f;
    return;
  }
  hipStream_t st;
  IDX_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() { (void)hipStreamDestroy(s); }
  } sg{st};
  const uint32_t rs_tiles = (uint32_t)(((uint64_t)len + kRsTile - 1) / kRsTile);
  const uint32_t rs_hist_n = rs_tiles * kRsDigits;
  const uint32_t scan_n = std::max(kcl, rs_hist_n);
  const uint32_t ntiles = (kcl + kScanTile - 1) / kScanTile;
  Buf d_seq(len), d_key(4ull * len), d_key2(4ull * len), d_val(4ull * len), d_val2(4ull * len);
  Buf d_counts(4ull * kcl), d_tiles(4ull * ((scan_n + kScanTile - 1) / kScanTile)), d_hist(4ull * rs_hist_n);
  const uint32_t end_bit = Bits(sentinel);
  hipEvent_t e0, e1;
  IDX_CHECK(hipEventCreate(&e0));
  IDX_CHECK(hipEventCreate(&e1));
  struct EventGuard {
    hipEvent_t a, b;
    ~EventGuard() {
      (void)hipEventDestroy(a);
      (void)hipEventDestroy(b);
    }
  } eg{e0, e1};
  IDX_CHECK(hipMemcpyAsync(d_seq.p, seq, len, hipMemcpyHostToDevice, st));
  IDX_CHECK(hipEventRecord(e0, st));
  IDX_CHECK(hipMemsetAsync(d_counts.p, 0, 4ull * kcl, st));
  hipLaunchKernelGGL(k_index_keys, dim3((len + kIdxBlock - 1) / kIdxBlock), dim3(kIdxBlock), 0, st,
                     d_seq.as<uint8_t>(), len, seed, span, sentinel, d_key.as<uint32_t>(), d_val.as<uint32_t>(),
                     d_counts.as<uint32_t>());
  hipLaunchKernelGGL(k_scan_tiles, dim3(ntiles), dim3(kIdxBlock), 0, st, d_counts.as<uint32_t>(), kcl,
                     d_tiles.as<uint32_t>());
  hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(kIdxBlock), 0, st, d_tiles.as<uint32_t>(), ntiles);
  hipLaunchKernelGGL(k_scan_add, dim3((kcl + kIdxBlock - 1) / kIdxBlock), dim3(kIdxBlock), 0, st,
                     d_counts.as<uint32_t>(), kcl, d_tiles.as<uint32_t>());
  IDX_CHECK(hipGetLastError());
  // stable LSD radix sort of (key, j), ping-ponging between the two buffer pairs
  uint32_t *kin = d_key.as<uint32_t>(), *vin = d_val.as<uint32_t>();
  uint32_t *kout = d_key2.as<uint32_t>(), *vout = d_val2.as<uint32_t>();
  const uint32_t hist_tiles = (rs_hist_n + kScanTile - 1) / kScanTile;
  for (uint32_t shift = 0; shift < end_bit; shift += kRsBits) {
    const bool last = shift + kRsBits >= end_bit;
    hipLaunchKernelGGL(k_rs_hist, dim3(rs_tiles), dim3(kIdxBlock), 0, st, kin, len, shift, rs_tiles,
                       d_hist.as<uint32_t>());
    hipLaunchKernelGGL(k_scan_tiles, dim3(hist_tiles), dim3(kIdxBlock), 0, st, d_hist.as<uint32_t>(), rs_hist_n,
                       d_tiles.as<uint32_t>());
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(kIdxBlock), 0, st, d_tiles.as<uint32_t>(), hist_tiles);
    hipLaunchKernelGGL(k_scan_add, dim3((rs_hist_n + kIdxBlock - 1) / kIdxBlock), dim3(kIdxBlock), 0, st,
                       d_hist.as<uint32_t>(), rs_hist_n, d_tiles.as<uint32_t>());
    hipLaunchKernelGGL(k_rs_scatter, dim3(rs_tiles), dim3(kIdxBlock), 0, st, kin, vin, len, shift, rs_tiles,
                       d_hist.as<uint32_t>(), kout, vout, !last);
    IDX_CHECK(hipGetLastError());
    std::swap(kin, kout);
    std::swap(vin, vout);
  }
  IDX_CHECK(hipEventRecord(e1, st));
  IDX_CHECK(hipMemcpyAsync(keys_count, d_counts.p, 4ull * kcl, hipMemcpyDeviceToHost, st));
  IDX_CHECK(hipStreamSynchronize(st));
  const uint32_t n = keys_count[kcl - 1];
  if (n > len) throw Error("index: position count out of range");
  if (n) IDX_CHECK(hipMemcpyAsync(positions, vin, 4ull * n, hipMemcpyDeviceToHost, st));
  IDX_CHECK(hipStreamSynchronize(st));
  *npos = n;
  if (device_ms) IDX_CHECK(hipEventElapsedTime(device_ms, e0, e1));
}

}  // namespace ghostm

extern "C" int GhostmBuildIndexGpu(const uint8_t *seq, uint32_t len, uint32_t seed, uint32_t kcl,
                                   uint32_t *keys_count, uint32_t *positions, uint32_t *npos, int device,
                                   float *device_ms) {
  try {
    if ((!seq && len) || !keys_count || !npos || (!positions && len)) throw ghostm::Error("index: null argument");
    ghostm::BuildIndexDevice(seq, len, seed, kcl, keys_count, positions, npos, device, device_ms);
    return 0;
  } catch (std::exception &e) {
    ghostm::SetLastErrorMessage(e.what());
    return 1;
  }
}
