// qformat.hip — the `qry` formatter's per-residue work on the GPU.
//
// Reference: QueryCreator (query_creator.cpp:191-517).
//   protein  every record's letters -> residue codes (sequence.cpp:63-87), cut at
//            or X-padded to the record width (388-423)
//   DNA      every read of the chunk cut/padded to the chunk's first read length
//            (254-255), then six frames: forward offsets 0..2 and the reverse
//            complement's 0..2 (242-279); a stop codon switches the frame to '*'
//            until the next ATG (280-312); frames '*'-padded to dna_len/3 letters,
//            then coded and cut/padded to the width like protein records
//
// The host keeps what is sequential in the file format (FASTA parsing, chunk
// cuts, names) and hands the chunk's letters over as one concatenated buffer.
//   k_qry_protein  one wave per record: coalesced reads of the record's letters,
//                  one LDS table lookup, coalesced writes (HBM-bound)
//   k_qry_frames   one wave per read, 64 letters of a frame at a time; the
//                  stop/ATG state (a scan along the frame in the reference) is
//                  the last event at or before each letter, found by ballots
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "../../include/ghostm_hip.h"
#include "common.h"
#include "formats.h"

namespace ghostm {

void SetLastErrorMessage(const std::string &m);

namespace {

#define QF_CHECK(expr)                                                                   \
  do {                                                                                   \
    hipError_t err_ = (expr);                                                            \
    if (err_ != hipSuccess)                                                              \
      throw Error(std::string("HIP error '") + hipGetErrorString(err_) + "' at " #expr); \
  } while (0)

constexpr uint32_t kQfBlock = 256;

// Lookup tables (one small device buffer, staged into LDS per block).
struct QfTables {
  uint8_t protein[256];  // letter -> residue code (ProteinCode)
  uint8_t dna[256];      // letter -> base code (DnaCode: A0 C1 G2 T3, '-' 5, else 4)
  uint8_t codon[128];    // 2-bit codon (first base major) -> residue code; 64 = ambiguous
};

struct QfArgs {
  const uint8_t *raw;
  const unsigned long long *off;
  const uint32_t *len;
  uint32_t nrec, width, dna_len;
  uint8_t *out;
  const QfTables *tab;
};

constexpr uint32_t kQfWaves = kQfBlock / 64;

// One wave per record (grid-stride): lanes walk the record's letters and its
// output bytes contiguously, the code table in LDS.
__global__ __launch_bounds__(kQfBlock) void k_qry_protein(QfArgs a) {
  __shared__ uint8_t s_code[256];
  s_code[threadIdx.x] = a.tab->protein[threadIdx.x];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t r = blockIdx.x * kQfWaves + (threadIdx.x >> 6); r < a.nrec; r += gridDim.x * kQfWaves) {
    const uint32_t n = min(a.len[r], a.width);
    const uint8_t *src = a.raw + a.off[r];
    uint8_t *dst = a.out + (uint64_t)r * a.width;
    for (uint32_t k = lane; k < a.width; k += 64) dst[k] = k < n ? s_code[src[k]] : (uint8_t)kBaseX;
  }
}

// One wave per read (grid-stride), its six frames in turn, 64 letters at a time:
// lane t codes letter t (the codon ending at strand position o + 2 + 3t). The
// stop/ATG state of a letter is the type of the last event (ATG clears, a stop
// codon sets) at or before it, else the state carried from the previous 64
// letters: two ballots and a leading-bit search, no sequential walk.
__global__ __launch_bounds__(kQfBlock) void k_qry_frames(QfArgs a) {
  __shared__ uint8_t s_base[256];
  __shared__ uint8_t s_codon[128];
  s_base[threadIdx.x] = a.tab->dna[threadIdx.x];
  if (threadIdx.x < 128) s_codon[threadIdx.x] = a.tab->codon[threadIdx.x];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t n = a.dna_len;
  const uint32_t letters = n / 3;  // every frame after '*' padding
  const uint32_t keep = min(letters, a.width);
  const unsigned long long upto = ~0ull >> (63 - lane);  // lanes 0..lane
  for (uint32_t r = blockIdx.x * kQfWaves + (threadIdx.x >> 6); r < a.nrec; r += gridDim.x * kQfWaves) {
    const uint32_t rl = a.len[r];
    const uint8_t *dna = a.raw + a.off[r];
    for (uint32_t f = 0; f < 6; ++f) {
      const uint32_t s = f / 3, o = f - s * 3;
      // base at strand position j (reads shorter than dna_len are padded with 4)
      auto base = [&](uint32_t j) -> uint32_t {
        const uint32_t p = s ? n - 1 - j : j;
        uint32_t b = p < rl ? s_base[dna[p]] : 4u;
        if (s && b <= 3) b = (~b) & 3u;
        return b;
      };
      uint8_t *rec = a.out + ((uint64_t)r * 6 + f) * a.width;
      uint32_t carry = 0;  // stop state entering this group of 64 letters
      for (uint32_t t0 = 0; t0 < keep; t0 += 64) {
        const uint32_t t = t0 + lane, k = o + 2 + 3 * t;
        uint32_t code = 24, ev = 0;  // '*' padding past the last codon
        if (t < keep && k < n) {
          const uint32_t b0 = base(k - 2), b1 = base(k - 1), b2 = base(k);
          const uint32_t codon = (b0 > 3 || b1 > 3 || b2 > 3) ? 64u : (b0 << 4 | b1 << 2 | b2);
          code = s_codon[codon];
          ev = codon == 14 ? 1u : (codon == 48 || codon == 50 || codon == 56) ? 2u : 0u;  // ATG / TAA TAG TGA
        }
        const unsigned long long evm = __ballot(ev != 0), setm = __ballot(ev == 2);
        const unsigned long long mine = evm & upto;
        const uint32_t stop = mine ? (uint32_t)(setm >> (63 - __clzll(mine))) & 1u : carry;
        if (t < keep) rec[t] = stop ? (uint8_t)24 : (uint8_t)code;
        carry = evm ? (uint32_t)(setm >> (63 - __clzll(evm))) & 1u : carry;
      }
      for (uint32_t t = keep + lane; t < a.width; t += 64) rec[t] = kBaseX;
    }
  }
}

struct Buf {
  void *p = nullptr;
  explicit Buf(size_t bytes) { QF_CHECK(hipMalloc(&p, bytes < 256 ? 256 : bytes)); }
  ~Buf() {
    if (p) (void)hipFree(p);
  }
  Buf(const Buf &) = delete;
  Buf &operator=(const Buf &) = delete;
  template <class T> T *as() const { return static_cast<T *>(p); }
};

QfTables MakeTables() {
  QfTables t;
  for (int i = 0; i < 256; ++i) {
    t.protein[i] = ProteinCode((unsigned char)i);
    t.dna[i] = DnaCode((unsigned char)i);
  }
  // the standard genetic code, first base major over A C G T (formatter.cpp
  // kCodons), as residue codes
  const char *letters = "KNKNTTTTRSRSIIMIQHQHPPPPRRRRLLLLEDEDAAAAGGGGVVVV*Y*YSSSS*CWCLFLF";
  for (int i = 0; i < 128; ++i) t.codon[i] = kBaseX;
  for (int i = 0; i < 64; ++i) t.codon[i] = ProteinCode((unsigned char)letters[i]);
  return t;
}

}  // namespace

void FormatQueriesDevice(const uint8_t *raw, uint64_t raw_len, const uint64_t *offsets, const uint32_t *lengths,
                         uint32_t n, uint32_t width, uint32_t dna_len, uint8_t *records, int device,
                         float *device_ms) {
  if (device_ms) *device_ms = 0.f;
  const uint64_t nout = (uint64_t)n * (dna_len ? 6 : 1);
  if (n == 0 || width == 0) return;
  for (uint32_t r = 0; r < n; ++r)
    if (offsets[r] + lengths[r] > raw_len) throw Error("qry: record outside the letter buffer");
  int ndev = 0;
  QF_CHECK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) throw Error("qry: no such device");
  QF_CHECK(hipSetDevice(device));
  hipStream_t st;
  QF_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() { (void)hipStreamDestroy(s); }
  } sg{st};
  Buf d_raw(raw_len), d_off(8ull * n), d_len(4ull * n), d_out(nout * width), d_tab(sizeof(QfTables));
  hipEvent_t e0, e1;
  QF_CHECK(hipEventCreate(&e0));
  QF_CHECK(hipEventCreate(&e1));
  struct EventGuard {
    hipEvent_t a, b;
    ~EventGuard() {
      (void)hipEventDestroy(a);
      (void)hipEventDestroy(b);
    }
  } eg{e0, e1};
  if (raw_len) QF_CHECK(hipMemcpyAsync(d_raw.p, raw, raw_len, hipMemcpyHostToDevice, st));
  QF_CHECK(hipMemcpyAsync(d_off.p, offsets, 8ull * n, hipMemcpyHostToDevice, st));
  QF_CHECK(hipMemcpyAsync(d_len.p, lengths, 4ull * n, hipMemcpyHostToDevice, st));
  const QfTables tables = MakeTables();
  QF_CHECK(hipMemcpyAsync(d_tab.p, &tables, sizeof(tables), hipMemcpyHostToDevice, st));
  QfArgs a{d_raw.as<uint8_t>(), d_off.as<unsigned long long>(), d_len.as<uint32_t>(), n, width, dna_len,
           d_out.as<uint8_t>(), d_tab.as<QfTables>()};
  // one wave per record / read, grid-stride over at most 64 K blocks
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((n + kQfWaves - 1) / kQfWaves, 65536);
  QF_CHECK(hipEventRecord(e0, st));
  if (dna_len) hipLaunchKernelGGL(k_qry_frames, dim3(blocks), dim3(kQfBlock), 0, st, a);
  else hipLaunchKernelGGL(k_qry_protein, dim3(blocks), dim3(kQfBlock), 0, st, a);
  QF_CHECK(hipGetLastError());
  QF_CHECK(hipEventRecord(e1, st));
  QF_CHECK(hipMemcpyAsync(records, d_out.p, nout * width, hipMemcpyDeviceToHost, st));
  QF_CHECK(hipStreamSynchronize(st));
  if (device_ms) QF_CHECK(hipEventElapsedTime(device_ms, e0, e1));
}

}  // namespace ghostm

extern "C" int GhostmFormatQueriesGpu(const uint8_t *raw, uint64_t raw_len, const uint64_t *offsets,
                                      const uint32_t *lengths, uint32_t n, uint32_t width, uint32_t dna_len,
                                      uint8_t *records, int device, float *device_ms) {
  try {
    if (n && (!offsets || !lengths || !records || (!raw && raw_len))) throw ghostm::Error("qry: null argument");
    ghostm::FormatQueriesDevice(raw, raw_len, offsets, lengths, n, width, dna_len, records, device, device_ms);
    return 0;
  } catch (std::exception &e) {
    ghostm::SetLastErrorMessage(e.what());
    return 1;
  }
}
