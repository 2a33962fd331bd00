// ghostm_oracle.cpp — TEST INFRASTRUCTURE ONLY. Never linked into, loaded by, or
// called from the product (ghostm_amd/). Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may run it, as the checker / CPU baseline.
//
// A single-threaded CPU restatement of GHOSTM 2.0's `aln` path, written from the
// reference's behaviour (not its text). Every stage keeps the reference's loop
// order and integer/float types so its output is byte-identical:
//   option parsing ........ reference aligner.cpp:225-345
//   chunk loops ........... aligner.cpp:65-223
//   seed search ........... aligner.cpp:383-521  (SearchNextCpu, incl. batch cut)
//   score DP .............. aligner.cpp:545-685  (CalculateScoreCpu)
//   merge ................. aligner.cpp:687-769  (libstdc++ std::sort, unstable)
//   traceback ............. aligner.cpp:771-949
//   output ................ aligner.cpp:951-1012, statistics.cpp:40-59, 134-146
//   matrix reader ......... score_matrix_reader.cpp:44-113
//   file formats .......... query_reader.cpp:34-102, query.cpp:37-79,
//                           db_reader.cpp:34-77, db.cpp:36-123, db.h:106-135
// Pinned against the reference CPU build (oracle/_ref, see oracle/Makefile) and
// the README known-answer output; see tests/test_oracle.py.
//
// Usage: ghostm_oracle aln -i QUERY -d DB -o OUT [reference aln flags]
#include <algorithm>
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <list>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>
#include <getopt.h>

namespace oracle {

// Stage dumps for stage-level parity tests (env GHOSTM_ORACLE_DUMP=<prefix>):
//   <prefix>.cand  u32 {qid, start, score, end} per scored candidate, batch order
//   <prefix>.tb    u32 {qid, end, start, aln_len, aln_match} per traceback
static FILE *DumpFile(const char *suffix) {
  const char *p = getenv("GHOSTM_ORACLE_DUMP");
  if (!p) return nullptr;
  std::string path = std::string(p) + suffix;
  return fopen(path.c_str(), "ab");
}

static const int kAlphabet = 32;   // common.h:31
static const uint8_t kEnd = 25;    // common.h:34
static const uint8_t kX = 23;      // common.h:35

// ---------------------------------------------------------------- sequence codes
// Protein ASCII -> code (reference sequence.cpp:63-87): the 25 letters below get
// codes 0..24 in this order; upper and lower case alike; everything else is X.
static uint8_t ProteinCode(unsigned char ch) {
  static const char kOrder[] = "ARNDCQEGHILKMFPSTWYVBJZX*";
  static uint8_t table[256];
  static bool init = false;
  if (!init) {
    for (int i = 0; i < 256; ++i) table[i] = kX;
    for (int i = 0; kOrder[i]; ++i) {
      table[(unsigned char)kOrder[i]] = (uint8_t)i;
      if (kOrder[i] >= 'A' && kOrder[i] <= 'Z') table[(unsigned char)(kOrder[i] + 32)] = (uint8_t)i;
    }
    // the reference table maps 'U','O','X' (and lower case) to X, '*' to 24
    init = true;
  }
  return table[ch];
}

// ---------------------------------------------------------------- score matrix
struct Matrix {
  std::string name;
  std::vector<int> m;  // [db_code*32 + query_code]
};

// BLOSUM62 used when the -M file cannot be opened (score_matrix_reader.cpp:40-60).
static const char kB62Letters[] = "ARNDCQEGHILKMFPSTWYVBZX*";
static const signed char kB62[24][24] = {
  { 4,-1,-2,-2, 0,-1,-1, 0,-2,-1,-1,-1,-1,-2,-1, 1, 0,-3,-2, 0,-2,-1, 0,-4},
  {-1, 5, 0,-2,-3, 1, 0,-2, 0,-3,-2, 2,-1,-3,-2,-1,-1,-3,-2,-3,-1, 0,-1,-4},
  {-2, 0, 6, 1,-3, 0, 0, 0, 1,-3,-3, 0,-2,-3,-2, 1, 0,-4,-2,-3, 3, 0,-1,-4},
  {-2,-2, 1, 6,-3, 0, 2,-1,-1,-3,-4,-1,-3,-3,-1, 0,-1,-4,-3,-3, 4, 1,-1,-4},
  { 0,-3,-3,-3, 9,-3,-4,-3,-3,-1,-1,-3,-1,-2,-3,-1,-1,-2,-2,-1,-3,-3,-2,-4},
  {-1, 1, 0, 0,-3, 5, 2,-2, 0,-3,-2, 1, 0,-3,-1, 0,-1,-2,-1,-2, 0, 3,-1,-4},
  {-1, 0, 0, 2,-4, 2, 5,-2, 0,-3,-3, 1,-2,-3,-1, 0,-1,-3,-2,-2, 1, 4,-1,-4},
  { 0,-2, 0,-1,-3,-2,-2, 6,-2,-4,-4,-2,-3,-3,-2, 0,-2,-2,-3,-3,-1,-2,-1,-4},
  {-2, 0, 1,-1,-3, 0, 0,-2, 8,-3,-3,-1,-2,-1,-2,-1,-2,-2, 2,-3, 0, 0,-1,-4},
  {-1,-3,-3,-3,-1,-3,-3,-4,-3, 4, 2,-3, 1, 0,-3,-2,-1,-3,-1, 3,-3,-3,-1,-4},
  {-1,-2,-3,-4,-1,-2,-3,-4,-3, 2, 4,-2, 2, 0,-3,-2,-1,-2,-1, 1,-4,-3,-1,-4},
  {-1, 2, 0,-1,-3, 1, 1,-2,-1,-3,-2, 5,-1,-3,-1, 0,-1,-3,-2,-2, 0, 1,-1,-4},
  {-1,-1,-2,-3,-1, 0,-2,-3,-2, 1, 2,-1, 5, 0,-2,-1,-1,-1,-1, 1,-3,-1,-1,-4},
  {-2,-3,-3,-3,-2,-3,-3,-3,-1, 0, 0,-3, 0, 6,-4,-2,-2, 1, 3,-1,-3,-3,-1,-4},
  {-1,-2,-2,-1,-3,-1,-1,-2,-2,-3,-3,-1,-2,-4, 7,-1,-1,-4,-3,-2,-2,-1,-2,-4},
  { 1,-1, 1, 0,-1, 0, 0, 0,-1,-2,-2, 0,-1,-2,-1, 4, 1,-3,-2,-2, 0, 0, 0,-4},
  { 0,-1, 0,-1,-1,-1,-1,-2,-2,-1,-1,-1,-1,-2,-1, 1, 5,-2,-2, 0,-1,-1, 0,-4},
  {-3,-3,-4,-4,-2,-2,-3,-2,-2,-3,-2,-3,-1, 1,-4,-3,-2,11, 2,-3,-4,-3,-2,-4},
  {-2,-2,-2,-3,-2,-1,-2,-3, 2,-1,-1,-2,-1, 3,-3,-2,-2, 2, 7,-1,-3,-2,-1,-4},
  { 0,-3,-3,-3,-1,-2,-2,-3,-3, 3, 1,-2, 1,-1,-2,-2, 0,-3,-1, 4,-3,-2,-1,-4},
  {-2,-1, 3, 4,-3, 0, 1,-1, 0,-3,-4, 0,-3,-3,-2, 0,-1,-4,-3,-3, 4, 1,-1,-4},
  {-1, 0, 0, 1,-3, 3, 4,-2, 0,-3,-3, 1,-1,-3,-1, 0,-1,-3,-2,-2, 1, 4,-1,-4},
  { 0,-1,-1,-1,-2,-1,-1,-1,-1,-1,-1,-1,-1,-1,-2, 0, 0,-2,-1,-1,-1,-1,-1,-4},
  {-4,-4,-4,-4,-4,-4,-4,-4,-4,-4,-4,-4,-4,-4,-4,-4,-4,-4,-4,-4,-4,-4,-4, 1}};

// NCBI-layout text: a heading line of letters, then rows "<letter> v v v ...".
// Tokens are split on single spaces; at most 24 columns and 24 rows are read;
// '#' lines and empty lines are skipped (score_matrix_reader.cpp:73-113).
static void ParseMatrixText(std::istream &in, Matrix *out) {
  out->m.assign(kAlphabet * kAlphabet, 0);
  std::vector<char> cols(kAlphabet, 0), rows(kAlphabet, 0);
  int line_no = 0;
  std::string line;
  while (!in.eof()) {
    std::getline(in, line);
    if (line.empty() || line[0] == '#' || line_no >= kEnd) continue;
    std::vector<std::string> tok;
    size_t p = 0;
    while (p <= line.size()) {
      size_t q = line.find(' ', p);
      if (q == std::string::npos) q = line.size();
      if (q > p) tok.push_back(line.substr(p, q - p));
      p = q + 1;
    }
    for (int i = 0; i < (int)tok.size() && i < kEnd; ++i) {
      if (line_no == 0) {
        cols[i] = tok[i][0];
      } else if (i == 0) {
        rows[line_no - 1] = tok[i][0];
      } else {
        int v = atoi(tok[i].c_str());
        out->m[ProteinCode((unsigned char)rows[line_no - 1]) * kAlphabet +
               ProteinCode((unsigned char)cols[i - 1])] = v;
      }
    }
    ++line_no;
  }
}

static Matrix ReadMatrix(const std::string &path) {
  Matrix mx;
  std::ifstream f(path.c_str());
  if (f) {
    size_t slash = path.find_last_of('/');
    mx.name = slash == std::string::npos ? path : path.substr(slash + 1);
    ParseMatrixText(f, &mx);
    return mx;
  }
  mx.name = "BLOSUM62";
  mx.m.assign(kAlphabet * kAlphabet, 0);
  for (int r = 0; r < 24; ++r)
    for (int c = 0; c < 24; ++c)
      mx.m[ProteinCode(kB62Letters[r]) * kAlphabet + ProteinCode(kB62Letters[c])] = kB62[r][c];
  return mx;
}

// ---------------------------------------------------------------- files
template <class T> static bool ReadPod(std::ifstream &f, T *v) {
  f.read(reinterpret_cast<char *>(v), sizeof(T));
  return (bool)f;
}

static std::vector<std::string> ReadNames(const std::string &path, uint32_t n) {
  std::vector<std::string> names(n);
  std::ifstream f(path.c_str());
  if (!f) return names;
  uint32_t i = 0;
  std::string line;
  for (; i < n && !f.eof(); ++i) {
    std::getline(f, line);
    names[i] = line;
  }
  if (i < n) std::cerr << "warning : couldn't read all sequence names" << std::endl;
  return names;
}

struct QueryChunk {
  uint32_t n = 0, L = 0;
  std::vector<std::string> names;
  std::vector<uint8_t> seq;
};

struct QuerySet {
  std::string prefix;
  uint32_t division = 0, next = 0;
  explicit QuerySet(const std::string &p) : prefix(p) {
    std::ifstream f((p + ".inf").c_str(), std::ios::binary);
    if (f) ReadPod(f, &division);
  }
  bool Read(uint32_t id, QueryChunk *q) {
    if (id >= division) return false;
    std::string base = prefix + "_" + std::to_string(id);
    std::ifstream f((base + ".inf").c_str(), std::ios::binary);
    if (!f) return false;
    ReadPod(f, &q->n);
    ReadPod(f, &q->L);
    next = id + 1;
    q->names = ReadNames(base + ".nam", q->n);
    q->seq.assign((size_t)q->n * q->L, 0);
    std::ifstream s((base + ".seq").c_str(), std::ios::binary);
    s.read(reinterpret_cast<char *>(q->seq.data()), q->seq.size());
    return true;
  }
};

struct DbChunk {
  uint32_t n = 0, len = 0;
  std::vector<std::string> names;
  std::vector<uint32_t> pos;
  std::vector<uint8_t> seq;
  uint32_t seed = 0, kcl = 0, npos = 0;
  std::vector<uint32_t> keys_count, positions;

  // db.h:106-135 — subject containing a concatenated position
  uint32_t SubjectOf(uint32_t p) const {
    if (pos[n - 1] <= p && p < len) return n - 1;
    uint32_t lo = 0, hi = n - 2;
    while (lo <= hi) {
      uint32_t mid = (lo + hi) / 2;
      if (pos[mid] <= p && p < pos[mid + 1]) return mid;
      if (pos[mid] < p) lo = mid + 1; else hi = mid - 1;
    }
    return UINT_MAX;
  }
};

struct DbSet {
  std::string prefix;
  uint32_t division = 0, seed = 0, maxlen = 0, next = 0;
  uint64_t sum_length = 0;
  explicit DbSet(const std::string &p) : prefix(p) {
    std::ifstream f((p + ".inf").c_str(), std::ios::binary);
    if (f) {
      ReadPod(f, &division); ReadPod(f, &seed); ReadPod(f, &maxlen); ReadPod(f, &sum_length);
    }
  }
  bool Read(DbChunk *d) {
    if (next >= division) return false;
    std::string base = prefix + "_" + std::to_string(next);
    std::ifstream f((base + ".inf").c_str(), std::ios::binary);
    if (!f) return false;
    ReadPod(f, &d->n);
    ReadPod(f, &d->len);
    ++next;
    d->names = ReadNames(base + ".nam", d->n);
    d->pos.assign(d->n, 0);
    { std::ifstream s((base + ".pos").c_str(), std::ios::binary);
      s.read(reinterpret_cast<char *>(d->pos.data()), 4 * (size_t)d->n); }
    d->seq.assign(d->len, 0);
    { std::ifstream s((base + ".seq").c_str(), std::ios::binary);
      s.read(reinterpret_cast<char *>(d->seq.data()), d->len); }
    std::ifstream s((base + ".ind").c_str(), std::ios::binary);
    if (s) {
      ReadPod(s, &d->seed); ReadPod(s, &d->kcl); ReadPod(s, &d->npos);
      d->keys_count.assign(d->kcl, 0);
      d->positions.assign(d->npos, 0);
      s.read(reinterpret_cast<char *>(d->keys_count.data()), 4 * (size_t)d->kcl);
      s.read(reinterpret_cast<char *>(d->positions.data()), 4 * (size_t)d->npos);
    }
    return true;
  }
};

// ---------------------------------------------------------------- hit record
struct Hit {
  uint32_t qid = UINT_MAX, sid = UINT_MAX;
  std::string sname;
  uint32_t score = 0, start = UINT_MAX, end = UINT_MAX;
  uint32_t len = UINT_MAX, match = UINT_MAX;
  float id = 0.0f;
};

struct ByScoreDesc {
  bool operator()(const Hit &a, const Hit &b) const { return a.score > b.score; }
};

// ---------------------------------------------------------------- options
struct Options {
  std::string out, qprefix, dbprefix, matrix_file = "BLOSUM62";
  uint32_t qstart = UINT_MAX, qend = UINT_MAX;
  uint32_t log_region = 4, shift = 2, threshold = 2, max_list = 1u << 27;
  int open = -11, ext = -1;
  uint32_t extend = 2, best = 10;
  int device = -1, style = 0;
  bool verbose = false;
  float lambda = 0, K = 0, H = 0;
  Matrix mx;
};

static void ParseOptions(int argc, char **argv, Options *o) {
  optind = 1;
  int c;
  while ((c = getopt(argc, argv, "b:d:D:e:E:G:i:l:M:o:r:s:t:S:L:y:v")) >= 0) {
    switch (c) {
      case 'b': o->best = atoi(optarg); break;
      case 'd': o->dbprefix = optarg; break;
      case 'D': o->device = atoi(optarg); break;
      case 'e': o->extend = atoi(optarg); break;
      case 'E': o->ext = -atoi(optarg); break;
      case 'G': o->open = -atoi(optarg); break;
      case 'i': o->qprefix = optarg; break;
      case 'S': o->qstart = atoi(optarg); break;
      case 'L': o->qend = atoi(optarg); break;
      case 'l': o->max_list = atoi(optarg) * (1 << 20); break;
      case 'M': o->matrix_file = optarg; break;
      case 'o': o->out = optarg; break;
      case 'r': {
        int lr = (int)log2(atoi(optarg));
        o->log_region = lr < 1 ? 1 : lr;
        break;
      }
      case 's': o->shift = atoi(optarg); break;
      case 't': o->threshold = atoi(optarg); break;
      case 'y': o->style = atoi(optarg); break;
      case 'v': o->verbose = true; break;
      default: throw std::invalid_argument("");
    }
  }
  if (const char *e = getenv("GHOSTM_MAX_LIST_OVERRIDE")) o->max_list = (uint32_t)strtoul(e, nullptr, 10);
  o->mx = ReadMatrix(o->matrix_file);
  if (o->style == 0) {  // statistics.cpp:134-146
    if (o->mx.name == "BLOSUM62" && o->open == -11 && o->ext == -1) {
      o->lambda = 0.267f; o->K = 0.041f; o->H = 0.14f;
    } else if (o->mx.name == "PAM30" && o->open == -9 && o->ext == -1) {
      o->lambda = 0.294f; o->K = 0.11f; o->H = 0.61f;
    } else {
      throw std::invalid_argument("error: not support score option");
    }
  }
}

// ---------------------------------------------------------------- the path
class Search {
 public:
  Search(const Options &o, const QueryChunk &q, const DbChunk &d) : o_(o), q_(q), d_(d) {}

  // aligner.cpp:383-521. Appends the next batch of candidates to `batch`
  // (query id, start); returns false when the chunk is exhausted.
  void Next(std::vector<Hit> *batch) {
    batch->clear();
    if (next_query_ == q_.n) return;
    batch->insert(batch->end(), carry_.begin(), carry_.end());
    carry_.clear();
    uint64_t count = batch->size();
    uint32_t seed_len = 0;
    for (uint32_t s = d_.seed; s; s >>= 1) ++seed_len;
    const uint32_t nlists = (q_.L - seed_len) / o_.shift + 1;
    const uint32_t thr = o_.threshold - 1;  // unsigned, as in the reference
    std::vector<const uint32_t *> lst(nlists);
    std::vector<uint32_t> lst_len(nlists), cursor(nlists), head(nlists);
    for (uint32_t i = next_query_; i < q_.n; ++i) {
      const uint8_t *qs = &q_.seq[(size_t)i * q_.L];
      for (uint32_t j = 0; j < nlists; ++j) {
        const uint8_t *w = qs + j * o_.shift;
        uint32_t key = 0, t = 0;
        for (uint32_t s = d_.seed; s; s >>= 1, ++t)
          if (s & 1) key = (key << 5) | w[t];
        uint32_t b = d_.keys_count[key], e = d_.keys_count[key + 1];
        lst[j] = d_.positions.data() + b;
        lst_len[j] = e - b;
        const uint32_t diag0 = j * o_.shift;
        uint32_t k = 0;
        while (k < lst_len[j] && lst[j][k] < diag0) ++k;
        head[j] = UINT_MAX;
        cursor[j] = k;
        if (k < lst_len[j]) {
          head[j] = (lst[j][k] - diag0) >> o_.log_region;
          cursor[j] = k + 1;
        }
      }
      uint32_t bin = 0, cnt = 0;
      for (;;) {
        uint32_t nb = UINT_MAX;
        for (uint32_t j = 0; j < nlists; ++j) nb = std::min(nb, head[j]);
        if (nb == UINT_MAX) break;
        uint32_t nc = 0;
        for (uint32_t j = 0; j < nlists; ++j) {
          if (head[j] != nb) continue;
          ++nc;
          head[j] = UINT_MAX;
          const uint32_t diag0 = j * o_.shift;
          for (uint32_t k = cursor[j]; k < lst_len[j]; ++k) {
            uint32_t bk = (lst[j][k] - diag0) >> o_.log_region;
            if (bk != nb) { head[j] = bk; cursor[j] = k + 1; break; }
          }
        }
        if (nb - bin == 1) cnt += nc;
        if (cnt > thr) Emit(i, bin << o_.log_region, &count);
        cnt = nc;
        bin = nb;
      }
      if (cnt > thr) Emit(i, bin << o_.log_region, &count);
      if (count > o_.max_list) {  // the query stays carried into the next batch
        next_query_ = i + 1;
        // test hook: where the batch loop cuts (query i's candidates open the next batch)
        if (getenv("GHOSTM_ORACLE_BATCHES")) fprintf(stderr, "batch_cut %u\n", i);
        return;
      }
      batch->insert(batch->end(), carry_.begin(), carry_.end());
      carry_.clear();
    }
    next_query_ = q_.n;
  }

  // aligner.cpp:545-685 — Gotoh local score of the padded query against the window.
  void Score(std::vector<Hit> *batch) {
    const uint32_t L = q_.L;
    const uint32_t base = L + 2 * o_.extend + 2 * (1u << o_.log_region);
    const int *M = o_.mx.m.data();
    std::vector<int> H(L + 1), E(L + 1);
    uint32_t end_col = 0;
    for (Hit &h : *batch) {
      int off = (int)(h.start - o_.extend);
      if (off < 0) off = 0;
      uint32_t width = base;
      if (off + width > d_.len) width = d_.len - off;
      const uint8_t *qs = &q_.seq[(size_t)h.qid * L];
      std::fill(H.begin(), H.end(), 0);
      std::fill(E.begin(), E.end(), 0);
      int best = 0;
      for (uint32_t j = 0; j < width; ++j) {
        const uint8_t c = d_.seq[off + j];
        if (c == kEnd) {
          std::fill(H.begin(), H.end(), 0);
          std::fill(E.begin(), E.end(), 0);
          continue;
        }
        const int *row = M + c * kAlphabet;
        int diag = 0, F = 0;
        for (uint32_t k = 1; k <= L; ++k) {
          int cell = std::max(0, diag + row[qs[k - 1]]);
          E[k] = std::max(E[k] + o_.ext, H[k] + o_.open);
          cell = std::max(cell, E[k]);
          F = std::max(F + o_.ext, H[k - 1] + o_.open);
          cell = std::max(cell, F);
          diag = H[k];
          H[k] = cell;
          if (cell >= best) { best = cell; end_col = j; }
        }
      }
      h.score = (uint32_t)best;
      h.end = off + end_col;
    }
    if (FILE *f = DumpFile(".cand")) {
      for (const Hit &h : *batch) {
        uint32_t rec[4] = {h.qid, h.start, h.score, h.end};
        fwrite(rec, 4, 4, f);
      }
      fclose(f);
    }
  }

  // aligner.cpp:771-949 — reverse DP from the end to find start, length, matches.
  void TraceBack(Hit *h) const {
    const int L = (int)q_.L;
    const uint32_t base = q_.L + 2 * o_.extend * 2 * (1u << o_.log_region);
    const int *M = o_.mx.m.data();
    const uint32_t p0 = h->end;
    uint32_t width = p0 < base ? p0 + 1 : base;
    const uint8_t *qs = &q_.seq[(size_t)h->qid * q_.L];
    std::vector<int> H(L + 1, 0), E(L + 1, 0);
    std::vector<uint32_t> AM(L + 1, 0), AL(L + 1, 0);
    int best = 0;
    uint32_t best_j = 0, best_m = 0, best_l = 0;
    for (uint32_t j = 0; j < width; ++j) {
      const uint8_t c = d_.seq[p0 - j];
      if (c == kEnd) break;
      const int *row = M + c * kAlphabet;
      int diag = 0, F = 0;
      uint32_t dm = 0, dl = 0;
      for (int k = L - 1; k >= 0; --k) {
        int cell = 0;
        uint32_t m = 0, l = 0;
        int s = diag + row[qs[k]];
        if (s > 0) { cell = s; m = dm + (c == qs[k] ? 1 : 0); l = dl + 1; }
        E[k] = std::max(E[k] + o_.ext, H[k] + o_.open);
        if (E[k] > cell) { cell = E[k]; m = AM[k]; l = AL[k] + 1; }
        F = std::max(F + o_.ext, H[k + 1] + o_.open);
        if (F > cell) { cell = F; m = AM[k + 1]; l = AL[k + 1] + 1; }
        diag = H[k]; H[k] = cell;
        dm = AM[k]; AM[k] = m;
        dl = AL[k]; AL[k] = l;
        if (cell > best) { best = cell; best_j = j; best_m = m; best_l = l; }
      }
    }
    h->start = p0 - best_j;
    h->id = (float)best_m / (float)best_l;
    h->len = best_l;
    h->match = best_m;
    if (FILE *f = DumpFile(".tb")) {
      uint32_t rec[5] = {h->qid, p0, h->start, h->len, h->match};
      fwrite(rec, 4, 5, f);
      fclose(f);
    }
  }

  // aligner.cpp:687-769 — per group of equal consecutive names: sort, resolve,
  // keep the first hit per subject, trace it back, stop at `best`.
  void Merge(std::vector<std::vector<Hit>> *results, std::vector<Hit> &batch) {
    std::vector<uint32_t> owner(d_.n, UINT_MAX);
    std::vector<Hit> group;
    size_t it = 0;
    std::string prev = q_.names[0];
    for (uint32_t i = 0; i < q_.n; ++i) {
      const std::string &name = q_.names[i];
      if (prev != name) Resolve(&group, i - 1, &owner, results);
      prev = name;
      for (; it < batch.size() && batch[it].qid == i; ++it) group.push_back(batch[it]);
      for (Hit &h : (*results)[i]) group.push_back(h);
      (*results)[i].clear();
    }
    Resolve(&group, q_.n - 1, &owner, results);
  }

 private:
  void Emit(uint32_t qid, uint32_t start, uint64_t *count) {
    Hit h;
    h.qid = qid;
    h.start = start;
    carry_.push_back(h);
    ++*count;
  }

  void Resolve(std::vector<Hit> *group, uint32_t id, std::vector<uint32_t> *owner,
               std::vector<std::vector<Hit>> *results) {
    std::sort(group->begin(), group->end(), ByScoreDesc());
    std::vector<Hit> &out = (*results)[id];
    for (Hit &h : *group) {
      if (h.sid == UINT_MAX) {
        uint32_t sid = d_.SubjectOf(h.end);
        if ((*owner)[sid] != id) {
          (*owner)[sid] = id;
          TraceBack(&h);
          h.sid = sid;
          h.sname = d_.names[sid];
          h.start -= d_.pos[sid];
          h.end -= d_.pos[sid];
          out.push_back(h);
        }
      } else {
        out.push_back(h);
      }
      if (out.size() >= o_.best) break;
    }
    group->clear();
  }

  const Options &o_;
  const QueryChunk &q_;
  const DbChunk &d_;
  uint32_t next_query_ = 0;
  std::vector<Hit> carry_;

 public:
  void Reset() { next_query_ = 0; carry_.clear(); }
};

// aligner.cpp:951-1012 with statistics.cpp:40-59
static void Write(std::ostream &out, const Options &o, const QueryChunk &q,
                  const std::vector<std::vector<Hit>> &results, uint32_t db_sum) {
  const float log2f_ = static_cast<float>(log(2.0));
  const float logK = logf(o.K);
  for (uint32_t i = 0; i < q.n; ++i) {
    const std::string &name = q.names[i];
    if (o.style == 1) {
      for (const Hit &h : results[i])
        out << name << "\t" << h.sname << "\t" << h.score << "\t" << h.start + 1 << "\t"
            << h.end + 1 << std::endl;
    } else if (o.style == 2) {
      for (const Hit &h : results[i])
        out << name << "\t" << h.sname << "\t" << h.score << "\t" << h.start + 1 << "\t"
            << h.end + 1 << "\t" << h.id << "\t" << h.len << "\t" << h.match << std::endl;
    } else {
      const size_t b = (size_t)i * q.L;
      size_t e = b + q.L - 1;
      while (e > b && q.seq[e] == kX) --e;
      const uint32_t qlen = (uint32_t)(e - b + 1);
      const uint64_t space = (uint64_t)qlen * (uint64_t)db_sum;
      for (const Hit &h : results[i]) {
        const int s = (int)h.score;
        const float bits = ((static_cast<float>(s) * o.lambda) - logK) / log2f_;
        const float ev = (float)((double)((float)space * o.K) *
                                 exp(static_cast<double>(-1.0 * s * o.lambda)));
        out << name << "\t" << h.sname << "\t" << h.id * 100 << "\t" << h.len << "\t"
            << h.match << "\t" << h.start + 1 << "\t" << h.end + 1 << "\t" << ev << "\t"
            << bits << "\t" << std::endl;
      }
    }
  }
}

static int Align(int argc, char **argv) {
  Options o;
  ParseOptions(argc, argv, &o);
  std::ofstream out(o.out.c_str());
  QuerySet qs(o.qprefix);
  QueryChunk q;
  bool have = o.qstart == UINT_MAX ? qs.Read(qs.next, &q) : qs.Read(o.qstart, &q);
  if (!have) {
    std::cerr << "[Aligner] error: don't find query file." << std::endl;
    return 0;
  }
  while (have) {
    std::vector<std::vector<Hit>> results(q.n);
    DbSet ds(o.dbprefix);
    DbChunk d;
    if (!ds.Read(&d)) {
      std::cerr << "[Aligner] error: don't find db file." << std::endl;
      break;
    }
    do {
      Search s(o, q, d);
      std::vector<Hit> batch;
      for (;;) {
        s.Next(&batch);
        if (batch.empty()) break;
        s.Score(&batch);
        s.Merge(&results, batch);
      }
      d = DbChunk();
    } while (ds.Read(&d));
    Write(out, o, q, results, (uint32_t)DbSet(o.dbprefix).sum_length);
    have = false;
    if (qs.next <= o.qend) have = qs.Read(qs.next, &q);
  }
  return 0;
}

}  // namespace oracle

int main(int argc, char **argv) {
  if (argc < 2 || strcmp(argv[1], "aln") != 0) {
    std::cerr << "usage: ghostm_oracle aln -i QUERY -d DB -o OUT [options]" << std::endl;
    return 1;
  }
  try {
    return oracle::Align(argc - 1, argv + 1);
  } catch (std::exception &e) {
    std::cerr << e.what() << std::endl;
  }
  return 0;
}
