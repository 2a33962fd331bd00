// formats.cpp — see formats.h for the layouts and the reference citations.
#include "formats.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <emmintrin.h>

#include <algorithm>
#include <climits>
#include <cstring>
#include <fstream>
#include <iostream>

#include "common.h"

namespace ghostm {

template <class T>
bool FileArray<T>::Map(const std::string &path, uint64_t off, size_t n) {
  *this = FileArray();
  if (n == 0) return true;
  const size_t bytes = n * sizeof(T);
  const int fd = open(path.c_str(), O_RDONLY);
  struct stat st {};
  const bool ok = fd >= 0 && fstat(fd, &st) == 0;
  if (ok && (uint64_t)st.st_size >= off + bytes) {
    // only the pages holding [off, off + bytes) (a shard's slice of a chunk)
    const uint64_t page = (uint64_t)sysconf(_SC_PAGESIZE);
    const uint64_t first = off / page * page;
    const size_t len = (size_t)(off + bytes - first);
    // the page tables filled by the threads that read the mapping (the staged
    // upload's copies and the query-length pass run on the worker pool), not
    // up front by this one (MAP_POPULATE); GHOSTM_MAP_POPULATE=1 restores it (A/B)
    static const bool populate = [] {
      const char *e = getenv("GHOSTM_MAP_POPULATE");
      return e && strcmp(e, "1") == 0;
    }();
    void *m = mmap(nullptr, len, PROT_READ, MAP_PRIVATE | (populate ? MAP_POPULATE : 0), fd, (off_t)first);
    if (m != MAP_FAILED) {
      if (!populate) madvise(m, len, MADV_WILLNEED);
      hold_ = std::shared_ptr<const void>(m, [len](const void *q) { munmap(const_cast<void *>(q), len); });
      p_ = reinterpret_cast<const T *>(static_cast<const char *>(m) + (off - first));
      n_ = n;
      close(fd);
      return true;
    }
  }
  // short or unmappable: what the file holds, zeros after it
  std::vector<T> v(n, T());
  if (ok) {
    char *dst = reinterpret_cast<char *>(v.data());
    size_t done = 0;
    while (done < bytes) {
      const ssize_t r = pread(fd, dst + done, bytes - done, (off_t)(off + done));
      if (r <= 0) break;
      done += (size_t)r;
    }
  }
  if (fd >= 0) close(fd);
  Own(std::move(v));
  return ok;
}

template <class T>
void FileArray<T>::Own(std::vector<T> v) {
  auto own = std::make_shared<std::vector<T>>(std::move(v));
  p_ = own->data();
  n_ = own->size();
  hold_ = own;
}

template class FileArray<uint8_t>;
template class FileArray<uint32_t>;

uint8_t ProteinCode(unsigned char ch) {
  struct Table {
    uint8_t t[256];
    Table() {
      const char *order = "ARNDCQEGHILKMFPSTWYVBJZX*";
      for (int i = 0; i < 256; ++i) t[i] = kBaseX;
      for (int i = 0; order[i]; ++i) {
        unsigned char u = (unsigned char)order[i];
        t[u] = (uint8_t)i;
        if (u >= 'A' && u <= 'Z') t[u + 32] = (uint8_t)i;
      }
    }
  };
  static const Table table;
  return table.t[ch];
}

uint8_t DnaCode(unsigned char ch) {
  switch (ch) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    case '-': return 5;
    default: return 4;
  }
}

uint32_t SeedLength(uint32_t seed) {
  uint32_t n = 0;
  for (; seed; seed >>= 1) ++n;
  return n;
}

uint32_t SeedWeight(uint32_t seed) {
  uint32_t n = 0;
  for (; seed; seed >>= 1) n += seed & 1;
  return n;
}

template <class T>
static void ReadRaw(std::ifstream &f, T *p, size_t count) {
  f.read(reinterpret_cast<char *>(p), sizeof(T) * count);
}

void NameTable::push_back(std::string_view s) {
  if (!own_) {
    auto o = std::make_shared<std::string>();
    if (!end_.empty()) o->assign(Base(), end_.back() + 1);
    own_ = o;
    hold_.reset();
    data_ = nullptr;
  }
  own_->append(s.data(), s.size());
  if (own_->size() > UINT32_MAX) throw std::length_error("sequence names over 4 GB");
  end_.push_back((uint32_t)own_->size());
  own_->push_back('\n');
}

void NameTable::AdoptLines(std::shared_ptr<const void> hold, const char *data, std::vector<uint32_t> ends) {
  *this = NameTable();
  hold_ = std::move(hold);
  data_ = data;
  end_ = std::move(ends);
}

NameTable NameTable::Slice(size_t i0, size_t n) const {
  NameTable t;
  if (n == 0) return t;
  const uint32_t b = i0 ? end_[i0 - 1] + 1 : 0;
  std::vector<uint32_t> ends(n);
  for (size_t k = 0; k < n; ++k) ends[k] = end_[i0 + k] - b;
  auto own = std::make_shared<std::string>(Base() + b, (size_t)(end_[i0 + n - 1] + 1 - b));
  t.AdoptLines(own, own->data(), std::move(ends));
  return t;
}

// Offsets of the first `want` newlines of buf (16 bytes per compare: names are
// ~8 bytes, so a memchr per line spent most of its time on call overhead).
static void FindNewlines(const char *buf, size_t size, uint32_t want, std::vector<uint32_t> *out) {
  out->reserve(want);
  size_t i = 0;
  const __m128i nl = _mm_set1_epi8('\n');
  for (; i + 16 <= size && out->size() < want; i += 16) {
    uint32_t m = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i *>(buf + i)), nl));
    while (m && out->size() < want) {
      out->push_back((uint32_t)(i + (uint32_t)__builtin_ctz(m)));
      m &= m - 1;
    }
  }
  for (; i < size && out->size() < want; ++i)
    if (buf[i] == '\n') out->push_back((uint32_t)i);
}

NameTable ReadNameLines(const std::string &path, uint32_t n, bool *complete) {
  NameTable names;
  if (complete) *complete = true;
  {
    // the file mapped, split at its first n newlines: the same names as the
    // getline loop below whenever the file holds n terminated lines (the usual
    // case); anything shorter takes that loop
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) {
      for (uint32_t i = 0; i < n; ++i) names.push_back(std::string_view());
      return names;
    }
    struct stat st {};
    if (n && fstat(fd, &st) == 0 && st.st_size > 0 && (uint64_t)st.st_size <= UINT32_MAX) {
      const size_t len = (size_t)st.st_size;
      void *m = mmap(nullptr, len, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
      if (m != MAP_FAILED) {
        std::shared_ptr<const void> hold(m, [len](const void *q) { munmap(const_cast<void *>(q), len); });
        std::vector<uint32_t> ends;
        FindNewlines(static_cast<const char *>(m), len, n, &ends);
        if (ends.size() == n) {
          close(fd);
          names.AdoptLines(std::move(hold), static_cast<const char *>(m), std::move(ends));
          return names;
        }
      }
    }
    close(fd);
  }
  std::ifstream f(path.c_str());
  uint32_t i = 0;
  std::string line;
  if (f) {
    for (; i < n && !f.eof(); ++i) {
      std::getline(f, line);
      names.push_back(line);
    }
  }
  if (i < n) {
    if (f) std::cerr << "warning : couldn't read all sequence names" << std::endl;
    if (complete) *complete = false;
    for (; i < n; ++i) names.push_back(std::string_view());  // the missing names read as empty
  }
  return names;
}

QueryFile::QueryFile(const std::string &p) : prefix(p) {
  std::ifstream f((p + ".inf").c_str(), std::ios::binary);
  if (!f) return;
  ReadRaw(f, &division, 1);
  ReadRaw(f, &max_length, 1);
  ReadRaw(f, &max_nseq, 1);
}

bool QueryFile::ReadChunk(uint32_t id, QueryChunk *q) const {
  if (id >= division) return false;
  const std::string base = prefix + "_" + std::to_string(id);
  std::ifstream f((base + ".inf").c_str(), std::ios::binary);
  if (!f) return false;
  q->id = id;
  ReadRaw(f, &q->nseq, 1);
  ReadRaw(f, &q->L, 1);
  q->names = ReadNameLines(base + ".nam", q->nseq, nullptr);
  q->seq.Map(base + ".seq", 0, (size_t)q->nseq * q->L);
  return true;
}

uint32_t QueryResidues(const uint8_t *s, uint32_t L) {
  // the last byte that is not padding, eight bytes at a time from the end
  constexpr uint64_t kPad8 = 0x0101010101010101ull * kBaseX;
  uint32_t e = L;
  while (e >= 9) {
    uint64_t w;
    std::memcpy(&w, s + e - 8, 8);
    const uint64_t x = w ^ kPad8;
    if (x) return e - 8 + (uint32_t)(63 - __builtin_clzll(x)) / 8 + 1;
    e -= 8;
  }
  uint32_t k = e - 1;
  while (k > 0 && s[k] == kBaseX) --k;
  return k + 1;
}

bool QueryFile::IndexChunk(uint32_t id, QueryChunkIndex *q) const {
  if (id >= division) return false;
  q->base = prefix + "_" + std::to_string(id);
  {
    std::ifstream f((q->base + ".inf").c_str(), std::ios::binary);
    if (!f) return false;
    q->id = id;
    ReadRaw(f, &q->nseq, 1);
    ReadRaw(f, &q->L, 1);
  }
  const uint32_t n = q->nseq, L = q->L;
  // residues of every row, from a read-only mapping of the .seq (rows past the
  // end of a short file are zeros, as ReadChunk leaves them)
  q->qlen.assign(n, 1);
  if (L > 0 && n > 0) {
    const int fd = open((q->base + ".seq").c_str(), O_RDONLY);
    struct stat st {};
    const size_t want = (size_t)n * L;
    size_t have = 0;
    const uint8_t *map = nullptr;
    if (fd >= 0 && fstat(fd, &st) == 0 && st.st_size > 0) {
      have = std::min(want, (size_t)st.st_size);
      void *m = mmap(nullptr, have, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
      if (m != MAP_FAILED) map = static_cast<const uint8_t *>(m);
      else have = 0;
    }
    std::vector<uint8_t> row(L);
    for (uint32_t i = 0; i < n; ++i) {
      const size_t at = (size_t)i * L;
      if (at + L <= have) {
        q->qlen[i] = QueryResidues(map + at, L);
      } else {
        std::fill(row.begin(), row.end(), 0);
        if (at < have) std::memcpy(row.data(), map + at, have - at);
        q->qlen[i] = QueryResidues(row.data(), L);
      }
    }
    if (map) munmap(const_cast<uint8_t *>(map), have);
    if (fd >= 0) close(fd);
  }
  // name lines: the file's bytes and line offsets when it holds n terminated
  // lines (ReadNameLines' fast case); otherwise every name the reference's way
  q->nam.clear();
  q->line.clear();
  q->names.clear();
  {
    std::ifstream b((q->base + ".nam").c_str(), std::ios::binary);
    if (b) {
      b.seekg(0, std::ios::end);
      const std::streamoff size = b.tellg();
      if (size > 0) {
        q->nam.resize((size_t)size);
        b.seekg(0);
        b.read(&q->nam[0], size);
        if (b.gcount() != size) q->nam.clear();
      }
    }
    q->line.reserve((size_t)n + 1);
    q->line.push_back(0);
    const char *p = q->nam.data(), *e = p + q->nam.size();
    while (q->line.size() <= n) {
      const char *nl = static_cast<const char *>(memchr(p, '\n', (size_t)(e - p)));
      if (!nl) break;
      q->line.push_back((uint64_t)(nl - q->nam.data()) + 1);
      p = nl + 1;
    }
    if (q->line.size() != (size_t)n + 1) {
      q->nam.clear();
      q->line.clear();
      q->names = ReadNameLines(q->base + ".nam", n, nullptr);
    }
  }
  q->group_start.assign(n, 1);
  for (uint32_t i = 1; i < n; ++i) {
    if (!q->names.empty()) {
      q->group_start[i] = q->names[i] != q->names[i - 1];
    } else {
      const uint64_t a0 = q->line[i - 1], a1 = q->line[i] - 1, b0 = q->line[i], b1 = q->line[i + 1] - 1;
      q->group_start[i] = !(a1 - a0 == b1 - b0 && std::memcmp(&q->nam[a0], &q->nam[b0], a1 - a0) == 0);
    }
  }
  return true;
}

void QueryChunkIndex::ReadSlice(uint32_t i0, uint32_t n, QueryChunk *q) const {
  q->id = id;
  q->nseq = n;
  q->L = L;
  if (!names.empty()) {
    q->names = names.Slice(i0, n);
  } else {
    // the slice's lines of the .nam bytes
    const uint64_t b = line[i0], e = line[i0 + n];
    std::vector<uint32_t> ends(n);
    for (uint32_t k = 0; k < n; ++k) ends[k] = (uint32_t)(line[i0 + k + 1] - 1 - b);
    auto own = std::make_shared<std::string>(nam, b, e - b);
    q->names.AdoptLines(own, own->data(), std::move(ends));
  }
  // (a short file leaves zeros, as ReadChunk)
  q->seq.Map(base + ".seq", (uint64_t)i0 * L, (size_t)n * L);
}

DbFile::DbFile(const std::string &p) : prefix(p) {
  std::ifstream f((p + ".inf").c_str(), std::ios::binary);
  if (!f) return;
  ReadRaw(f, &division, 1);
  ReadRaw(f, &seed, 1);
  ReadRaw(f, &max_length, 1);
  ReadRaw(f, &sum_length, 1);
}

bool DbFile::ReadChunk(uint32_t id, DbChunk *d) const {
  if ((int64_t)id >= (int64_t)division) return false;
  const std::string base = prefix + "_" + std::to_string(id);
  std::ifstream f((base + ".inf").c_str(), std::ios::binary);
  if (!f) return false;
  d->id = id;
  ReadRaw(f, &d->nseq, 1);
  ReadRaw(f, &d->len, 1);
  d->names = ReadNameLines(base + ".nam", d->nseq, nullptr);
  d->starts.assign(d->nseq, 0);
  {
    std::ifstream s((base + ".pos").c_str(), std::ios::binary);
    if (s) ReadRaw(s, d->starts.data(), d->nseq);
  }
  d->seq.Map(base + ".seq", 0, d->len);
  std::ifstream s((base + ".ind").c_str(), std::ios::binary);
  if (s) {
    ReadRaw(s, &d->seed, 1);
    ReadRaw(s, &d->kcl, 1);
    ReadRaw(s, &d->npos, 1);
    s.close();
    d->keys_count.Map(base + ".ind", 12, d->kcl);
    d->positions.Map(base + ".ind", 12 + 4 * (uint64_t)d->kcl, d->npos);
  }
  return true;
}

uint32_t DbChunk::SubjectOf(uint32_t p) const {
  // Same search as DB::GetID: the last subject first, then a u32 binary search.
  if (starts[nseq - 1] <= p && p < len) return nseq - 1;
  uint32_t lo = 0, hi = nseq - 2;
  while (lo <= hi) {
    const uint32_t mid = (lo + hi) / 2;
    if (starts[mid] <= p && p < starts[mid + 1]) return mid;
    if (starts[mid] < p) lo = mid + 1;
    else hi = mid - 1;
  }
  return UINT_MAX;
}

}  // namespace ghostm
