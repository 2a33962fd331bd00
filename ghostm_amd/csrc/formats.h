// formats.h — readers for the formatted query and database files consumed by
// `aln` (on-disk layout defined by the reference formatters):
//   query  <p>.inf      {i32 division, u32 L, u32 max_nseq, 32 x i32 pad}   query_creator.cpp:327-346
//          <p>_<i>.inf  {u32 nseq, u32 L}; .nam one name per line; .seq nseq*L codes
//   db     <p>.inf      {i32 division, u32 seed, u32 maxlen, u64 sum_residues, pad}
//          <p>_<i>.inf  {u32 nseq, u32 len}; .nam; .pos u32[nseq] subject starts;
//          .seq u8[len] END-separated; .ind {u32 seed, u32 kcl, u32 npos,
//          u32 keys_count[kcl] (CSR offsets), u32 positions[npos]}
// Readers mirror QueryReader/Query (query_reader.cpp:34-102, query.cpp:37-79) and
// DBReader/DB/Index (db_reader.cpp:34-77, db.cpp:36-123, index.h:86-126).
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

namespace ghostm {

// Sequence names of a chunk: the .nam file's own bytes (a read-only mapping of
// its page-cache pages: no copy, no zero-filled buffer) and the offset of each
// name's newline, instead of one std::string per name (cfg 4's 1 M query names
// took ~10 ms per query chunk to build as strings, most of the session's file
// loading). Names added one by one (the getline path, slices) are kept in an
// owned buffer in the same layout: each name followed by one separator byte.
class NameTable {
 public:
  size_t size() const { return end_.size(); }
  bool empty() const { return end_.empty(); }
  std::string_view operator[](size_t i) const {
    const uint32_t b = i ? end_[i - 1] + 1 : 0;
    return std::string_view(Base() + b, (size_t)(end_[i] - b));
  }
  void clear() { *this = NameTable(); }
  void push_back(std::string_view s);
  // the lines of a mapped or owned buffer: name i ends at ends[i] (excluded),
  // the next one starts at ends[i] + 1
  void AdoptLines(std::shared_ptr<const void> hold, const char *data, std::vector<uint32_t> ends);
  // names [i0, i0 + n) as a table of their own
  NameTable Slice(size_t i0, size_t n) const;

 private:
  const char *Base() const { return own_ ? own_->data() : data_; }
  std::shared_ptr<const void> hold_;    // the mapping (or an owned buffer) data_ points into
  const char *data_ = nullptr;
  std::shared_ptr<std::string> own_;    // names added one by one
  std::vector<uint32_t> end_;           // name i = [end_[i - 1] + 1, end_[i])
};

// A read-only array of a chunk file's contents: a private, pre-faulted mapping
// of the file (its page-cache pages: no copy, no zero-fill page faults), or
// an owned buffer (a slice, or a file shorter than its header says, the rest
// zeros as the reference's unchecked reads leave it).
template <class T>
class FileArray {
 public:
  const T *data() const { return p_; }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  const T &operator[](size_t i) const { return p_[i]; }
  const T *begin() const { return p_; }
  const T *end() const { return p_ + n_; }
  // n elements of `path` from byte offset `off`; false if it cannot be opened
  // (the array is then n zeros)
  bool Map(const std::string &path, uint64_t off, size_t n);
  void Own(std::vector<T> v);
  void Release() { *this = FileArray(); }
  // empties the array and hands over what held its contents (the mapping or
  // the owned vector), so the caller can drop it elsewhere
  std::shared_ptr<const void> Detach() {
    std::shared_ptr<const void> h = std::move(hold_);
    *this = FileArray();
    return h;
  }

 private:
  const T *p_ = nullptr;
  size_t n_ = 0;
  std::shared_ptr<const void> hold_;  // the mapping or the owned vector
};

struct QueryChunk {
  uint32_t id = 0;
  uint32_t nseq = 0;
  uint32_t L = 0;                  // fixed record width (X padded)
  NameTable names;                 // one per record
  FileArray<uint8_t> seq;          // nseq * L codes
};

// WriteOutput's query length (reference aligner.cpp:959-961): the index of the
// last non-X code + 1, at least 1; also the query's residues for the metric.
uint32_t QueryResidues(const uint8_t *row, uint32_t L);

// One query chunk indexed for a rank-local read (multi-GPU shards, SURVEY.md §8
// e1): every query's residue count from the .seq rows and its name-group start
// from the .nam lines, without building the names of queries the rank will not
// search. ReadSlice then reads only the rank's rows and names.
struct QueryChunkIndex {
  uint32_t id = 0, nseq = 0, L = 0;
  std::vector<uint32_t> qlen;          // QueryResidues of every query
  std::vector<uint8_t> group_start;    // query i's name differs from query i-1's (i = 0: 1)
  // queries [i0, i0 + n) as ReadChunk would read them (names, codes)
  void ReadSlice(uint32_t i0, uint32_t n, QueryChunk *out) const;

  std::string base;                    // <prefix>_<id>
  std::string nam;                     // the .nam file, when it holds nseq terminated lines
  std::vector<uint64_t> line;          // line k = nam[line[k], line[k + 1] - 1)
  NameTable names;                     // otherwise every name, read the reference's way
};

struct QueryFile {
  std::string prefix;
  uint32_t division = 0, max_length = 0, max_nseq = 0;
  explicit QueryFile(const std::string &prefix);
  // Chunk `id` or false if id >= division / files missing.
  bool ReadChunk(uint32_t id, QueryChunk *out) const;
  // Index of chunk `id` (see QueryChunkIndex) or false as ReadChunk.
  bool IndexChunk(uint32_t id, QueryChunkIndex *out) const;
};

struct DbChunk {
  uint32_t id = 0;
  uint32_t nseq = 0;
  uint32_t len = 0;                // concatenated length incl. END separators
  NameTable names;
  std::vector<uint32_t> starts;    // subject start offsets (.pos)
  FileArray<uint8_t> seq;
  uint32_t seed = 0, kcl = 0, npos = 0;
  FileArray<uint32_t> keys_count;
  FileArray<uint32_t> positions;
  // Subject containing concatenated position p (DB::GetID, db.h:106-135).
  uint32_t SubjectOf(uint32_t p) const;
};

struct DbFile {
  std::string prefix;
  int32_t division = 0;
  uint32_t seed = 0, max_length = 0;
  uint64_t sum_length = 0;
  explicit DbFile(const std::string &prefix);
  bool ReadChunk(uint32_t id, DbChunk *out) const;
};

// Seed helpers (Index::GetSeedLength / GetSeedWeight, index.h:116-141).
uint32_t SeedLength(uint32_t seed);
uint32_t SeedWeight(uint32_t seed);

NameTable ReadNameLines(const std::string &path, uint32_t n, bool *complete);

}  // namespace ghostm
