// host_buffers.h — host memory for the formatted output (the session's text and
// hit records, rebuilt every run).
//
// The first run of a session formats into fresh memory, and first-touch page
// faults serialise on the process's memory map: 64 MB touched by 16 threads
// took 37 ms in 4 KB pages against 7 ms in 2 MB pages (tools/microbench/
// pagefault.cpp). A cfg3 session formats 49 MB of text and 32 MB of records,
// and its first segment's formatting ran 12.2 ms against 5.4 ms in a warm
// session (profiles/r5b/bench_cfg3_trace.txt). So these buffers are anonymous
// mappings advised as huge pages, and the text grows without zero-filling
// (std::string::resize writes every byte it adds).
#pragma once
#include <sys/mman.h>

#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <new>

namespace ghostm {

constexpr size_t kHugeMin = size_t(2) << 20;  // smaller requests come from malloc

// Zeroed memory; large blocks are their own mappings, advised as huge pages.
inline void *HostAlloc(size_t bytes) {
  if (bytes < kHugeMin) {
    void *p = std::calloc(1, bytes ? bytes : 1);
    if (!p) throw std::bad_alloc();
    return p;
  }
  void *p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) throw std::bad_alloc();
  madvise(p, bytes, MADV_HUGEPAGE);  // best effort (THP may be off)
  return p;
}

inline void HostFree(void *p, size_t bytes) {
  if (!p) return;
  if (bytes < kHugeMin)
    std::free(p);
  else
    munmap(p, bytes);
}

// std::vector allocator over HostAlloc / HostFree.
template <class T>
struct HostAllocator {
  using value_type = T;
  HostAllocator() = default;
  template <class U>
  HostAllocator(const HostAllocator<U> &) {}
  T *allocate(size_t n) { return static_cast<T *>(HostAlloc(n * sizeof(T))); }
  void deallocate(T *p, size_t n) { HostFree(p, n * sizeof(T)); }
  template <class U>
  bool operator==(const HostAllocator<U> &) const { return true; }
  template <class U>
  bool operator!=(const HostAllocator<U> &) const { return false; }
};

// Raw text bytes: capacity from HostAlloc, grown geometrically by copying the
// used bytes only; clear() keeps the capacity (a reused part faults nothing).
class TextBuf {
 public:
  TextBuf() = default;
  TextBuf(const TextBuf &) = delete;
  TextBuf &operator=(const TextBuf &) = delete;
  TextBuf(TextBuf &&o) noexcept : p_(o.p_), n_(o.n_), cap_(o.cap_) { o.p_ = nullptr, o.n_ = o.cap_ = 0; }
  TextBuf &operator=(TextBuf &&o) noexcept {
    if (this != &o) {
      HostFree(p_, cap_);
      p_ = o.p_, n_ = o.n_, cap_ = o.cap_;
      o.p_ = nullptr, o.n_ = o.cap_ = 0;
    }
    return *this;
  }
  ~TextBuf() { HostFree(p_, cap_); }

  const char *data() const { return p_; }
  size_t size() const { return n_; }
  size_t room() const { return cap_ - n_; }  // bytes writable at data() + size() without growing
  void clear() { n_ = 0; }
  void reserve(size_t cap) {
    if (cap <= cap_) return;
    char *q = static_cast<char *>(HostAlloc(cap));
    if (n_) std::memcpy(q, p_, n_);
    HostFree(p_, cap_);
    p_ = q;
    cap_ = cap;
  }
  // room for `need` more bytes; returns where they go
  char *Reserve(size_t need) {
    if (n_ + need > cap_) reserve(n_ + need > 2 * cap_ + 4096 ? n_ + need : 2 * cap_ + 4096);
    return p_ + n_;
  }
  void Commit(const char *end) { n_ = (size_t)(end - p_); }

 private:
  char *p_ = nullptr;
  size_t n_ = 0, cap_ = 0;
};

}  // namespace ghostm
