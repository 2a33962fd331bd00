// Host test of ghostm_amd/csrc/host_buffers.h, built with AddressSanitizer by
// tests/test_host_buffers.py: TextBuf growth across the malloc / mapping
// boundary keeps every byte, clear() keeps the capacity, moves transfer
// ownership; HostAllocator vectors and HostAlloc's zeroed memory.
#include "host_buffers.h"

#include <cstdio>
#include <string>
#include <vector>

int main() {
  int failures = 0;
  auto check = [&](bool ok, const char *what) {
    if (!ok) {
      std::printf("FAIL %s\n", what);
      ++failures;
    }
  };
  ghostm::TextBuf t;
  std::string want;
  unsigned x = 12345;
  for (int line = 0; line < 200000; ++line) {  // ~9 MB: crosses kHugeMin several times
    const size_t len = 10 + (x = x * 1103515245u + 12345u) % 70;
    char *p = t.Reserve(len + 1);
    for (size_t k = 0; k < len; ++k) p[k] = (char)('a' + (line + k) % 26);
    p[len] = '\n';
    want.append(p, len + 1);
    t.Commit(p + len + 1);
  }
  check(t.size() == want.size() && std::string(t.data(), t.size()) == want, "grown text equals the appended lines");
  check(t.room() >= 1 && t.Reserve(t.room()) == t.data() + t.size(), "room() bytes fit without growing");
  const char *before = t.data();
  t.clear();
  check(t.size() == 0, "clear empties");
  char *p = t.Reserve(want.size());
  check(p == before, "clear keeps the capacity");
  ghostm::TextBuf u(std::move(t));
  check(t.data() == nullptr && t.size() == 0 && u.data() == before, "move transfers the buffer");
  ghostm::TextBuf v;
  v = std::move(u);
  check(v.data() == before && u.data() == nullptr, "move assignment transfers the buffer");
  std::vector<int, ghostm::HostAllocator<int>> big;
  for (int k = 0; k < 3000000; ++k) big.push_back(k);  // 12 MB of mappings, grown by copies
  bool ok = true;
  for (int k = 0; k < 3000000; ++k) ok = ok && big[k] == k;
  check(ok, "HostAllocator vector keeps its elements");
  for (size_t n : {size_t(100), size_t(3) << 20}) {
    unsigned char *z = static_cast<unsigned char *>(ghostm::HostAlloc(n));
    bool zero = true;
    for (size_t k = 0; k < n; ++k) zero = zero && z[k] == 0;
    check(zero, "HostAlloc returns zeroed memory");
    ghostm::HostFree(z, n);
  }
  std::printf("%d failures\n", failures);
  return failures ? 1 : 0;
}
