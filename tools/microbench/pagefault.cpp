// Host page-fault throughput on the GPU box (first touch of fresh memory), for
// the formatter's text buffers: N MB touched by T threads, plain pages vs
// MADV_HUGEPAGE vs MAP_POPULATE, and a second touch of the same memory.
//   g++ -O2 -pthread -o /tmp/pagefault tools/microbench/pagefault.cpp && /tmp/pagefault 128
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

static double Touch(char *p, size_t n, int threads) {
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> ts;
  const size_t per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([=] {
      const size_t lo = t * per, hi = std::min(n, lo + per);
      if (lo < hi) std::memset(p + lo, 1, hi - lo);
    });
  for (auto &t : ts) t.join();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e3;
}

int main(int argc, char **argv) {
  const size_t mb = argc > 1 ? atoi(argv[1]) : 128;
  const size_t n = mb << 20;
  for (const char *f : {"/sys/kernel/mm/transparent_hugepage/enabled", "/sys/kernel/mm/transparent_hugepage/defrag"}) {
    std::ifstream in(f);
    std::string s;
    std::getline(in, s);
    printf("%s: %s\n", f, s.c_str());
  }
  for (int threads : {1, 4, 8, 16}) {
    for (int mode = 0; mode < 3; ++mode) {
      const int flags = MAP_PRIVATE | MAP_ANONYMOUS | (mode == 2 ? MAP_POPULATE : 0);
      auto t0 = std::chrono::steady_clock::now();
      char *p = (char *)mmap(nullptr, n, PROT_READ | PROT_WRITE, flags, -1, 0);
      if (mode == 1) madvise(p, n, MADV_HUGEPAGE);
      const double map_ms = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e3;
      const double first = Touch(p, n, threads), second = Touch(p, n, threads);
      printf("%3zu MB threads %2d %-12s map %7.2f ms first touch %7.2f ms (%.1f GB/s) second %6.2f ms\n", mb, threads,
             mode == 0 ? "plain" : mode == 1 ? "hugepage" : "populate", map_ms, first, n / first / 1e6, second);
      munmap(p, n);
    }
  }
  return 0;
}
