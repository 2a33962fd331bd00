// Page-cache write rates of one 25 MB output file on the box: one pwrite
// thread (the streamed writer's way) against ftruncate + a shared mapping filled
// by T threads in parallel (memcpy into the mapped pages), fsync never called.
//   g++ -O2 -pthread tools/microbench/filewrite.cpp -o /tmp/filewrite && /tmp/filewrite /tmp/fw
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static double Now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
  const std::string path = argc > 1 ? argv[1] : "/tmp/fw";
  const size_t bytes = 25u << 20;
  std::vector<char> src(bytes);
  for (size_t i = 0; i < bytes; ++i) src[i] = (char)('a' + i % 26);
  for (int rep = 0; rep < 3; ++rep) {
    for (int threads : {0, 1, 4, 8, 16}) {
      unlink(path.c_str());
      sync();
      usleep(200000);
      const double t0 = Now();
      const int fd = open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
      if (threads == 0) {
        for (size_t off = 0; off < bytes; off += 1u << 20) pwrite(fd, src.data() + off, 1u << 20, (off_t)off);
      } else {
        if (ftruncate(fd, (off_t)bytes) != 0) return 1;
        char *m = (char *)mmap(nullptr, bytes, PROT_WRITE, MAP_SHARED, fd, 0);
        if (m == MAP_FAILED) return 2;
        std::vector<std::thread> ts;
        for (int t = 0; t < threads; ++t)
          ts.emplace_back([&, t] {
            const size_t lo = bytes * t / threads, hi = bytes * (t + 1) / threads;
            std::memcpy(m + lo, src.data() + lo, hi - lo);
          });
        for (auto &t : ts) t.join();
        munmap(m, bytes);
      }
      close(fd);
      printf("rep %d %s: %.2f ms\n", rep, threads ? ("mmap x" + std::to_string(threads)).c_str() : "pwrite x1",
             (Now() - t0) * 1e3);
    }
  }
  unlink(path.c_str());
  return 0;
}
