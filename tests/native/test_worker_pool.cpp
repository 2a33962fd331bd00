// Stress test of ghostm::WorkerPool (ghostm_amd/csrc/worker_pool.h), built for
// the host with ThreadSanitizer by tests/test_worker_pool.py: many concurrent
// callers, nested jobs, exceptions, and every piece run exactly once.
#include "worker_pool.h"

#include <atomic>
#include <cstdio>
#include <stdexcept>
#include <thread>
#include <vector>

int main() {
  ghostm::WorkerPool &pool = ghostm::WorkerPool::Get();
  int failures = 0;
  // concurrent callers, each with its own job
  std::vector<std::thread> callers;
  std::atomic<int> bad{0};
  for (int c = 0; c < 6; ++c) {
    callers.emplace_back([&pool, &bad, c] {
      for (int rep = 0; rep < 200; ++rep) {
        const unsigned pieces = 1 + (unsigned)((c * 7 + rep) % 17);
        std::vector<int> hits(pieces, 0);
        pool.Run(pieces, [&](unsigned t) { hits[t] += 1; });
        for (int h : hits)
          if (h != 1) bad++;
      }
    });
  }
  for (auto &t : callers) t.join();
  if (bad) {
    printf("concurrent: %d pieces not run exactly once\n", bad.load());
    ++failures;
  }
  // nested: every outer piece runs an inner job
  std::atomic<int> inner{0};
  pool.Run(8, [&](unsigned) { pool.Run(5, [&](unsigned) { inner++; }); });
  if (inner != 40) {
    printf("nested: %d inner pieces, want 40\n", inner.load());
    ++failures;
  }
  // an exception in one piece reaches the caller after every piece has run
  std::atomic<int> ran{0};
  bool caught = false;
  try {
    pool.Run(9, [&](unsigned t) {
      ran++;
      if (t == 4) throw std::runtime_error("piece 4");
    });
  } catch (const std::runtime_error &) {
    caught = true;
  }
  if (!caught || ran != 9) {
    printf("exception: caught %d, ran %d\n", (int)caught, ran.load());
    ++failures;
  }
  printf("%d failures\n", failures);
  return failures ? 1 : 0;
}
