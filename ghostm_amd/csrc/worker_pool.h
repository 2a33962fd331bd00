// WorkerPool: the persistent host threads behind ParallelFor (aligner.cpp).
#pragma once

#include <algorithm>
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace ghostm {

// Persistent workers behind ParallelFor. A fresh std::thread per piece cost
// tens of microseconds each, paid on every segment's text formatting (the last
// segment's is on the step's critical path). The calling thread takes pieces
// too, so nested or concurrent ParallelFor calls always finish, whatever the
// workers are doing. A job lives on its caller's stack: a worker touches it
// only while it holds a claimed, unfinished piece, and the caller returns only
// once every piece is done.
class WorkerPool {
 public:
  static WorkerPool &Get() {
    static WorkerPool *pool = new WorkerPool();  // never destroyed: workers outlive static destruction
    return *pool;
  }

  // pieces 0 .. pieces-1 of fn, claimed in order; the pool grows to at most
  // max_threads - 1 workers for it (the caller works too)
  void Run(unsigned pieces, const std::function<void(unsigned)> &fn, unsigned max_threads = ~0u) {
    Job job;
    job.fn = &fn;
    job.n = pieces;
    job.errors.resize(pieces);
    std::unique_lock<std::mutex> lk(mu_);
    Grow(std::min(pieces, std::max(max_threads, 1u)) - 1);
    jobs_.push_back(&job);
    lk.unlock();
    cv_.notify_all();
    lk.lock();
    if (job.next < job.n) {
      const unsigned t = job.next++;
      lk.unlock();
      Work(&job, t);
      lk.lock();
    }
    jobs_.erase(std::find(jobs_.begin(), jobs_.end(), &job));
    done_cv_.wait(lk, [&] { return job.done == job.n; });
    lk.unlock();
    for (auto &ep : job.errors)
      if (ep) std::rethrow_exception(ep);
  }

 private:
  struct Job {
    const std::function<void(unsigned)> *fn = nullptr;
    unsigned n = 0, next = 0, done = 0;  // next, done: guarded by mu_
    std::vector<std::exception_ptr> errors;
  };

  // runs claimed piece t, then claims the next ones until none is left
  void Work(Job *job, unsigned t) {
    while (true) {
      try {
        (*job->fn)(t);
      } catch (...) {
        job->errors[t] = std::current_exception();
      }
      std::unique_lock<std::mutex> lk(mu_);
      const bool last = ++job->done == job->n;
      if (job->next < job->n) {
        t = job->next++;
        continue;  // lk released by its destructor at the loop's end
      }
      lk.unlock();  // job may be gone from here on
      if (last) done_cv_.notify_all();
      return;
    }
  }

  void Loop() {
    std::unique_lock<std::mutex> lk(mu_);
    while (true) {
      Job *job = nullptr;
      cv_.wait(lk, [&] { return (job = Open()) != nullptr; });
      const unsigned t = job->next++;
      lk.unlock();
      Work(job, t);
      lk.lock();
    }
  }

  Job *Open() const {  // mu_ held
    for (Job *j : jobs_)
      if (j->next < j->n) return j;
    return nullptr;
  }

  void Grow(unsigned want) {  // mu_ held
    want = std::min(want, 63u);
    for (; workers_ < want; ++workers_) std::thread([this] { Loop(); }).detach();
  }

  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<Job *> jobs_;
  unsigned workers_ = 0;
};

}  // namespace ghostm
