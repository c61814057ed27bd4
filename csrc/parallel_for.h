// Host parallel-for of the native core on a persistent worker pool.
//
// The streaming path calls into the host kernels (JSON extraction, record encoding) thousands of
// times per second from several threads at once (one reader per Kafka partition + the engine
// thread); spawning std::threads per call cost more than the work itself at small micro-batches.
// Workers are created once (FDX_HOST_THREADS, default min(hardware threads, 16)); every call is a
// job whose chunks are taken by an atomic counter, and the calling thread works on its own job
// too, so concurrent and nested calls cannot deadlock.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace fdx {

class HostPool {
 public:
  struct Job {
    const std::function<void(int64_t, int64_t)>* fn;
    int64_t n, chunk, nchunks;
    std::atomic<int64_t> next{0};
    std::atomic<int64_t> done{0};
  };

  static HostPool& get() {
    static HostPool pool;
    return pool;
  }

  int size() const { return (int)workers_.size() + 1; }

  void run(int64_t n, int nchunks, const std::function<void(int64_t, int64_t)>& fn) {
    auto job = std::make_shared<Job>();
    job->fn = &fn;
    job->n = n;
    job->nchunks = nchunks;
    job->chunk = (n + nchunks - 1) / nchunks;
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back(job);
    }
    cv_.notify_all();
    work(*job);
    while (job->done.load(std::memory_order_acquire) < job->nchunks) std::this_thread::yield();
  }

  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  HostPool() {
    int n = (int)std::max(1u, std::thread::hardware_concurrency());
    n = std::min(n, 16);
    if (const char* e = std::getenv("FDX_HOST_THREADS")) n = std::max(1, std::atoi(e));
    for (int i = 0; i + 1 < n; ++i) workers_.emplace_back([this] { loop(); });
  }

  static void work(Job& j) {
    for (;;) {
      const int64_t c = j.next.fetch_add(1, std::memory_order_relaxed);
      if (c >= j.nchunks) return;
      const int64_t lo = c * j.chunk, hi = std::min(j.n, lo + j.chunk);
      if (lo < hi) (*j.fn)(lo, hi);
      j.done.fetch_add(1, std::memory_order_acq_rel);
    }
  }

  void loop() {
    for (;;) {
      std::shared_ptr<Job> job;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
        if (stop_) return;
        job = q_.front();
        if (job->next.load(std::memory_order_relaxed) >= job->nchunks) {   // fully handed out
          q_.pop_front();
          continue;
        }
      }
      work(*job);
      std::lock_guard<std::mutex> g(m_);
      if (!q_.empty() && q_.front() == job) q_.pop_front();
    }
  }

  std::vector<std::thread> workers_;
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::shared_ptr<Job>> q_;
  bool stop_ = false;
};

template <class Fn>
void parallel_for(int64_t n, int threads, int64_t min_chunk, Fn&& fn) {
  if (n <= 0) return;
  HostPool& pool = HostPool::get();
  if (threads <= 0) threads = pool.size();
  threads = (int)std::min<int64_t>(threads, std::max<int64_t>(1, n / std::max<int64_t>(1, min_chunk)));
  if (threads <= 1) { fn(0, n); return; }
  const std::function<void(int64_t, int64_t)> f = [&fn](int64_t lo, int64_t hi) { fn(lo, hi); };
  pool.run(n, threads, f);
}

}  // namespace fdx
