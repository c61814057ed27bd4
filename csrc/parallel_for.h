// Minimal std::thread parallel-for for the host (CPU) paths of the native core.
#pragma once
#include <algorithm>
#include <cstdint>
#include <thread>
#include <vector>

namespace fdx {

template <class Fn>
void parallel_for(int64_t n, int threads, int64_t min_chunk, Fn&& fn) {
  if (n <= 0) return;
  if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
  threads = (int)std::min<int64_t>(threads, std::max<int64_t>(1, n / std::max<int64_t>(1, min_chunk)));
  if (threads <= 1) { fn(0, n); return; }
  std::vector<std::thread> pool;
  const int64_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const int64_t lo = t * chunk, hi = std::min(n, lo + chunk);
    if (lo < hi) pool.emplace_back([&fn, lo, hi] { fn(lo, hi); });
  }
  for (auto& th : pool) th.join();
}

}  // namespace fdx
