// Host-side parallel loop for the once-per-polygon-set builders (tessellation, chip
// table).  Threads = OMP_NUM_THREADS when set (the GPU box sets it to its CPU share),
// else the hardware concurrency, capped at 32.  Work is split into contiguous chunks
// handed out dynamically; callers write only to per-index slots so results do not
// depend on the schedule.
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <thread>
#include <vector>

namespace mgpu {

inline int host_threads() {
  int n = 0;
  if (const char* s = std::getenv("OMP_NUM_THREADS")) n = std::atoi(s);
  if (n <= 0) n = (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(n, 32));
}

// fn(begin, end, thread_index) over [0, n) in chunks of `grain`.
template <class F>
void parallel_for(int64_t n, int64_t grain, F&& fn) {
  const int T = (int)std::min<int64_t>(host_threads(), (n + grain - 1) / std::max<int64_t>(grain, 1));
  if (T <= 1) {
    if (n > 0) fn((int64_t)0, n, 0);
    return;
  }
  std::atomic<int64_t> next{0};
  auto work = [&](int t) {
    for (;;) {
      const int64_t b = next.fetch_add(grain);
      if (b >= n) break;
      fn(b, std::min(n, b + grain), t);
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < T; t++) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
}

inline int parallel_slots(int64_t n, int64_t grain) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), (n + grain - 1) / std::max<int64_t>(grain, 1)));
}

}  // namespace mgpu
