// provider_cost.cpp -- where a TileProvider::next() token's time goes (tools only, CPU; r05).  The reference's
// next() (src/tile_provider.cpp:27-67) and token destructor (include/vpt/tile_provider.hpp:22-27) per token:
// a relaxed fetch_add on the shared job counter, jid / T and jid % T by the runtime tile count (a 64-bit
// division), the tile's wave load, and on release a seq_cst store plus notify_all.  Each line adds one of
// them to a single-thread loop over a C3 frame's 8 294 400 jobs; then the restated provider itself
// (tests/native/tile_provider_headless.hpp) on 1 / 2 / 4 threads.
//   g++ -O2 -std=c++20 -pthread -I tests/native tools/probes/provider_cost.cpp -o /tmp/provider_cost && /tmp/provider_cost
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

#include "tile_provider_headless.hpp"

int main() {
  const size_t T = 32400, N = T * 256;
  std::vector<std::atomic<unsigned>> tw(T);
  std::atomic<size_t> idx{0};
  volatile size_t vT = T;  // the tile count is a runtime value in the reference (m_tile_wave.size())
  auto run = [&](const char* name, auto f) {
    idx = 0;
    for (auto& w : tw) w.store(0);
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t s = 0;
    for (;;) {
      const size_t j = idx.fetch_add(1, std::memory_order_relaxed);
      if (j >= N) break;
      s += f(j);
    }
    const double d = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("%-30s %6.2f ns/token  (%llu)\n", name, d / N * 1e9, (unsigned long long)s);
  };
  run("fetch_add", [&](size_t j) { return j; });
  run("+ jid / T, jid % T", [&](size_t j) { const size_t t = vT; return (1 + j / t) + j % t; });
  run("+ the tile's wave load", [&](size_t j) {
    const size_t t = vT, ti = j % t;
    return (size_t)tw[ti].load(std::memory_order_relaxed) + 1 + j / t;
  });
  run("+ seq_cst store (token dtor)", [&](size_t j) {
    const size_t t = vT, ti = j % t;
    const size_t r = tw[ti].load(std::memory_order_relaxed);
    tw[ti] = (unsigned)(1 + j / t);
    return r;
  });
  run("+ notify_all", [&](size_t j) {
    const size_t t = vT, ti = j % t;
    const size_t r = tw[ti].load(std::memory_order_relaxed);
    tw[ti] = (unsigned)(1 + j / t);
    tw[ti].notify_all();
    return r;
  });
  for (int th : {1, 2, 4}) {
    vpt_headless::TileProvider tp(1920, 1080, 256, 8, 8);
    std::vector<uint64_t> got(th, 0);
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (int i = 0; i < th; ++i)
      pool.emplace_back([&, i] {
        for (;;) {
          auto tok = tp.next();
          if (!tok) break;
          ++got[i];
        }
      });
    for (auto& t : pool) t.join();
    const double d = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t n = 0;
    for (uint64_t g : got) n += g;
    std::printf("restated TileProvider, %d thread(s): %7.1f ms, %5.1f M tokens/s\n", th, d * 1e3, n / d / 1e6);
  }
  return 0;
}
