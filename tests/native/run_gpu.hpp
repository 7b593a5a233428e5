// run_gpu.hpp — the drop-in for vpt::run (include/vpt/worker.hpp:11, src/worker.cpp:92-208) on one
// MI355X context, over the reference's TileProvider.  INTEGRATION.md §2 shows this file verbatim;
// tests/native/run_gpu_harness.cpp compiles it against a headless restatement of TileProvider and
// tests/test_gpu_integration.py drives it from several host threads.
//
// TileProvider::next() blocks until the same tile's previous wave has been released
// (src/tile_provider.cpp:40-60), so a thread that holds a token while calling next() deadlocks on
// itself as soon as the job counter has moved one wave past that token — which, with other threads
// taking jobs, can happen at any batch size.  run_gpu therefore holds no token across next(): each
// token is released as soon as its job id is recorded.  Every recorded job is rendered (no token
// is dropped), and the GPU film needs no tile exclusivity: its adds are fp32 atomics.
#pragma once

#include <cstdint>
#include <mutex>
#include <utility>
#include <vector>

#include "vpt_gpu.h"

// Renders every job `tp` hands out on `ctx` (asynchronously on `hip_stream`, batch_jobs job ids per
// round of token taking, launches overlapping the next round), then adds the context's film into the
// caller's reference-layout film (float[H][W][4], Image<float,4>).  Returns VPT_OK or the first
// error code (vpt_last_error() has the message).  Several threads may call it with one `tp` and one
// `film_host`, each with its own context (one per GPU, as main.cpp:63-68 starts one run per worker).
template <class Provider>
int run_gpu(vpt_gpu_ctx* ctx, Provider& tp, float* film_host, uint64_t batch_jobs, void* hip_stream = nullptr) {
  static std::mutex film_mu;  // the host film is shared by every caller
  std::vector<std::pair<uint64_t, uint64_t>> runs;  // contiguous (jid_begin, count) runs
  for (;;) {
    runs.clear();
    uint64_t taken = 0;
    while (taken < batch_jobs) {
      auto t = tp.next();  // released at the end of this iteration, before the next next()
      if (!t) break;
      const uint64_t jid = t.jid();
      if (!runs.empty() && runs.back().first + runs.back().second == jid)
        ++runs.back().second;
      else
        runs.emplace_back(jid, 1);
      ++taken;
    }
    if (taken == 0) break;  // waves exhausted, stop_at_next_wave() or stop_now() (tile_provider.cpp:33-34)
    for (const auto& r : runs)
      if (int rc = vpt_gpu_render_jobs(ctx, r.first, r.second, nullptr, hip_stream)) return rc;
  }
  if (int rc = vpt_gpu_sync(ctx)) return rc;
  std::lock_guard<std::mutex> lock(film_mu);
  return vpt_gpu_film_add_to_host(ctx, film_host);
}
