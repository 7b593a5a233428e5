// vpt_ctx.h — the host side's internal state, shared by the context / render / ABI translation unit
// (vpt_gpu.hip) and the feed protocol's (vpt_feed.cpp): an integrator context, a feed, and the few functions
// one calls in the other.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "vpt_internal.h"
#include "vpt_launch.h"

#define VPT_HIP(call)                                                                                 \
  do {                                                                                                \
    hipError_t e_ = (call);                                                                           \
    if (e_ != hipSuccess)                                                                             \
      return ::vpt::set_error(VPT_E_HIP, std::string(#call " failed: ") + hipGetErrorString(e_));            \
  } while (0)

// A context's job order (vpt_gpu_set_job_order); A/B builds override it.
#ifndef VPT_DEFAULT_JOB_ORDER
#define VPT_DEFAULT_JOB_ORDER VPT_ORDER_COST_SAME_TILE
#endif

// The density-only kernel takes its run-skipping variant when this share of the interior cells has a run
// radius >= 2 (C2's cube: 1.0; the cloud: below it; r06zb: C3 on it 21 % slower).
#ifndef VPT_RUNS_MIN_FRACTION
#define VPT_RUNS_MIN_FRACTION 0.25
#endif

namespace vpt {
struct DeviceGrid {
  void* cells8 = nullptr;
  void* runs8 = nullptr;
  void* walk8 = nullptr;
  double run_fraction = 0.0;
  void* cells128 = nullptr;
  void* root = nullptr;
  void* bricks = nullptr;
  DevGrid dev{};
  size_t bytes = 0;
};

}  // namespace vpt

namespace vpt {
// The shared state of an open feed, as its launch sees it (see KernelEnvT::fetch_feed).
struct FeedLaunch {
  const uint64_t* word;
  uint64_t* ring;
  uint64_t mask;
  unsigned* error;
  uint64_t* started;
  uint64_t* waiting;
  uint32_t* tile_done;  // nullptr unless a staged feed
};
}  // namespace vpt

struct vpt_gpu_feed;

struct vpt_gpu_ctx {
  int device = 0;
  vpt_configuration cfg{};
  vpt::DevScene scene{};
  vpt::DeviceGrid density, temperature;
  float* bb = nullptr;
  float* cie = nullptr;
  float* film = nullptr;
  uint64_t film_count = 0;
  // Per-launch job / event counters: a ring of kLaunchSlots pairs, so launches on different streams
  // of one context never share a counter.  slot_done[i] is recorded on the stream of the launch
  // that last used slot i; the next launch to take slot i waits for it on its own stream first.
  unsigned long long* job_counter = nullptr;  // [kLaunchSlots][2]: jobs, events
  hipEvent_t slot_done[64] = {};
  bool slot_used[64] = {};
  uint32_t next_slot = 0;
  std::mutex slot_mu;
  unsigned long long* counters = nullptr;
  unsigned long long* prof = nullptr;
  vpt::DevScene* scene_dev = nullptr;  // the kernel's copy of scene (read through ScenePtr)
  // Latency-bound launches (fewer work items than the grid has lanes): their own gates (a second
  // device copy of the scene with lat_gate[] in place of the gates) and jobs spread over wavefronts.
  vpt::DevScene* scene_lat_dev = nullptr;
  int lat_gate[4] = {1, 65, 1, 1};   // gate_min, gate_idle, gate_eval, gate_walk
  int lat_wave_lanes = 0;            // 0: spread the items evenly over the grid's wavefronts
  hipStream_t stream = nullptr;
  bool use_runs = false;             // density-only kernel variant with run skipping (see create)
  int pixel_chunk = 0;               // throughput mode: pixels per work item (0 = auto, see render)
  int grid_blocks = 0;               // resident capacity (or the set_tuning override)
  int cus = 1;                       // compute units of the device
  bool grid_user = false;            // grid_blocks set by vpt_gpu_set_tuning: use it as is
  int order_mode = VPT_DEFAULT_JOB_ORDER;
  int order_tail_waves = 0;        // VPT_ORDER_COST_TAIL: tile-major waves (0 = auto)
  uint32_t* order = nullptr;       // tile ranks by descending cost (device), built on first use
  std::vector<float> tile_cost;    // host copy of the estimates
  uint32_t* perm = nullptr;        // explicit job order of launches with perm_n jobs (device)
  uint64_t perm_n = 0;
  std::vector<uint32_t> tile_rank;
  float* staging = nullptr;        // pinned host buffer of film_count floats (vpt_gpu_film_flush_to_host)
  // Feeds whose launches have ended, kept for reuse: while a feed is open its launch holds the device,
  // and a call that waits for the whole device (hipFree, hipHostFree, hipHostMalloc may) would wait for
  // that launch -- i.e. until its lanes give up -- so a feed's memory is allocated once and freed with
  // the context.
  std::vector<vpt_gpu_feed*> feed_pool;
  // Feeds launched and not yet closed: a call that waits for the context's launches (wait_ctx) would wait
  // for such a feed's lanes to give up (30 s) and lose its work, so those calls refuse while it is > 0.
  std::atomic<int> open_feeds{0};
  // Pinned zeros: staged feeds clear their film and tile counts with host-to-device copies, which the copy
  // engines run beside a launch that holds every CU (a fill kernel would wait for it; r05a probe).
  float* zeros = nullptr;
  int lat_mode = -1;              // latency kernel: -1 auto (launches of <= lat_per_cu blocks per CU), 0 off, 1 on
  int lat_ungated = 0;             // its partly filled launches read the latency gates (1) or the context's (0)
  int lat_per_cu = 1;              // resident blocks per CU of the latency kernel
  int compact_every = 0;           // live-path compaction on partly filled latency launches: meeting period (0 off)
  int compact_per_cu = 0;          // resident blocks per CU of the compacting kernel (its LDS exchange)
  // The ordered film (vpt_gpu_set_film_order): the sample buffer of ordered launches (one at a time: each
  // waits for the previous one's vpt_film_order_kernel, samples_done), and the largest buffer a launch may use
  // (0 = auto, 3/4 of the device's free memory when it grows; larger launches are split).
  int film_order = VPT_FILM_ORDERED;
  uint64_t film_order_max = 0;
  float* samples = nullptr;
  uint64_t samples_bytes = 0;
  hipEvent_t samples_done = nullptr;
  bool samples_used = false;
  uint64_t ordered_launches = 0, atomic_launches = 0;  // (vpt_gpu_film_order_info)
  // The drop-in's ordered frame (vpt_gpu_frame_open / _finish): its feed launches also store the samples of the
  // frame's tiles [frame_tile_lo, + frame_tiles) from job frame_jid_lo on into the sample buffer above, frame_waves
  // waves of those tiles (0: no frame open); the order pass writes frame_film (device, film_count floats), copied
  // into the host film through staging.
  uint64_t frame_waves = 0, frame_jid_lo = 0;
  uint32_t frame_tile_lo = 0, frame_tiles = 0;
  float* frame_film = nullptr;
  // vpt_gpu_create's phases (ms): grid flatten + majorant fix, grid upload, the rest, the tile-cost pass, device bind
  double setup_ms[5] = {};
};

// A feed: one launch of the production kernel that renders job ids as the host pushes them (see
// include/vpt_gpu.h).  Its host-pinned, coherent block holds the published word, the error word and the
// started hint, then the ring of job ids, then the per-tile job counts pushed.
struct vpt_gpu_feed {
  vpt_gpu_ctx* ctx = nullptr;
  hipStream_t stream = nullptr;
  float* film = nullptr;
  uint64_t* block = nullptr;  // hipHostMalloc'd: [8] word, error word, waiting word, padding, [4..8) the started
                              // hints; [cap] ring; uint32 counts[T]
  uint64_t* word = nullptr;
  uint32_t* error = nullptr;    // block[1]: a lane that gave up waiting stores 1 here
  uint64_t* started = nullptr;  // block[4..4 + kHintSlots): reported reserved items (kStartedHint)
  uint64_t* waiting = nullptr;  // block[2]: the job count a wavefront saw when it ran out of published items
  uint64_t* ring = nullptr;
  uint32_t* counts = nullptr;
  bool stage = false;
  // Staged feeds: the launch counts the jobs it completes per tile in device memory; snapshots and the final
  // collect copy that and the film into pinned memory with the copy engines (beside the launch, which holds
  // every CU) and add what is new since the previous copy into the caller's film.
  uint32_t* done_dev = nullptr;   // uint32[T]
  float* pin_film = nullptr;      // film_count floats, pinned
  uint32_t* pin_done = nullptr;   // uint32[T], pinned
  std::vector<float> shown;       // the film as already added to the caller's film
  std::vector<uint32_t> shown_done;
  hipStream_t copy_stream = nullptr;
  hipStream_t own_stream = nullptr;  // a staged feed's launch stream when the caller passes none
  bool ring_clean = false;           // every slot holds kFeedEmpty (a completed feed's lanes marked them all)
  uint64_t cap = 0;
  uint64_t published = 0;
  uint64_t started_seen = 0;
  std::chrono::steady_clock::time_point started_moved{};  // when started_seen last moved (vpt_gpu_feed_backlog)
  std::chrono::steady_clock::time_point stale_traced{};
  hipEvent_t closed_ev = nullptr;
  bool closed = false;
  bool launched = false;     // the launch starts once launch_at items are published, or at close
  bool counted = false;      // counted in ctx->open_feeds (launched, not closed)
  uint64_t launch_at = 0;
  vpt::FeedLaunch fl{};
};


namespace vpt::host {
// vpt_gpu.hip
int ctx_device(vpt_gpu_ctx* ctx);  // binds the calling thread to the context's device
// Renders jobs [jid_begin, jid_begin + jid_count) (the launch's kernel variant, grid and job order chosen here);
// feed != nullptr: the feed's launch (job ids from its ring).
int render(vpt_gpu_ctx* ctx, uint64_t jid_begin, uint64_t jid_count, float* film, float* records, void* stream_ptr,
           vpt_event* events = nullptr, uint64_t event_cap = 0, uint32_t* slot_out = nullptr,
           const vpt::FeedLaunch* feed = nullptr);
// The sample-count channel of a closed feed: each pixel of tile t gains counts_dev[t] (vpt_tile_count_kernel).
int launch_tile_counts(vpt_gpu_ctx* ctx, float* film, const uint32_t* counts_dev, hipStream_t s);
// vpt_feed.cpp
void feed_pool_free(vpt_gpu_ctx* ctx);  // frees the context's pooled feeds (vpt_gpu_destroy)
}  // namespace vpt::host
