// vpt_gpu.hip — the integrator context and the C ABI around the kernels (include/vpt_gpu.h): grid upload,
// scene constants, the launch choices of render() (kernel variant, grid size, job order, the ordered film's
// sample buffer and film pass), counters and knobs.  The device code is vpt_kernels.h (included here, the one
// translation unit that launches it); the feeds' host protocol is vpt_feed.cpp; the state both share is
// vpt_ctx.h.
//
// Kernel shape: a persistent grid sized to the device's resident capacity.  Every lane runs the state machine
// of vpt_integrator.h; when its (tile, wave) job ends it takes the next job id from a device counter, so lanes
// are refilled until the job range is drained and every wave reaches ST_DONE.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <memory>
#include <atomic>
#include <mutex>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "vpt_ctx.h"
#include "vpt_kernels.h"

namespace vpt {

static thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

}  // namespace vpt

using vpt::host::ctx_device;
using vpt::host::render;

namespace vpt {
static int upload(const void* src, size_t n, void** dst, size_t& bytes) {
  *dst = nullptr;
  if (n == 0) return VPT_OK;
  VPT_HIP(hipMalloc(dst, n));
  VPT_HIP(hipMemcpy(*dst, src, n, hipMemcpyHostToDevice));
  bytes += n;
  return VPT_OK;
}

static int upload_grid(const HostGrid& h, DeviceGrid& d) {
  d.dev = h.dev;
  int rc;
  // The stencil pool is 9 KiB per leaf (4.5x the voxels): a large sparse volume can exceed the
  // device's memory.  Say so before the first allocation instead of failing inside hipMalloc.
  const size_t need = h.cells8.size() * sizeof(int2) + h.runs8.size() + h.walk8.size() * sizeof(uint32_t) +
                      h.cells128.size() * sizeof(int2) + h.root.size() * sizeof(RootTileDev) +
                      h.bricks.size() * sizeof(float);
  size_t free_b = 0, total_b = 0;
  VPT_HIP(hipMemGetInfo(&free_b, &total_b));
  if (need > free_b)
    return set_error(VPT_E_NOMEM, "grid upload: needs " + std::to_string(need >> 20) + " MiB (" +
                                      std::to_string(h.dev.leaf_count) + " leaves x 9 KiB stencil pool + tables), " +
                                      std::to_string(free_b >> 20) + " MiB free on the device");
  if ((rc = upload(h.cells8.data(), h.cells8.size() * sizeof(int2), &d.cells8, d.bytes))) return rc;
  if ((rc = upload(h.runs8.data(), h.runs8.size(), &d.runs8, d.bytes))) return rc;
  if ((rc = upload(h.walk8.data(), h.walk8.size() * sizeof(uint32_t), &d.walk8, d.bytes))) return rc;
  d.run_fraction = h.run_fraction;
  if ((rc = upload(h.cells128.data(), h.cells128.size() * sizeof(int2), &d.cells128, d.bytes))) return rc;
  if ((rc = upload(h.root.data(), h.root.size() * sizeof(RootTileDev), &d.root, d.bytes))) return rc;
  if ((rc = upload(h.bricks.data(), h.bricks.size() * sizeof(float), &d.bricks, d.bytes))) return rc;
  d.dev.cells8 = (const int2*)d.cells8;
  d.dev.runs8 = (const uint8_t*)d.runs8;
  d.dev.walk8 = (const uint32_t*)d.walk8;
  d.dev.cells128 = (const int2*)d.cells128;
  d.dev.root = (const RootTileDev*)d.root;
  d.dev.bricks = (const float*)d.bricks;
  return VPT_OK;
}

static void free_grid(DeviceGrid& d) {
  (void)hipFree(d.cells8);
  (void)hipFree(d.runs8);
  (void)hipFree(d.walk8);
  (void)hipFree(d.cells128);
  (void)hipFree(d.root);
  (void)hipFree(d.bricks);
  d = DeviceGrid{};
}

}  // namespace vpt

namespace {

constexpr int kProfWords = 2 * vpt::PB_COUNT + vpt::PT_COUNT;
constexpr uint32_t kLaunchSlots = 64;
// Latency-bound launches: at most this many work items per wavefront of the grid (see render()).
constexpr uint64_t kSpreadLanes = 6;

int wait_ctx(vpt_gpu_ctx* ctx);

// Device copy of the scene constants, which every in-flight launch of this context reads: wait for
// the context's launches (wait_ctx), copy on the context's stream and wait for the copy (the next
// render may use another stream).
int push_scene(vpt_gpu_ctx* ctx) {
  int rc = wait_ctx(ctx);
  if (rc) return rc;
  vpt::DevScene lat = ctx->scene;
  lat.gate_min = ctx->lat_gate[0];
  lat.gate_idle = ctx->lat_gate[1];
  lat.gate_eval = ctx->lat_gate[2];
  lat.gate_walk = ctx->lat_gate[3];
  lat.wave_lanes = ctx->lat_wave_lanes;
  VPT_HIP(hipMemcpyAsync(ctx->scene_dev, &ctx->scene, sizeof(vpt::DevScene), hipMemcpyHostToDevice, ctx->stream));
  VPT_HIP(hipMemcpyAsync(ctx->scene_lat_dev, &lat, sizeof(vpt::DevScene), hipMemcpyHostToDevice, ctx->stream));
  VPT_HIP(hipStreamSynchronize(ctx->stream));
  return VPT_OK;
}

// The counter pair of the next launch on stream s: ordered after the previous launch that used the
// same ring slot (whatever stream it ran on), then zeroed on s.
int take_slot(vpt_gpu_ctx* ctx, hipStream_t s, uint32_t& slot) {
  std::lock_guard<std::mutex> lock(ctx->slot_mu);
  slot = ctx->next_slot;
  ctx->next_slot = (ctx->next_slot + 1) % kLaunchSlots;
  if (ctx->slot_used[slot]) VPT_HIP(hipStreamWaitEvent(s, ctx->slot_done[slot], 0));
  VPT_HIP(hipMemsetAsync(ctx->job_counter + 2 * slot, 0, 2 * sizeof(unsigned long long), s));
  return VPT_OK;
}

int release_slot(vpt_gpu_ctx* ctx, hipStream_t s, uint32_t slot) {
  std::lock_guard<std::mutex> lock(ctx->slot_mu);
  VPT_HIP(hipEventRecord(ctx->slot_done[slot], s));
  ctx->slot_used[slot] = true;
  return VPT_OK;
}

// Waits for every launch of this context, whatever stream it was enqueued on, and for the context's
// own stream -- not for other contexts' work on the device (a context per thread never stalls
// behind another's frames).  Each launch records its ring slot's event after its kernels
// (release_slot), and a launch that reuses a slot is ordered after the slot's previous launch
// (take_slot), so the latest event of every used slot covers all of them.
// The events are snapshotted under the lock and waited for after it is released, so a wait never
// blocks another thread's take_slot.
int wait_ctx(vpt_gpu_ctx* ctx) {
  if (ctx->open_feeds.load() > 0)
    return vpt::set_error(VPT_E_STATE, "a feed of this context is open: close it before calls that wait for the "
                                       "context's launches (ADVICE r04)");
  hipEvent_t ev[kLaunchSlots];
  uint32_t n = 0;
  {
    std::lock_guard<std::mutex> lock(ctx->slot_mu);
    for (uint32_t i = 0; i < kLaunchSlots; ++i)
      if (ctx->slot_used[i]) ev[n++] = ctx->slot_done[i];
  }
  for (uint32_t i = 0; i < n; ++i) VPT_HIP(hipEventSynchronize(ev[i]));
  if (ctx->stream) VPT_HIP(hipStreamSynchronize(ctx->stream));
  return VPT_OK;
}


void destroy(vpt_gpu_ctx* ctx) {
  if (!ctx) return;
  vpt::host::feed_pool_free(ctx);
  (void)hipSetDevice(ctx->device);
  vpt::free_grid(ctx->density);
  vpt::free_grid(ctx->temperature);
  (void)hipFree(ctx->bb);
  (void)hipFree(ctx->cie);
  (void)hipFree(ctx->film);
  (void)hipFree(ctx->job_counter);
  (void)hipFree(ctx->counters);
  (void)hipFree(ctx->prof);
  (void)hipFree(ctx->scene_dev);
  (void)hipFree(ctx->scene_lat_dev);
  (void)hipFree(ctx->order);
  (void)hipFree(ctx->perm);
  (void)hipFree(ctx->samples);
  (void)hipFree(ctx->frame_film);
  if (ctx->samples_done) (void)hipEventDestroy(ctx->samples_done);
  for (uint32_t i = 0; i < kLaunchSlots; ++i)
    if (ctx->slot_done[i]) (void)hipEventDestroy(ctx->slot_done[i]);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->staging) (void)hipHostFree(ctx->staging);
  delete ctx;
}

// The descending-cost tile ranks of ctx->tile_cost, uploaded as the job order.
int rank_tiles(vpt_gpu_ctx* ctx) {
  const uint64_t T = ctx->scene.T;
  ctx->tile_rank.resize(T);
  for (uint64_t i = 0; i < T; ++i) ctx->tile_rank[i] = (uint32_t)i;
  std::stable_sort(ctx->tile_rank.begin(), ctx->tile_rank.end(),
                   [&](uint32_t a, uint32_t b) { return ctx->tile_cost[a] > ctx->tile_cost[b]; });
  uint32_t* d = nullptr;
  VPT_HIP(hipMalloc((void**)&d, T * sizeof(uint32_t)));
  const hipError_t e = hipMemcpy(d, ctx->tile_rank.data(), T * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(d);
    return vpt::set_error(VPT_E_HIP, std::string("tile order upload: ") + hipGetErrorString(e));
  }
  (void)hipFree(ctx->order);
  ctx->order = d;
  return VPT_OK;
}

// Tile costs (vpt_tile_cost_kernel) and the descending-cost tile ranks, once per context.
int ensure_order(vpt_gpu_ctx* ctx) {
  if (ctx->order) return VPT_OK;
  const auto t0 = std::chrono::steady_clock::now();
  struct Lap {  // (the cost pass's time, vpt_gpu_setup_timings)
    vpt_gpu_ctx* c;
    std::chrono::steady_clock::time_point t0;
    ~Lap() { c->setup_ms[3] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
  } lap{ctx, t0};
  if (ctx->open_feeds.load() > 0)  // the cost pass and its copy would wait for the feed's launch
    return vpt::set_error(VPT_E_STATE, "tile costs: a feed of this context is open (compute them before)");
  const uint64_t T = ctx->scene.T;
  float* cost = nullptr;
  VPT_HIP(hipMalloc((void**)&cost, T * sizeof(float)));
  hipLaunchKernelGGL(vpt::vpt_tile_cost_kernel, dim3((unsigned)((T + 255) / 256)), dim3(256), 0, nullptr,
                     ctx->scene_dev, cost);
  ctx->tile_cost.assign(T, 0.0f);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpy(ctx->tile_cost.data(), cost, T * sizeof(float), hipMemcpyDeviceToHost);
  (void)hipFree(cost);
  if (e != hipSuccess) return vpt::set_error(VPT_E_HIP, std::string("tile cost pass: ") + hipGetErrorString(e));
  return rank_tiles(ctx);
}

// The ordered film's sample buffer for a launch of `bytes`: the context's, grown if needed.  nullptr (VPT_OK)
// when it must grow while a feed of the context is open -- freeing or allocating device memory could wait for
// the feed's launch -- and that launch then adds into the film with atomics.
int ensure_samples(vpt_gpu_ctx* ctx, uint64_t bytes, float*& out) {
  out = nullptr;
  if (ctx->samples_bytes >= bytes) {
    out = ctx->samples;
    return VPT_OK;
  }
  if (ctx->open_feeds.load() > 0) return VPT_OK;
  if (ctx->samples_used) VPT_HIP(hipEventSynchronize(ctx->samples_done));  // (ordered launches are serialised)
  if (ctx->samples) {
    (void)hipFree(ctx->samples);
    ctx->samples = nullptr;
    ctx->samples_bytes = 0;
  }
  const hipError_t e = hipMalloc((void**)&ctx->samples, bytes);
  if (e != hipSuccess) {
    ctx->samples = nullptr;
    (void)hipGetLastError();
    return vpt::set_error(VPT_E_NOMEM, "ordered film: " + std::to_string(bytes >> 20) + " MiB sample buffer: " +
                                           hipGetErrorString(e) + " (vpt_gpu_set_film_order's max_bytes splits launches)");
  }
  ctx->samples_bytes = bytes;
  out = ctx->samples;
  return VPT_OK;
}

// The largest sample buffer an ordered launch may use (bytes).
uint64_t ordered_cap(vpt_gpu_ctx* ctx, uint64_t want) {
  if (ctx->film_order_max) return ctx->film_order_max;
  if (want <= ctx->samples_bytes) return ctx->samples_bytes;
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return ctx->samples_bytes;
  return (uint64_t)(free_b + ctx->samples_bytes) / 4 * 3;
}

}  // namespace

int vpt::host::ctx_device(vpt_gpu_ctx* ctx) {
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return vpt::set_error(VPT_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
  return VPT_OK;
}

int vpt::host::launch_tile_counts(vpt_gpu_ctx* ctx, float* film, const uint32_t* counts_dev, hipStream_t s) {
  const uint64_t npix = (uint64_t)ctx->scene.W * (uint64_t)ctx->scene.H;
  hipLaunchKernelGGL(vpt::vpt_tile_count_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, s, ctx->scene_dev,
                     film, counts_dev);
  VPT_HIP(hipGetLastError());
  return VPT_OK;
}

int vpt::host::render(vpt_gpu_ctx* ctx, uint64_t jid_begin, uint64_t jid_count, float* film, float* records,
                      void* stream_ptr, vpt_event* events, uint64_t event_cap, uint32_t* slot_out,
                      const vpt::FeedLaunch* feed) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "render: null context");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if (jid_count == 0) return VPT_OK;
  if (feed && (ctx->scene.pixel_mode || records || events))
    return vpt::set_error(VPT_E_INVALID, "render: feeds run the reference RNG mode's production kernels only");
  // The ordered film: production launches of the reference RNG mode (debug launches and feeds add atomically).
  // A launch whose sample buffer would exceed the cap is rendered as consecutive launches (whole waves where it
  // can); each adds its own waves in order, so the film is the same.
  const uint64_t per_job = (uint64_t)ctx->scene.tile_area * 3 * sizeof(float);
  const bool ordered = ctx->film_order == VPT_FILM_ORDERED && !feed && !records && !events && !ctx->scene.pixel_mode;
  if (ordered) {
    const uint64_t max_jobs = std::min<uint64_t>(ordered_cap(ctx, jid_count * per_job) / per_job, 0xffffffffULL);
    if (max_jobs == 0) return vpt::set_error(VPT_E_NOMEM, "ordered film: no room for one job's samples");
    if (jid_count > max_jobs) {
      const uint64_t T = ctx->scene.T;
      const uint64_t chunk = max_jobs >= T ? max_jobs / T * T : max_jobs;
      for (uint64_t b = 0; b < jid_count; b += chunk)
        if ((rc = render(ctx, jid_begin + b, std::min(chunk, jid_count - b), film, nullptr, stream_ptr))) return rc;
      return VPT_OK;
    }
  }
  const uint64_t total = ctx->scene.T * (uint64_t)ctx->cfg.num_waves;
  (void)total;  // jids beyond num_waves are valid jobs too (TileProvider only stops at requested_waves)
  hipStream_t s = (hipStream_t)stream_ptr;  // NULL = the null stream (HIP convention)
  vpt::KernelArgs env{};
  env.jid_begin = jid_begin;
  env.jid_count = jid_count;
  env.pixel_chunk = 1;
  if (ctx->scene.pixel_mode) {  // work items are chunks of pixel_chunk pixels of one job
    const uint64_t area = ctx->scene.tile_area;
    if (jid_count > UINT64_MAX / area) return vpt::set_error(VPT_E_INVALID, "render: job range too large");
    const uint64_t items = jid_count * area;
    // One work item per pixel makes every pixel a device-wide atomic on the launch's job counter, and a
    // wavefront's fetches then serialise there (C3: 530 M pixels, 546 ms vs 348 in the reference mode,
    // r03zf).  Pixels are taken pixel_chunk at a time: the largest power of two dividing the tile area that
    // still leaves >= 32 chunks per resident lane (C3 / C5: 32 pixels; C2, C1: 1 -- C2 ran 41.6 ms with 1
    // pixel per item, 43.7 with 4, r03zg), or the vpt_gpu_set_pixel_chunk value.  Every pixel keeps its own
    // stream: samples do not depend on it.
    uint64_t K = 1;
    if (ctx->pixel_chunk > 0) {
      K = (uint64_t)ctx->pixel_chunk;
    } else {
      const uint64_t lanes = (uint64_t)ctx->grid_blocks * vpt::kBlockThreads;
      while (area % (2 * K) == 0 && items / (2 * K) >= 32 * lanes) K *= 2;
    }
    env.pixel_chunk = (uint32_t)K;
    env.jid_count = items / K;
  }
  env.film = film ? film : ctx->film;
  env.records = records;
  env.tile_area = ctx->scene.tw * ctx->scene.th;
  env.prof_buf = ctx->prof;
  env.order = nullptr;
  env.perm = nullptr;
  env.order_tail_k0 = 0;
  env.order_tail_n = 0;
  env.order_group = vpt::kOrderGroup;
  // Partly filled launches (a few work items per resident lane: small frames, few waves, a GPU's share
  // of a frame dealt over several): a launch lasts as long as its slowest jobs, and a job's lane runs
  // faster with fewer waves per SIMD, so the grid is sized to round(1 + 1.8 x) blocks per CU (at most
  // the resident capacity), x = items per resident lane.  Same jobs, same samples.  Measured (r03h,
  // profiles/archive/r03h_grid_sweep.txt; C3 frames of spp waves, 4 / 5 / 6 / 7 blocks per CU, ms): spp 16
  // (x 1.1) 54.5 / 55.0 / 55.4 / 57.5 (3: 51.5); spp 24 (x 1.7) 57.3 / 61.0 / 64.7 / 65.7; spp 32
  // (x 2.3, the 8-GPU share) 70.4 / 66.9 / 67.5 / 71.2; spp 48 (x 3.4) 92.2 / 90.8 / 89.7 / 87.9; from
  // spp 96 on (and C5's shares) the full grid is best.  C2 (262 144 jobs, x 0.57 -> 2 blocks per CU,
  // r02g: 1 / 1.5 / 1.75 / 2 / 2.5 / 3 / 4 / 5 blocks per CU 167.7 / 124.4 / 112.9 / 98.7-99.3 / 104.4 /
  // 104.5-105.3 / 106.7 / 109.9 ms).  (r02's rule, ~2 items per lane, gave 7 blocks from x 1.9 on.)
  uint32_t blocks = (uint32_t)ctx->grid_blocks;
  // Latency-bound launch (at most kSpreadLanes items per wavefront of the grid, e.g. C1's 4 096 jobs):
  // the launch lasts as long as its slowest job, and a job runs fastest on a wavefront with few other
  // paths (the wavefront executes every block any of its lanes needs).  Such a launch keeps the whole
  // grid, the first ~items / wavefronts lanes of each wavefront take the jobs, and it runs with the
  // latency gates (every block runs for one lane).  Measured, C1 (r02): 43.3 ms (256 blocks x 64
  // lanes) -> 20.5 ms (1 792 blocks, one lane per wavefront, gates 1:65:1:1).  Same jobs, same samples.
  const bool latency = env.jid_count <= kSpreadLanes * ((uint64_t)blocks * (vpt::kBlockThreads / 64));
  const uint64_t cus = (uint64_t)ctx->cus;
  if (!ctx->grid_user && !latency) {
    const uint64_t resident_per_cu = std::max<uint64_t>(1, blocks / cus);
    const double x = (double)env.jid_count / ((double)blocks * vpt::kBlockThreads);  // items per resident lane
    const uint64_t per_cu = std::min<uint64_t>(resident_per_cu, (uint64_t)std::max(1.0, std::floor(1.5 + 1.8 * x)));
    blocks = (uint32_t)std::min<uint64_t>(blocks, cus * per_cu);
  }
#ifdef VPT_JOB_LOG
  const bool temp = ctx->scene.has_temperature != 0, dbg = events != nullptr;  // records = the job log
#else
  const bool temp = ctx->scene.has_temperature != 0, dbg = records != nullptr || events != nullptr;
#endif
  // The latency kernel (lane cold state in VGPRs, VPT_WAVES_LAT waves per SIMD) for launches that fill at
  // most its resident grid anyway: latency-bound ones on its whole grid with the latency gates (C1 20.7-21.2
  // -> 19.2-19.7 ms, r04e / r04z), and partly filled ones whose rule above gives <= lat_per_cu blocks per CU
  // with the context's gates (C2 100.0-101.3 -> 95.7-96.6 ms, the 8-GPU C3 share of 32 waves 66.1-66.6 ->
  // 65.1-65.3; with the latency gates they ran slower, 108.3-109.8 / 75.2-76.1 ms: its one-lane blocks add
  // wave instructions to launches that are issue-bound; r04k, profiles/archive/r04k_lat_gated_ab.txt).  lat_mode 1
  // forces it.  Same jobs, same samples.
  const uint64_t lat_blocks = cus * (uint64_t)ctx->lat_per_cu;
  const bool use_lat = !dbg && !feed && ctx->lat_mode != 0 &&
                       (ctx->lat_mode == 1 || (!ctx->grid_user && (latency || blocks <= lat_blocks)));
  if (use_lat) blocks = (uint32_t)std::min<uint64_t>(latency ? lat_blocks : blocks, lat_blocks);
  // Live-path compaction (vpt_gpu_set_compaction): partly filled launches of the latency kernel whose grid fits
  // the compacting kernel's occupancy (its LDS exchange: 2 blocks per CU; C2 runs 2).
  const bool compact = use_lat && !latency && ctx->compact_every > 0 &&
                       (uint64_t)blocks <= cus * (uint64_t)std::max(0, ctx->compact_per_cu);
  const uint64_t T = ctx->scene.T;
  if (!feed && ctx->order_mode != VPT_ORDER_JID && jid_begin % T == 0 && jid_count % T == 0 && jid_count < (1ULL << 32)) {
    // whole waves: take the jobs in cost order (same jobs, same samples)
    if ((rc = ensure_order(ctx))) return rc;
    const uint32_t n = (uint32_t)(jid_count / T);
    uint32_t tail = 0;  // VPT_ORDER_COST_WAVE_MAJOR
    // Same-tile order only where each sample has a slot of its own (the ordered film): with film atomics a
    // wavefront's 64 lanes would add to one pixel at once.  And not in partly filled launches (a few jobs per
    // lane, the latency kernel with the context's gates), which last as long as their costliest jobs: r06ze, C2
    // 98.1-98.5 vs 96.4-96.9 ms, C3's 8-GPU share (32 waves) 65.0-65.7 vs 62.6-63.6 with the cost tail.  Full
    // launches: C3 321.8-322.0 vs 334.3-334.5 ms, C4 71.0-71.2 vs 80.2-80.7 (profiles/r06ze_same_tile_ab.txt).
    const bool same_tile = ctx->order_mode == VPT_ORDER_COST_SAME_TILE && ordered && !ctx->frame_waves &&
                           !(use_lat && !latency);
    if (ctx->order_mode == VPT_ORDER_COST_TILE_MAJOR || same_tile) tail = n;
    if (same_tile) env.order_group = 1;
    if (ctx->order_mode == VPT_ORDER_COST_TAIL || (ctx->order_mode == VPT_ORDER_COST_SAME_TILE && !same_tile)) {
      // the last ~6 x (resident lanes / T) waves (C3: 61 of 256): measured best of 2x..16x
      const uint64_t lanes = (uint64_t)blocks * vpt::kBlockThreads;
      const uint64_t want = ctx->order_tail_waves > 0 ? (uint64_t)ctx->order_tail_waves : (6 * lanes + T - 1) / T;
      tail = (uint32_t)std::min<uint64_t>(n, want);
    }
    env.order = ctx->order;
    env.order_tail_n = tail;
    env.order_tail_k0 = (n - tail) * (uint32_t)T;
  }
  if (!feed && ctx->perm && ctx->perm_n == jid_count && !ctx->scene.pixel_mode) env.perm = ctx->perm;
  float* samples = nullptr;
  // (while the drop-in's ordered frame is open its feeds own the sample buffer: other launches add with atomics)
  if (ordered && !ctx->frame_waves && (rc = ensure_samples(ctx, jid_count * per_job, samples))) return rc;
  env.samples = samples;
  if (samples) {
    ++ctx->ordered_launches;
    if (ctx->samples_used) VPT_HIP(hipStreamWaitEvent(s, ctx->samples_done, 0));  // the buffer's previous launch
  } else if (!feed) {
    ++ctx->atomic_launches;
  }
  uint32_t slot = 0;
  if ((rc = take_slot(ctx, s, slot))) return rc;
  env.job_counter = ctx->job_counter + 2 * slot;
  env.events = events;
  env.feed_word = feed ? feed->word : nullptr;
  env.feed_ring = feed ? feed->ring : nullptr;
  env.feed_mask = feed ? feed->mask : 0;
  env.feed_error = feed ? feed->error : nullptr;
  env.feed_started = feed ? feed->started : nullptr;
  env.feed_waiting = feed ? feed->waiting : nullptr;
  env.feed_hint_mask = (uint32_t)(vpt::kHintSlots - 1);
  env.tile_done = feed ? feed->tile_done : nullptr;
  env.frame = feed && ctx->frame_waves ? ctx->samples : nullptr;  // (the drop-in's ordered frame, vpt_gpu_frame_open)
  env.frame_w0 = ctx->frame_jid_lo / ctx->scene.T;
  env.frame_slots = env.frame ? ctx->frame_waves * ctx->frame_tiles : 0;
  env.frame_tile_lo = ctx->frame_tile_lo;
  env.frame_tiles = ctx->frame_tiles;
  env.compact_every = 0;
  env.event_count = ctx->job_counter + 2 * slot + 1;
  env.event_cap = event_cap;
  if (slot_out) *slot_out = slot;
  // (a compacting launch reads the context's scene, whose wave_lanes is 64: a path moved into another thread's
  // slot must be able to fetch there -- with fewer fetching lanes per wavefront, live paths packed into the
  // first slots would leave the fetching slots to finished ones)
  const vpt::DevScene* scene =
      latency || (use_lat && ctx->lat_ungated && !compact) ? ctx->scene_lat_dev : ctx->scene_dev;
  if (use_lat) {
    env.compact_every = (uint32_t)std::max(1, ctx->compact_every);
    if (compact) {
      auto kernel = temp ? vpt::vpt_integrate_kernel<true, false, false, true, true>
                         : ctx->use_runs ? vpt::vpt_integrate_kernel<false, false, true, true, true>
                                         : vpt::vpt_integrate_kernel<false, false, false, true, true>;
      hipLaunchKernelGGL(kernel, dim3(blocks), dim3(vpt::kBlockThreads), vpt::kXchgBytes, s, env, scene, ctx->counters);
    } else {
      auto kernel = temp ? vpt::vpt_integrate_kernel<true, false, false, true>
                         : ctx->use_runs ? vpt::vpt_integrate_kernel<false, false, true, true>
                                         : vpt::vpt_integrate_kernel<false, false, false, true>;
      hipLaunchKernelGGL(kernel, dim3(blocks), dim3(vpt::kBlockThreads), 0, s, env, scene, ctx->counters);
    }
  } else if (feed) {  // (never a debug launch: no records or events)
    auto kernel = temp ? vpt::vpt_integrate_kernel<true, false, false, false, false, true>
                       : ctx->use_runs ? vpt::vpt_integrate_kernel<false, false, true, false, false, true>
                                       : vpt::vpt_integrate_kernel<false, false, false, false, false, true>;
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(vpt::kBlockThreads), 0, s, env, scene, ctx->counters);
  } else {
    auto kernel = temp ? (dbg ? vpt::vpt_integrate_kernel<true, true, false> : vpt::vpt_integrate_kernel<true, false, false>)
                       : ctx->use_runs
                           ? (dbg ? vpt::vpt_integrate_kernel<false, true, true> : vpt::vpt_integrate_kernel<false, false, true>)
                           : (dbg ? vpt::vpt_integrate_kernel<false, true, false> : vpt::vpt_integrate_kernel<false, false, false>);
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(vpt::kBlockThreads), 0, s, env, scene, ctx->counters);
  }
  VPT_HIP(hipGetLastError());
  const uint64_t npix = (uint64_t)ctx->scene.W * (uint64_t)ctx->scene.H;
  if (samples) {  // the film, pixel by pixel in wave order (sample counts included)
    const uint64_t threads = ctx->scene.T * (uint64_t)ctx->scene.tile_area;
    hipLaunchKernelGGL(vpt::vpt_film_order_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                       ctx->scene_dev, env.film, samples, jid_begin, jid_count);
    VPT_HIP(hipGetLastError());
    VPT_HIP(hipEventRecord(ctx->samples_done, s));
    ctx->samples_used = true;
  } else if (!feed) {  // a feed adds its sample counts when it is closed (vpt_tile_count_kernel)
    hipLaunchKernelGGL(vpt::vpt_count_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, s, ctx->scene_dev,
                       env.film, jid_begin, jid_count);
    VPT_HIP(hipGetLastError());
  }
  return release_slot(ctx, s, slot);
}

extern "C" {

const char* vpt_last_error(void) { return vpt::g_last_error.c_str(); }
int vpt_abi_version(void) { return VPT_ABI_VERSION; }

int vpt_gpu_device_count(int* count) {
  if (!count) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_device_count: null argument");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return VPT_OK;
}

int vpt_gpu_find_seeds(int device, uint32_t out0, uint32_t out1, uint32_t* seeds, int max_seeds, int* n_found) {
  if (!n_found || max_seeds < 0 || (max_seeds > 0 && !seeds))
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_find_seeds: bad argument");
  *n_found = 0;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return vpt::set_error(VPT_E_HIP, "vpt_gpu_find_seeds: no HIP device");
  if (device < 0 || device >= ndev) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_find_seeds: bad device index");
  VPT_HIP(hipSetDevice(device));
  constexpr uint32_t kCap = 64, kPerThread = 1024, kThreads = 256;
  hipStream_t s = nullptr;
  VPT_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint32_t* d = nullptr;
  uint32_t host[kCap + 1] = {};
  hipError_t e = hipMalloc((void**)&d, (kCap + 1) * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemsetAsync(d, 0, (kCap + 1) * sizeof(uint32_t), s);
  if (e == hipSuccess) {
    const uint64_t blocks = ((1ULL << 32) / kPerThread + kThreads - 1) / kThreads;
    hipLaunchKernelGGL(vpt::vpt_seed_search_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s, out0, out1, kPerThread,
                       d + 1, d, kCap);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(host, d, sizeof host, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(d);
  (void)hipStreamDestroy(s);
  if (e != hipSuccess) return vpt::set_error(VPT_E_HIP, std::string("vpt_gpu_find_seeds: ") + hipGetErrorString(e));
  const uint32_t n = std::min(host[0], kCap);
  std::sort(host + 1, host + 1 + n);
  for (uint32_t i = 0; i < n && (int)i < max_seeds; ++i) seeds[i] = host[1 + i];
  *n_found = (int)host[0];
  return VPT_OK;
}

}  // extern "C"

// The host side of Volume::Volume: the grids flattened (leaf-slot and walk tables, the stencil pool) with the
// density's majorants fixed for interpolation (volume.cpp:162-170; temperature is only sampled) -- the ABI's
// vpt_host_grids (vpt_grids_flatten), uploaded by create_on.
struct vpt_host_grids {
  vpt::HostGrid density, temperature;
  bool has_temperature = false;
  vpt::ValueRange temp_range;  // the temperature grid's value extremes (blackbody_rows_suffice)
  double flatten_ms = 0;
};

namespace {
using HostGrids = vpt_host_grids;
// ms[0] += the time taken.
int build_grids(const vpt_grid_desc* density, const vpt_grid_desc* temperature, HostGrids& g, double* ms) {
  const auto t0 = std::chrono::steady_clock::now();
  // The temperature grid is flattened on a thread of its own beside the density's: each build has serial
  // stretches (node sets, leaf loops) and page-faults its fresh tables in (vpt_last_error is per thread: the
  // temperature's message is carried back).
  int trc = VPT_OK;
  std::string tmsg;
  std::thread temp_build;
  if (temperature)
    temp_build = std::thread([&] {
      if ((trc = vpt::build_host_grid(*temperature, false, 0, g.temperature)))
        tmsg = vpt_last_error();
      else
        g.temp_range = vpt::value_range(*temperature, 0);
    });
  int rc = vpt::build_host_grid(*density, true, 0, g.density);
  if (rc == VPT_OK) vpt::compute_runs(g.density, 0);
  if (temp_build.joinable()) temp_build.join();
  if (rc) return rc;
  if (trc) return vpt::set_error(trc, tmsg);
  g.has_temperature = temperature != nullptr;
  if (ms) *ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return VPT_OK;
}

// A context on `device` from grids already flattened (vpt_gpu_create, vpt_gpu_create_many).
int create_on(const vpt_configuration* cfg, const HostGrids& grids, const float* blackbody_500x3, int device,
              vpt_gpu_ctx** out) {
  *out = nullptr;
  std::unique_ptr<vpt_gpu_ctx, void (*)(vpt_gpu_ctx*)> ctx(new vpt_gpu_ctx(), destroy);
  ctx->device = device;
  ctx->cfg = *cfg;
  ctx->setup_ms[0] = grids.flatten_ms;
  using clk = std::chrono::steady_clock;
  auto t = clk::now();
  auto lap = [&](int i) {  // setup phases (vpt_gpu_setup_timings)
    const auto now = clk::now();
    ctx->setup_ms[i] += std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
  };
  int rc = ctx_device(ctx.get());
  if (rc) return rc;
  lap(4);
  if ((rc = vpt::build_scene(*cfg, ctx->scene))) return rc;
  if ((rc = vpt::upload_grid(grids.density, ctx->density))) return rc;
  if (grids.has_temperature && (rc = vpt::upload_grid(grids.temperature, ctx->temperature))) return rc;
  lap(1);
  const bool has_temperature = grids.has_temperature;
  // The run-skipping kernel variant is for grids with large equal-majorant regions (C2's constant
  // cube: 36 % of the interior cells have run radius >= 2; the 512^3 cloud: 4 %, where the variant
  // would cost more than it skips).  vpt_gpu_set_run_skipping overrides the choice.
  ctx->use_runs = !has_temperature && ctx->density.run_fraction >= VPT_RUNS_MIN_FRACTION;
  ctx->scene.density = ctx->density.dev;
  vpt::scene_finalize(ctx->scene);  // uses only the density map (host copy of the values)
  ctx->scene.temperature = ctx->temperature.dev;
  ctx->scene.has_temperature = has_temperature ? 1 : 0;
  ctx->scene.bb_lds_ok = has_temperature ? vpt::blackbody_rows_suffice(grids.temp_range, cfg->volume_parameters.temperature_scale,
                                                                    cfg->volume_parameters.temperature_offset, vpt::kBbLdsRows)
                                     : 0;

  std::vector<float> bb(501 * 3, 0.0f);  // row 500 = 0 (reference reads past its table)
  if (blackbody_500x3)
    std::memcpy(bb.data(), blackbody_500x3, 500 * 3 * sizeof(float));
  else
    vpt::blackbody_table(bb.data());
  size_t scratch = 0;
  if ((rc = vpt::upload(bb.data(), bb.size() * sizeof(float), (void**)&ctx->bb, scratch))) return rc;
  if ((rc = vpt::upload(vpt::cie_table(), 471 * 3 * sizeof(float), (void**)&ctx->cie, scratch))) return rc;
  ctx->scene.bb = ctx->bb;
  ctx->scene.cie = ctx->cie;

  ctx->film_count = (uint64_t)cfg->output_size[0] * (uint64_t)cfg->output_size[1] * 4;
  VPT_HIP(hipMalloc((void**)&ctx->film, ctx->film_count * sizeof(float)));
  VPT_HIP(hipMemset(ctx->film, 0, ctx->film_count * sizeof(float)));
  VPT_HIP(hipMalloc((void**)&ctx->job_counter, kLaunchSlots * 2 * sizeof(unsigned long long)));  // jobs, events
  for (uint32_t i = 0; i < kLaunchSlots; ++i)
    VPT_HIP(hipEventCreateWithFlags(&ctx->slot_done[i], hipEventDisableTiming));
  VPT_HIP(hipMalloc((void**)&ctx->counters, vpt::kCounterCount * sizeof(unsigned long long)));
  VPT_HIP(hipMemset(ctx->counters, 0, vpt::kCounterCount * sizeof(unsigned long long)));
  VPT_HIP(hipMalloc((void**)&ctx->prof, kProfWords * sizeof(unsigned long long)));
  VPT_HIP(hipMemset(ctx->prof, 0, kProfWords * sizeof(unsigned long long)));
  VPT_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
  VPT_HIP(hipEventCreateWithFlags(&ctx->samples_done, hipEventDisableTiming));

  // Persistent grid: as many blocks as are resident at once.
  int per_cu = 0, cus = 0;
  // sized for the production kernel of this scene; the debug variant is launched with the same grid
  VPT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &per_cu, has_temperature ? vpt::vpt_integrate_kernel<true, false, false>
                           : (ctx->use_runs ? vpt::vpt_integrate_kernel<false, false, true> : vpt::vpt_integrate_kernel<false, false, false>),
      vpt::kBlockThreads, 0));
  VPT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  if (per_cu < 1) per_cu = 1;
  ctx->grid_blocks = per_cu * cus;
  int lat_per_cu = 0;
  VPT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &lat_per_cu, has_temperature ? vpt::vpt_integrate_kernel<true, false, false, true>
                               : (ctx->use_runs ? vpt::vpt_integrate_kernel<false, false, true, true>
                                                : vpt::vpt_integrate_kernel<false, false, false, true>),
      vpt::kBlockThreads, 0));
  ctx->lat_per_cu = std::max(1, std::min(lat_per_cu, per_cu));
  int compact_per_cu = 0;
  VPT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &compact_per_cu, has_temperature ? vpt::vpt_integrate_kernel<true, false, false, true, true>
                                   : (ctx->use_runs ? vpt::vpt_integrate_kernel<false, false, true, true, true>
                                                    : vpt::vpt_integrate_kernel<false, false, false, true, true>),
      vpt::kBlockThreads, vpt::kXchgBytes));
  ctx->compact_per_cu = compact_per_cu;
  ctx->cus = cus > 0 ? cus : 1;
  // Scheduling defaults from tools/tune.py sweeps on MI355X (C3, 256 spp): rare states run for >= 6
  // waiting lanes, density evaluations (with the deferred exact draw) for >= 36, everything runs when
  // < 8 lanes are walking; the walk loops while >= 4 lanes walk (r02 sweep: 6:8:36:4 363.7 ms vs
  // 6:12:32:4 366.6 ms, C4 103.7 vs 104.4).  The temperature kernel's rare blocks wait for 8 lanes since the film
  // regroup (C4 83.3-83.6 vs 83.9-84.3 ms over 4 alternating runs, profiles/archive/r05gates2_c4_gate_min.txt).
  ctx->scene.gate_min = has_temperature ? 8 : 6;
  // The temperature kernel runs its rare blocks at any count only once no lane walks (same-tile order; C4 at
  // gate_idle 8 / 4 / 2 / 1: 67.2-67.4 / 64.2-64.3 / 62.8 / 61.5 ms, profiles/r06zj_c4_gates.txt,
  // r06zk_gates_idle.txt).  (C3 measured 317.7 ms at 4 vs 321.9 at 8, but the density kernel's partly filled
  // launches -- C2, a GPU's share -- read the same gates and were tuned at 8: not changed.)
  ctx->scene.gate_idle = has_temperature ? 1 : 8;
  ctx->scene.gate_eval = 36;
  // The temperature kernel's walk loops while any lane walks (gate_walk 1) since the same-tile order: C4 67.3-67.8
  // ms vs 71.1-71.3 at 4, best of 3 twice (r06zg, profiles/r06zg_gates_same_tile.txt); C3 stays at 4 (1-3: flat).
  ctx->scene.gate_walk = has_temperature ? 1 : 4;
  ctx->scene.pixel_mode = 0;
  ctx->scene.wave_lanes = 64;
  ctx->scene.tile_area = (uint32_t)(ctx->scene.tw * ctx->scene.th);
  VPT_HIP(hipMalloc((void**)&ctx->scene_dev, sizeof(vpt::DevScene)));
  VPT_HIP(hipMalloc((void**)&ctx->scene_lat_dev, sizeof(vpt::DevScene)));
  if ((rc = push_scene(ctx.get()))) return rc;
  lap(2);
  *out = ctx.release();
  return VPT_OK;
}

int check_device(int device, const char* what) {
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0)
    return vpt::set_error(VPT_E_HIP, std::string(what) + ": no HIP device (the integrator has no CPU fallback)");
  if (device < 0 || device >= ndev) return vpt::set_error(VPT_E_INVALID, std::string(what) + ": bad device index");
  return VPT_OK;
}
}  // namespace

extern "C" {

int vpt_gpu_create(const vpt_configuration* cfg, const vpt_grid_desc* density, const vpt_grid_desc* temperature,
                   const float* blackbody_500x3, int device, vpt_gpu_ctx** out) {
  if (!cfg || !density || !out) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_create: null argument");
  *out = nullptr;
  if (int rc = check_device(device, "vpt_gpu_create")) return rc;
  HostGrids g;
  if (int rc = build_grids(density, temperature, g, &g.flatten_ms)) return rc;
  return create_on(cfg, g, blackbody_500x3, device, out);
}

int vpt_gpu_create_many(const vpt_configuration* cfg, const vpt_grid_desc* density, const vpt_grid_desc* temperature,
                        const float* blackbody_500x3, const int* devices, int n, vpt_gpu_ctx** out) {
  if (!cfg || !density || !out || !devices || n <= 0) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_create_many: bad argument");
  for (int i = 0; i < n; ++i) out[i] = nullptr;
  for (int i = 0; i < n; ++i)
    if (int rc = check_device(devices[i], "vpt_gpu_create_many")) return rc;
  vpt_host_grids* g = nullptr;
  if (int rc = vpt_grids_flatten(density, temperature, &g)) return rc;
  const int rc = vpt_gpu_create_from(cfg, g, blackbody_500x3, devices, n, out);
  vpt_grids_free(g);
  return rc;
}

int vpt_grids_flatten(const vpt_grid_desc* density, const vpt_grid_desc* temperature, vpt_host_grids** out) {
  if (!density || !out) return vpt::set_error(VPT_E_INVALID, "vpt_grids_flatten: null argument");
  *out = nullptr;
  std::unique_ptr<vpt_host_grids> g(new vpt_host_grids());
  if (int rc = build_grids(density, temperature, *g, &g->flatten_ms)) return rc;
  *out = g.release();
  return VPT_OK;
}

void vpt_grids_free(vpt_host_grids* grids) { delete grids; }

int vpt_gpu_create_from(const vpt_configuration* cfg, const vpt_host_grids* grids, const float* blackbody_500x3,
                        const int* devices, int n, vpt_gpu_ctx** out) {
  if (!cfg || !grids || !out || !devices || n <= 0) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_create_from: bad argument");
  for (int i = 0; i < n; ++i) out[i] = nullptr;
  for (int i = 0; i < n; ++i)
    if (int rc = check_device(devices[i], "vpt_gpu_create_from")) return rc;
  // one thread per device: each uploads the same host grids (vpt_last_error is per thread: the first failure's
  // message is carried back)
  std::vector<int> rcs((size_t)n, VPT_OK);
  std::vector<std::string> msgs((size_t)n);
  std::vector<std::thread> pool;
  for (int i = 0; i < n; ++i)
    pool.emplace_back([&, i] {
      rcs[(size_t)i] = create_on(cfg, *grids, blackbody_500x3, devices[i], &out[i]);
      if (rcs[(size_t)i]) msgs[(size_t)i] = vpt_last_error();
    });
  for (auto& th : pool) th.join();
  for (int i = 0; i < n; ++i)
    if (rcs[(size_t)i]) {
      for (int k = 0; k < n; ++k) {
        destroy(out[k]);
        out[k] = nullptr;
      }
      return vpt::set_error(rcs[(size_t)i], "device " + std::to_string(devices[i]) + ": " + msgs[(size_t)i]);
    }
  return VPT_OK;
}

int vpt_gpu_setup_timings(const vpt_gpu_ctx* ctx, double* ms, int n) {
  if (!ctx || !ms || n < 0) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_setup_timings: bad argument");
  for (int i = 0; i < n && i < 5; ++i) ms[i] = ctx->setup_ms[i];
  return VPT_OK;
}

int vpt_gpu_destroy(vpt_gpu_ctx* ctx) {
  destroy(ctx);
  return VPT_OK;
}

int vpt_gpu_job_space(const vpt_gpu_ctx* ctx, uint64_t* jobs_per_wave, uint64_t* total_jobs) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  if (jobs_per_wave) *jobs_per_wave = ctx->scene.T;
  if (total_jobs) *total_jobs = ctx->scene.T * (uint64_t)ctx->cfg.num_waves;
  return VPT_OK;
}

int vpt_gpu_render_jobs(vpt_gpu_ctx* ctx, uint64_t jid_begin, uint64_t jid_count, float* film_device,
                        void* hip_stream) {
  return render(ctx, jid_begin, jid_count, film_device, nullptr, hip_stream);
}

int vpt_gpu_render_jobs_records(vpt_gpu_ctx* ctx, uint64_t jid_begin, uint64_t jid_count, float* film_device,
                                float* records_device, void* hip_stream) {
  return render(ctx, jid_begin, jid_count, film_device, records_device, hip_stream);
}

int vpt_gpu_trace_jobs(vpt_gpu_ctx* ctx, uint64_t jid_begin, uint64_t jid_count, float* film_device,
                       vpt_event* events_device, uint64_t capacity, uint64_t* count, void* hip_stream) {
  if (!ctx || !events_device || !count) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_trace_jobs: null argument");
  *count = 0;
  uint32_t slot = 0;
  int rc = render(ctx, jid_begin, jid_count, film_device, nullptr, hip_stream, events_device, capacity, &slot);
  if (rc) return rc;
  if (jid_count == 0) return VPT_OK;
  unsigned long long n = 0;
  VPT_HIP(hipMemcpyAsync(&n, ctx->job_counter + 2 * slot + 1, sizeof n, hipMemcpyDeviceToHost, (hipStream_t)hip_stream));
  VPT_HIP(hipStreamSynchronize((hipStream_t)hip_stream));
  *count = n;
  return VPT_OK;
}

int vpt_gpu_majorant_trace(vpt_gpu_ctx* ctx, const float origin[3], const float direction[3], float* rows_host,
                           int max_rows, int* n_rows) {
  if (!ctx || !origin || !direction || !n_rows || (max_rows > 0 && !rows_host) || max_rows < 0)
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_majorant_trace: bad argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  float* rows = nullptr;
  int* n = nullptr;
  VPT_HIP(hipMalloc((void**)&rows, (size_t)(max_rows > 0 ? max_rows : 1) * 9 * sizeof(float)));
  if (hipMalloc((void**)&n, sizeof(int)) != hipSuccess) {
    (void)hipFree(rows);
    return vpt::set_error(VPT_E_HIP, "vpt_gpu_majorant_trace: hipMalloc failed");
  }
  hipLaunchKernelGGL(vpt::vpt_majorant_trace_kernel, dim3(1), dim3(64), 0, nullptr, ctx->scene_dev, origin[0],
                     origin[1], origin[2], direction[0], direction[1], direction[2], rows, max_rows, n);
  hipError_t e = hipGetLastError();
  int nn = 0;
  if (e == hipSuccess) e = hipMemcpy(&nn, n, sizeof nn, hipMemcpyDeviceToHost);
  if (e == hipSuccess && max_rows > 0)
    e = hipMemcpy(rows_host, rows, (size_t)std::min(nn, max_rows) * 9 * sizeof(float), hipMemcpyDeviceToHost);
  (void)hipFree(rows);
  (void)hipFree(n);
  if (e != hipSuccess) return vpt::set_error(VPT_E_HIP, std::string("vpt_gpu_majorant_trace: ") + hipGetErrorString(e));
  *n_rows = nn;
  return VPT_OK;
}

int vpt_gpu_set_rng_mode(vpt_gpu_ctx* ctx, int mode) {
  if (!ctx || (mode != VPT_RNG_REFERENCE && mode != VPT_RNG_PIXEL))
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_rng_mode: bad argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if (mode == VPT_RNG_PIXEL && (int64_t)ctx->scene.tw * ctx->scene.th >= (int64_t)vpt::kPixelTaken)
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_rng_mode: tile too large for the pixel mode");
  ctx->scene.pixel_mode = mode == VPT_RNG_PIXEL ? 1 : 0;
  ctx->scene.tile_area = (uint32_t)(ctx->scene.tw * ctx->scene.th);
  return push_scene(ctx);
}

int vpt_gpu_set_pixel_chunk(vpt_gpu_ctx* ctx, int chunk) {
  if (!ctx || chunk < 0 || (chunk & (chunk - 1)) != 0 || (chunk > 0 && ctx->scene.tile_area % (uint32_t)chunk != 0))
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_pixel_chunk: 0 or a power of two dividing the tile area");
  ctx->pixel_chunk = chunk;  // read by the next render's host code only: no wait
  return VPT_OK;
}

int vpt_gpu_set_run_skipping(vpt_gpu_ctx* ctx, int mode) {
  if (!ctx || mode < -1 || mode > 1) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_run_skipping: bad argument");
  if (mode == 1 && ctx->scene.has_temperature)
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_run_skipping: no run-skipping variant with a temperature grid");
  ctx->use_runs = mode < 0 ? (!ctx->scene.has_temperature && ctx->density.run_fraction >= VPT_RUNS_MIN_FRACTION) : mode == 1;
  return VPT_OK;
}

int vpt_gpu_kernel_variant(const vpt_gpu_ctx* ctx, int* has_temperature, int* run_skipping) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  if (has_temperature) *has_temperature = ctx->scene.has_temperature ? 1 : 0;
  if (run_skipping) *run_skipping = ctx->use_runs ? 1 : 0;
  return VPT_OK;
}

int vpt_gpu_set_film_order(vpt_gpu_ctx* ctx, int mode, uint64_t max_bytes) {
  if (!ctx || (mode != VPT_FILM_ATOMIC && mode != VPT_FILM_ORDERED))
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_film_order: bad argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  ctx->film_order = mode;
  ctx->film_order_max = max_bytes;
  if (mode == VPT_FILM_ATOMIC && ctx->samples && ctx->open_feeds.load() == 0) {  // the buffer is not needed
    if (ctx->samples_used) VPT_HIP(hipEventSynchronize(ctx->samples_done));
    (void)hipFree(ctx->samples);
    ctx->samples = nullptr;
    ctx->samples_bytes = 0;
  }
  return VPT_OK;
}

int vpt_gpu_film_order_info(const vpt_gpu_ctx* ctx, int* mode, uint64_t* buffer_bytes, uint64_t* ordered_launches,
                            uint64_t* atomic_launches) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  if (mode) *mode = ctx->film_order;
  if (buffer_bytes) *buffer_bytes = ctx->samples_bytes;
  if (ordered_launches) *ordered_launches = ctx->ordered_launches;
  if (atomic_launches) *atomic_launches = ctx->atomic_launches;
  return VPT_OK;
}

int vpt_gpu_set_job_order(vpt_gpu_ctx* ctx, int mode) {
  if (!ctx || mode < VPT_ORDER_JID || mode > VPT_ORDER_COST_SAME_TILE)
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_job_order: bad argument");
  ctx->order_mode = mode;
  return VPT_OK;
}

int vpt_gpu_set_job_order_tail(vpt_gpu_ctx* ctx, int waves) {
  if (!ctx || waves < 0) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_job_order_tail: bad argument");
  ctx->order_tail_waves = waves;
  return VPT_OK;
}

int vpt_gpu_tile_costs(vpt_gpu_ctx* ctx, float* cost, uint32_t* rank) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if ((rc = ensure_order(ctx))) return rc;
  if (cost) std::memcpy(cost, ctx->tile_cost.data(), ctx->tile_cost.size() * sizeof(float));
  if (rank) std::memcpy(rank, ctx->tile_rank.data(), ctx->tile_rank.size() * sizeof(uint32_t));
  return VPT_OK;
}

int vpt_gpu_set_tile_costs(vpt_gpu_ctx* ctx, const float* cost) {
  if (!ctx || !cost) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_tile_costs: null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  for (uint64_t i = 0; i < ctx->scene.T; ++i)  // NaN would break the sort's strict weak ordering
    if (!std::isfinite(cost[i])) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_tile_costs: non-finite cost");
  if ((rc = wait_ctx(ctx))) return rc;  // in-flight launches read the current order
  ctx->tile_cost.assign(cost, cost + ctx->scene.T);
  return rank_tiles(ctx);
}

int vpt_gpu_set_job_permutation(vpt_gpu_ctx* ctx, const uint32_t* perm, uint64_t n) {
  if (!ctx || (n && !perm)) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_job_permutation: null argument");
  if (n >= (1ULL << 32)) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_job_permutation: too many jobs");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  std::vector<uint8_t> seen(n, 0);
  for (uint64_t i = 0; i < n; ++i) {
    if (perm[i] >= n || seen[perm[i]]) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_job_permutation: not a permutation");
    seen[perm[i]] = 1;
  }
  if ((rc = wait_ctx(ctx))) return rc;  // in-flight launches may read the current one
  (void)hipFree(ctx->perm);
  ctx->perm = nullptr;
  ctx->perm_n = 0;
  if (n == 0) return VPT_OK;
  VPT_HIP(hipMalloc((void**)&ctx->perm, n * sizeof(uint32_t)));
  VPT_HIP(hipMemcpy(ctx->perm, perm, n * sizeof(uint32_t), hipMemcpyHostToDevice));
  ctx->perm_n = n;
  return VPT_OK;
}

int vpt_gpu_sync(vpt_gpu_ctx* ctx) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  return wait_ctx(ctx);
}

int vpt_gpu_stream_create(vpt_gpu_ctx* ctx, void** hip_stream) {
  if (!ctx || !hip_stream) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_stream_create: null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  hipStream_t s = nullptr;
  VPT_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *hip_stream = s;
  return VPT_OK;
}

int vpt_gpu_bind_thread_near(vpt_gpu_ctx* ctx, int* node_out) {
  if (node_out) *node_out = -1;
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_bind_thread_near: null context");
  char bus[64] = {};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, ctx->device) != hipSuccess) return VPT_OK;
  for (char* c = bus; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
  int node = -1;
  {
    std::ifstream in(std::string("/sys/bus/pci/devices/") + bus + "/numa_node");
    if (!(in >> node) || node < 0) return VPT_OK;
  }
  std::ifstream in("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string list;
  if (!std::getline(in, list)) return VPT_OK;
  // Allowed: the process's CPUs (its main thread's set: taskset / numactl restrict it), not this thread's own --
  // a thread inherits its creator's set, and a caller bound to the far node would otherwise pin its helpers
  // there too (r05n: a taker on node 1 made the pusher it started run there).
  cpu_set_t cur, near;
  CPU_ZERO(&near);
  if (sched_getaffinity(getpid(), sizeof cur, &cur) != 0) return VPT_OK;
  // "0-63,128-191"
  for (size_t pos = 0; pos < list.size();) {
    size_t end = list.find(',', pos);
    if (end == std::string::npos) end = list.size();
    const std::string r = list.substr(pos, end - pos);
    const size_t dash = r.find('-');
    const int a = std::atoi(r.c_str()), b = dash == std::string::npos ? a : std::atoi(r.c_str() + dash + 1);
    for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
      if (c >= 0 && CPU_ISSET(c, &cur)) CPU_SET(c, &near);
    pos = end + 1;
  }
  if (CPU_COUNT(&near) == 0) return VPT_OK;
  if (pthread_setaffinity_np(pthread_self(), sizeof near, &near) != 0) return VPT_OK;
  if (node_out) *node_out = node;
  return VPT_OK;
}

int vpt_gpu_stream_destroy(vpt_gpu_ctx* ctx, void* hip_stream) {
  if (!ctx || !hip_stream) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_stream_destroy: null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  VPT_HIP(hipStreamDestroy((hipStream_t)hip_stream));
  return VPT_OK;
}

int vpt_gpu_stream_sync(vpt_gpu_ctx* ctx, void* hip_stream) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_stream_sync: null context");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  VPT_HIP(hipStreamSynchronize((hipStream_t)hip_stream));
  return VPT_OK;
}

int vpt_gpu_film_alloc(vpt_gpu_ctx* ctx, float** film_device) {
  if (!ctx || !film_device) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_film_alloc: null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  float* f = nullptr;
  VPT_HIP(hipMalloc((void**)&f, ctx->film_count * sizeof(float)));
  const hipError_t e = hipMemset(f, 0, ctx->film_count * sizeof(float));
  if (e != hipSuccess) {
    (void)hipFree(f);
    return vpt::set_error(VPT_E_HIP, std::string("vpt_gpu_film_alloc: ") + hipGetErrorString(e));
  }
  *film_device = f;
  return VPT_OK;
}

int vpt_gpu_film_free(vpt_gpu_ctx* ctx, float* film_device) {
  if (!ctx || !film_device || film_device == ctx->film)
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_film_free: not a film from vpt_gpu_film_alloc");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  VPT_HIP(hipFree(film_device));
  return VPT_OK;
}

// The largest ordered-frame buffer (the 4K, 1 024-spp C5 frame on one GPU needs 102 GB).
constexpr uint64_t kFrameMaxBytes = 128ULL << 30;

int vpt_gpu_frame_open(vpt_gpu_ctx* ctx, uint64_t jid_lo, uint64_t* waves_io, uint32_t tile_lo, uint32_t tile_hi) {
  if (!ctx || !waves_io) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_frame_open: null argument");
  uint64_t waves = *waves_io;
  *waves_io = 0;
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if (ctx->open_feeds.load() > 0)  // (allocating could wait for a running feed's launch)
    return vpt::set_error(VPT_E_STATE, "vpt_gpu_frame_open: a feed of the context is open");
  const vpt::DevScene& S = ctx->scene;
  if (S.pixel_mode) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_frame_open: frames run the reference RNG mode");
  ctx->frame_waves = 0;
  if (waves == 0) return VPT_OK;
  if (tile_lo >= tile_hi || tile_hi > S.T) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_frame_open: bad tile range");
  const uint64_t per_wave = (uint64_t)(tile_hi - tile_lo) * (uint64_t)S.tile_area * 3 * sizeof(float);
  // as many of the waves asked for as fit 3/4 of the device's free memory (the buffer already held counted in), at
  // most kFrameMaxBytes
  size_t free_b = 0, total_b = 0;
  VPT_HIP(hipMemGetInfo(&free_b, &total_b));
  const uint64_t avail = std::min<uint64_t>(kFrameMaxBytes, (uint64_t)free_b / 4 * 3 + ctx->samples_bytes);
  waves = std::min<uint64_t>(waves, avail / per_wave);
  if (waves == 0) return vpt::set_error(VPT_E_NOMEM, "vpt_gpu_frame_open: not one wave of the frame fits the device");
  if (ctx->samples_used) VPT_HIP(hipEventSynchronize(ctx->samples_done));  // (an ordered launch's film pass)
  float* buf = nullptr;
  if ((rc = ensure_samples(ctx, waves * per_wave, buf))) return rc;
  if (!buf) return vpt::set_error(VPT_E_STATE, "vpt_gpu_frame_open: the sample buffer cannot grow now");
  if (!ctx->frame_film) VPT_HIP(hipMalloc((void**)&ctx->frame_film, ctx->film_count * sizeof(float)));
  if (!ctx->staging) VPT_HIP(hipHostMalloc((void**)&ctx->staging, ctx->film_count * sizeof(float), hipHostMallocDefault));
  ctx->frame_jid_lo = jid_lo;
  ctx->frame_tile_lo = tile_lo;
  ctx->frame_tiles = tile_hi - tile_lo;
  ctx->frame_waves = waves;
  *waves_io = waves;
  return VPT_OK;
}

int vpt_gpu_frame_finish(vpt_gpu_ctx* ctx, uint64_t jid_end, const float* prior, float* film_host) {
  if (!ctx || !film_host) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_frame_finish: null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  const uint64_t waves = ctx->frame_waves, lo = ctx->frame_jid_lo;
  if (!waves) return VPT_OK;  // no frame open
  ctx->frame_waves = 0;       // (closed, whatever follows)
  const vpt::DevScene& S = ctx->scene;
  const uint64_t w0 = lo / S.T;
  if (jid_end < lo || (jid_end > lo && (jid_end - 1) / S.T - w0 >= waves))
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_frame_finish: jobs beyond the frame's waves");
  if (ctx->open_feeds.load() > 0) return vpt::set_error(VPT_E_STATE, "vpt_gpu_frame_finish: a feed of the context is open");
  if (jid_end == lo) return VPT_OK;
  const size_t bytes = ctx->film_count * sizeof(float);
  if (prior)
    VPT_HIP(hipMemcpyAsync(ctx->frame_film, prior, bytes, hipMemcpyHostToDevice, ctx->stream));
  else
    VPT_HIP(hipMemsetAsync(ctx->frame_film, 0, bytes, ctx->stream));
  const uint32_t tile_lo = ctx->frame_tile_lo, tiles = ctx->frame_tiles, tile_hi = tile_lo + tiles;
  const uint64_t threads = (uint64_t)tiles * (uint64_t)S.tile_area;
  hipLaunchKernelGGL(vpt::vpt_frame_order_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, ctx->stream,
                     ctx->scene_dev, ctx->frame_film, ctx->samples, w0, tile_lo, tiles, lo, jid_end);
  VPT_HIP(hipGetLastError());
  VPT_HIP(hipEventRecord(ctx->samples_done, ctx->stream));  // (the next ordered launch waits for this pass)
  ctx->samples_used = true;
  VPT_HIP(hipMemcpyAsync(ctx->staging, ctx->frame_film, bytes, hipMemcpyDeviceToHost, ctx->stream));
  VPT_HIP(hipStreamSynchronize(ctx->stream));
  // the tiles' pixels into the host film, one contiguous run per image row and tile row (tiles are row-major)
  const uint64_t W = (uint64_t)S.W;
  auto put = [&](uint64_t y, uint64_t x0, uint64_t x1) {
    std::memcpy(film_host + (y * W + x0) * 4, ctx->staging + (y * W + x0) * 4, (x1 - x0) * 4 * sizeof(float));
  };
  if (S.single_pixel_enabled) {  // only that pixel has samples (worker.cpp:113-116)
    if (S.sp_x >= 0 && S.sp_y >= 0 && S.sp_x < S.W && S.sp_y < S.H) {
      const uint64_t t = (uint64_t)(S.sp_y / S.th) * S.ntx + (uint64_t)(S.sp_x / S.tw);
      if (t >= tile_lo && t < tile_hi) put((uint64_t)S.sp_y, (uint64_t)S.sp_x, (uint64_t)S.sp_x + 1);
    }
    return VPT_OK;
  }
  // image row y's run of the band: the band's tiles in tile row y / th (tiles are row-major)
  const uint64_t ntx = (uint64_t)S.ntx, y0 = tile_lo / ntx * (uint64_t)S.th,
                 y1 = std::min<uint64_t>((tile_hi + ntx - 1) / ntx * (uint64_t)S.th, (uint64_t)S.H);
  auto rows = [&](uint64_t ya, uint64_t yb) {
    for (uint64_t y = ya; y < yb; ++y) {
      const uint64_t ty = y / (uint64_t)S.th;
      const uint64_t a = std::max<uint64_t>(tile_lo, ty * ntx) - ty * ntx, b = std::min<uint64_t>(tile_hi, (ty + 1) * ntx) - ty * ntx;
      if (a < b) put(y, a * (uint64_t)S.tw, std::min<uint64_t>(b * (uint64_t)S.tw, W));
    }
  };
  const uint64_t nt = (y1 - y0) * W < (1u << 18) ? 1 : 8;  // (a 1080p film: 33 MB, copied by 8 threads)
  std::vector<std::thread> pool;
  for (uint64_t i = 1; i < nt; ++i) pool.emplace_back(rows, y0 + (y1 - y0) * i / nt, y0 + (y1 - y0) * (i + 1) / nt);
  rows(y0, y0 + (y1 - y0) / nt);
  for (auto& t : pool) t.join();
  return VPT_OK;
}

int vpt_gpu_film_flush_to_host(vpt_gpu_ctx* ctx, float* film_device, float* film_host) {
  if (!ctx || !film_host) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_film_flush_to_host: null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  float* f = film_device ? film_device : ctx->film;
  const size_t bytes = ctx->film_count * sizeof(float);
  if (!ctx->staging) VPT_HIP(hipHostMalloc((void**)&ctx->staging, bytes, hipHostMallocDefault));
  VPT_HIP(hipMemcpyAsync(ctx->staging, f, bytes, hipMemcpyDeviceToHost, ctx->stream));
  VPT_HIP(hipMemsetAsync(f, 0, bytes, ctx->stream));
  VPT_HIP(hipStreamSynchronize(ctx->stream));
  const float* src = ctx->staging;
  for (uint64_t i = 0; i < ctx->film_count; ++i) film_host[i] += src[i];
  return VPT_OK;
}

}  // extern "C"

extern "C" {

int vpt_gpu_film_clear(vpt_gpu_ctx* ctx) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if ((rc = wait_ctx(ctx))) return rc;  // renders into the film may be in flight on any stream
  VPT_HIP(hipMemsetAsync(ctx->film, 0, ctx->film_count * sizeof(float), ctx->stream));
  VPT_HIP(hipStreamSynchronize(ctx->stream));
  return VPT_OK;
}

int vpt_gpu_film_device_ptr(vpt_gpu_ctx* ctx, float** film_device, uint64_t* count) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  if (film_device) *film_device = ctx->film;
  if (count) *count = ctx->film_count;
  return VPT_OK;
}

int vpt_gpu_film_add_to_host(vpt_gpu_ctx* ctx, float* film_host) {
  if (!ctx || !film_host) return vpt::set_error(VPT_E_INVALID, "null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if ((rc = wait_ctx(ctx))) return rc;
  std::vector<float> tmp(ctx->film_count);
  VPT_HIP(hipMemcpy(tmp.data(), ctx->film, ctx->film_count * sizeof(float), hipMemcpyDeviceToHost));
  for (uint64_t i = 0; i < ctx->film_count; ++i) film_host[i] += tmp[i];
  return VPT_OK;
}

int vpt_gpu_counters(vpt_gpu_ctx* ctx, vpt_counters* out, int reset) {
  if (!ctx || !out) return vpt::set_error(VPT_E_INVALID, "null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if ((rc = wait_ctx(ctx))) return rc;
  unsigned long long c[vpt::kCounterCount];
  VPT_HIP(hipMemcpy(c, ctx->counters, sizeof c, hipMemcpyDeviceToHost));
  uint64_t* o = reinterpret_cast<uint64_t*>(out);
  for (int i = 0; i < vpt::kCounterCount; ++i) o[i] = c[i];
  if (reset) VPT_HIP(hipMemset(ctx->counters, 0, sizeof c));
  return VPT_OK;
}

int vpt_gpu_set_tuning(vpt_gpu_ctx* ctx, int gate_min, int gate_idle, int grid_blocks, int gate_eval, int gate_walk) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  // gate_idle >= 1 is what guarantees progress: with no lane walking, every waiting block runs.
  if (gate_idle == 0) return vpt::set_error(VPT_E_INVALID, "gate_idle must be >= 1 (0 can stall a wavefront)");
  if (gate_eval > 0) ctx->scene.gate_eval = gate_eval;
  if (gate_walk >= 0) ctx->scene.gate_walk = gate_walk;
  if (gate_min > 0) ctx->scene.gate_min = gate_min;
  if (gate_idle >= 0) ctx->scene.gate_idle = gate_idle;
  if ((rc = push_scene(ctx))) return rc;
  if (grid_blocks > 0) {
    ctx->grid_blocks = grid_blocks;
    ctx->grid_user = true;
  }
  return VPT_OK;
}

int vpt_gpu_set_latency_tuning(vpt_gpu_ctx* ctx, int wave_lanes, int gate_min, int gate_idle, int gate_eval,
                               int gate_walk) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  if (wave_lanes > 64) return vpt::set_error(VPT_E_INVALID, "wave_lanes must be <= 64");
  if (gate_idle == 0) return vpt::set_error(VPT_E_INVALID, "gate_idle must be >= 1 (0 can stall a wavefront)");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if (wave_lanes >= 0) ctx->lat_wave_lanes = wave_lanes;
  if (gate_min > 0) ctx->lat_gate[0] = gate_min;
  if (gate_idle >= 0) ctx->lat_gate[1] = gate_idle;
  if (gate_eval > 0) ctx->lat_gate[2] = gate_eval;
  if (gate_walk >= 0) ctx->lat_gate[3] = gate_walk;
  return push_scene(ctx);
}

int vpt_gpu_set_latency_kernel(vpt_gpu_ctx* ctx, int mode, int ungated) {
  if (!ctx || mode < -1 || mode > 1 || ungated < -1 || ungated > 1)
    return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_latency_kernel: bad argument");
  ctx->lat_mode = mode;  // read by the next render's host code only: no wait
  if (ungated >= 0) ctx->lat_ungated = ungated;
  return VPT_OK;
}

int vpt_gpu_profile(vpt_gpu_ctx* ctx, uint64_t* out, int n, int reset) {
  if (!ctx || !out) return vpt::set_error(VPT_E_INVALID, "null argument");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  if ((rc = wait_ctx(ctx))) return rc;
  std::vector<unsigned long long> v(kProfWords);
  VPT_HIP(hipMemcpy(v.data(), ctx->prof, v.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  if (n < (int)v.size()) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_profile: output too small");
  for (size_t i = 0; i < v.size(); ++i) out[i] = v[i];
  if (reset) VPT_HIP(hipMemset(ctx->prof, 0, v.size() * sizeof(unsigned long long)));
  return VPT_OK;
}

int vpt_gpu_launch_info(const vpt_gpu_ctx* ctx, int* grid_blocks, int* block_threads) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  if (grid_blocks) *grid_blocks = ctx->grid_blocks;
  if (block_threads) *block_threads = vpt::kBlockThreads;
  return VPT_OK;
}

int vpt_gpu_set_compaction(vpt_gpu_ctx* ctx, int every) {
  if (!ctx || every < 0) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_set_compaction: bad argument");
  ctx->compact_every = every;  // read by the next render's host code only: no wait
  return VPT_OK;
}

int vpt_gpu_latency_kernel_info(const vpt_gpu_ctx* ctx, int* mode, int* resident_blocks_per_cu) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "null context");
  if (mode) *mode = ctx->lat_mode;
  if (resident_blocks_per_cu) *resident_blocks_per_cu = ctx->lat_per_cu;
  return VPT_OK;
}

}  // extern "C"
