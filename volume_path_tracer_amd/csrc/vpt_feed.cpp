// vpt_feed.cpp — feeds (include/vpt_gpu.h vpt_gpu_feed_*): one running launch of the production kernel that
// renders the job ids the host pushes, through a host-pinned ring; the host side of the protocol whose device
// side is KernelEnvT::fetch_feed (vpt_kernels.h).  Staged feeds copy their film and per-tile counts out with the
// copy engines beside the launch (snapshots, collect).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "vpt_ctx.h"

using vpt::host::ctx_device;
using vpt::host::render;

namespace {
constexpr double kFeedHostWaitS = 120.0;  // a push waiting this long for a ring slot gives up
constexpr size_t kZeroBytes = 4u << 20;   // the context's pinned zeros (staged feeds' clears)

// VPT_FEED_TRACE=1: one stderr line per feed event (open / launch / close / a push's wait for a ring slot /
// snapshots / the end of its work), milliseconds since the first event -- for diagnosing a drop-in's protocol.
void feed_trace(const vpt_gpu_feed* f, const char* what, double a = 0, double b = 0) {
  static const bool on = std::getenv("VPT_FEED_TRACE") && std::atoi(std::getenv("VPT_FEED_TRACE")) > 0;
  if (!on) return;
  static const auto t0 = std::chrono::steady_clock::now();
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::fprintf(stderr, "feed %10.2f ms %p %-8s %.0f %.0f\n", ms, (const void*)f, what, a, b);
}

void feed_free(vpt_gpu_feed* f) {
  if (!f) return;
  (void)hipSetDevice(f->ctx->device);
  if (f->closed_ev) (void)hipEventDestroy(f->closed_ev);
  if (f->copy_stream) (void)hipStreamDestroy(f->copy_stream);
  if (f->own_stream) (void)hipStreamDestroy(f->own_stream);
  (void)hipHostFree(f->block);
  if (f->pin_film) (void)hipHostFree(f->pin_film);
  if (f->pin_done) (void)hipHostFree(f->pin_done);
  (void)hipFree(f->done_dev);
  delete f;
}

}  // namespace

void vpt::host::feed_pool_free(vpt_gpu_ctx* ctx) {
  for (vpt_gpu_feed* f : ctx->feed_pool) feed_free(f);
  ctx->feed_pool.clear();
  if (ctx->zeros) (void)hipHostFree(ctx->zeros);
  ctx->zeros = nullptr;
}

namespace {

// Publishes items [0, published) and, with close, the end of the feed (release: the ring and count
// stores are visible to the GPU before the word that publishes them).
void feed_publish(vpt_gpu_feed* f, bool close) {
  __atomic_store_n(f->word, f->published | (close ? vpt::kFeedClosed : 0), __ATOMIC_RELEASE);
}

// Zeroes `bytes` of device memory with host-to-device copies of the context's pinned zeros, enqueued on s:
// copy-engine work, which runs while another launch holds every CU (a fill kernel would wait for it).
int clear_by_copy(vpt_gpu_ctx* ctx, void* dev, size_t bytes, hipStream_t s) {
  if (!ctx->zeros) {
    VPT_HIP(hipHostMalloc((void**)&ctx->zeros, kZeroBytes, hipHostMallocDefault));
    std::memset(ctx->zeros, 0, kZeroBytes);
  }
  for (size_t off = 0; off < bytes; off += kZeroBytes)
    VPT_HIP(hipMemcpyAsync(static_cast<char*>(dev) + off, ctx->zeros, std::min(kZeroBytes, bytes - off),
                           hipMemcpyHostToDevice, s));
  return VPT_OK;
}

// The resources of a feed of ring size cap (and, staged, its copy-out buffers), from the context's pool or new.
int feed_get(vpt_gpu_ctx* ctx, uint64_t cap, bool stage, std::unique_ptr<vpt_gpu_feed, void (*)(vpt_gpu_feed*)>& f) {
  for (size_t i = 0; i < ctx->feed_pool.size(); ++i)
    if (ctx->feed_pool[i]->cap == cap && (!stage || ctx->feed_pool[i]->done_dev)) {  // a pooled feed of this window
      f.reset(ctx->feed_pool[i]);
      ctx->feed_pool.erase(ctx->feed_pool.begin() + (ptrdiff_t)i);
      return VPT_OK;
    }
  f.reset(new vpt_gpu_feed());
  f->ctx = ctx;
  f->cap = cap;
  const uint64_t T = ctx->scene.T;
  const size_t bytes = (vpt::kFeedHeaderWords + cap) * sizeof(uint64_t) + T * sizeof(uint32_t);
  VPT_HIP(hipHostMalloc((void**)&f->block, bytes, hipHostMallocCoherent | hipHostMallocMapped));
  f->word = f->block;
  f->error = reinterpret_cast<uint32_t*>(f->block + 1);
  f->started = f->block + 4;
  f->waiting = f->block + 2;
  f->ring = f->block + vpt::kFeedHeaderWords;
  f->counts = reinterpret_cast<uint32_t*>(f->ring + cap);
  VPT_HIP(hipEventCreateWithFlags(&f->closed_ev, hipEventDisableTiming));
  if (stage) {
    VPT_HIP(hipMalloc((void**)&f->done_dev, T * sizeof(uint32_t)));
    VPT_HIP(hipHostMalloc((void**)&f->pin_film, ctx->film_count * sizeof(float), hipHostMallocDefault));
    VPT_HIP(hipHostMalloc((void**)&f->pin_done, T * sizeof(uint32_t), hipHostMallocDefault));
    VPT_HIP(hipStreamCreateWithFlags(&f->copy_stream, hipStreamNonBlocking));
    VPT_HIP(hipStreamCreateWithFlags(&f->own_stream, hipStreamNonBlocking));
    f->shown.assign(ctx->film_count, 0.0f);
    f->shown_done.assign(T, 0u);
    if (int rc = clear_by_copy(ctx, f->done_dev, T * sizeof(uint32_t), f->copy_stream)) return rc;
    VPT_HIP(hipStreamSynchronize(f->copy_stream));
  }
  return VPT_OK;
}

uint64_t feed_cap(const vpt_gpu_ctx* ctx, uint64_t window) {
  // The ring holds at least twice the launch's lanes: a lane reserves an item only while some are
  // published, so reservations lead the consumed items by at most the lanes, and the host keeps pushing
  // while the lanes it has already fed work (C3: 458 752 lanes, ring 2^20).
  const uint64_t lanes = (uint64_t)ctx->grid_blocks * vpt::kBlockThreads;
  uint64_t cap = 1024;
  while ((cap < window || cap < 2 * lanes) && cap < (1ULL << 26)) cap <<= 1;
  return cap;
}
}  // namespace

namespace {
int feed_open(vpt_gpu_ctx* ctx, float* film_device, void* hip_stream, uint64_t window, bool stage, vpt_gpu_feed** out) {
  if (!ctx || !out || (!hip_stream && !stage)) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_open: null argument");
  *out = nullptr;
  if (ctx->scene.pixel_mode) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_open: feeds run the reference RNG mode");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  const uint64_t cap = feed_cap(ctx, window);
  std::unique_ptr<vpt_gpu_feed, void (*)(vpt_gpu_feed*)> f(nullptr, feed_free);
  if ((rc = feed_get(ctx, cap, stage, f))) return rc;
  f->stage = stage;
  f->stream = hip_stream ? (hipStream_t)hip_stream : f->own_stream;  // (staged: the feed's own stream if none)
  f->film = film_device ? film_device : ctx->film;
  f->published = 0;
  f->started_seen = 0;
  f->started_moved = {};
  f->closed = false;
  f->counted = false;
  if (!f->ring_clean)
    for (uint64_t i = 0; i < cap; ++i) f->ring[i] = vpt::kFeedEmpty;
  f->ring_clean = false;
  std::memset(f->counts, 0, ctx->scene.T * sizeof(uint32_t));
  __atomic_store_n(f->error, 0u, __ATOMIC_RELAXED);
  for (uint64_t i = 0; i < vpt::kHintSlots; ++i) __atomic_store_n(f->started + i, 0ULL, __ATOMIC_RELAXED);
  __atomic_store_n(f->waiting, 0ULL, __ATOMIC_RELAXED);
  __atomic_store_n(f->word, 0ULL, __ATOMIC_RELEASE);
  uint64_t* word_dev = nullptr;
  VPT_HIP(hipHostGetDevicePointer((void**)&word_dev, f->word, 0));
  f->fl = vpt::FeedLaunch{word_dev, word_dev + vpt::kFeedHeaderWords, cap - 1, reinterpret_cast<unsigned*>(word_dev + 1),
                          word_dev + 4, word_dev + 2,
                          stage ? f->done_dev : nullptr};
  // The launch is deferred until the ring holds as many items as it has lanes (or the feed is closed):
  // launched at once, its idle wavefronts would poll the host link for work (r04).
  f->launched = false;
  f->launch_at = (uint64_t)ctx->grid_blocks * vpt::kBlockThreads;
  // (With the urgent-fetch gate, launching at 1/4 or 1/16 of the lanes no longer stalls, but gains nothing
  // measurable either: C3 368.6-372.7 vs 368.4-376.2 ms, C4 116-137 vs 117-134; r05u2.)
  // (Launching at a quarter or a sixteenth of the lanes saved nothing and stalled: lanes racing past the
  // published count hold items their waves serve late, and the wrapping ring waits for them; r05k.)
  feed_trace(f.get(), stage ? "open_stg" : "open", (double)cap, (double)(uintptr_t)hip_stream);
  *out = f.release();
  return VPT_OK;
}

int feed_launch(vpt_gpu_feed* f) {
  if (f->launched) return VPT_OK;
  f->launched = true;
  if (!f->closed) {  // launched and open: it holds the device until it is closed
    ++f->ctx->open_feeds;
    f->counted = true;
  }
  feed_trace(f, "launch", (double)f->published);
  return render(f->ctx, 0, ~0ULL >> 1, f->film, nullptr, f->stream, nullptr, 0, nullptr, &f->fl);
}

// film_host += (the staged feed's film and per-tile counts as copied to pin_film / pin_done) - (what was added
// before), rows split over a few threads; shown := the copy.  Counts are integers (exact); the radiance
// channels telescope to the final film (the first add onto zero is exact).
void add_delta(vpt_gpu_feed* f, float* film_host) {
  const vpt::DevScene& S = f->ctx->scene;
  const uint64_t T = S.T;
  std::vector<uint32_t> dc(T);
  for (uint64_t t = 0; t < T; ++t) {
    // (a copy taken beside the launch reads memory, not the dirty L2 lines: it may lag, never lead; the max
    // keeps the counts monotone should an older value be read after a newer one)
    const uint32_t now = std::max(f->pin_done[t], f->shown_done[t]);
    dc[t] = now - f->shown_done[t];
    f->shown_done[t] = now;
  }
  auto rows = [&](int32_t y0, int32_t y1) {
    for (int32_t y = y0; y < y1; ++y) {
      const uint32_t* dct = dc.data() + (uint64_t)(y / S.th) * S.ntx;
      for (int32_t x = 0; x < S.W; ++x) {
        const uint64_t p = ((uint64_t)y * (uint64_t)S.W + (uint64_t)x) * 4;
        const bool counted = !S.single_pixel_enabled || (x == S.sp_x && y == S.sp_y);
        for (int c = 0; c < 3; ++c) {
          const float v = f->pin_film[p + c];
          film_host[p + c] += v - f->shown[p + c];
          f->shown[p + c] = v;
        }
        if (counted) film_host[p + 3] += (float)dct[x / S.tw];
      }
    }
  };
  const int32_t H = S.H;
  const unsigned hw = std::thread::hardware_concurrency();
  const int nt = (int)std::max(1u, std::min(8u, hw ? hw : 1u));
  if (nt == 1 || (uint64_t)S.W * (uint64_t)H < (1u << 16)) {
    rows(0, H);
    return;
  }
  std::vector<std::thread> pool;
  for (int i = 1; i < nt; ++i) pool.emplace_back(rows, (int32_t)((int64_t)H * i / nt), (int32_t)((int64_t)H * (i + 1) / nt));
  rows(0, (int32_t)((int64_t)H / nt));
  for (auto& t : pool) t.join();
}

// Copies a staged feed's film and per-tile counts with the copy engines and adds what is new into film_host.
// after_end: ordered after the feed's launch (exact); else beside it (what it has completed so far).
int feed_snapshot(vpt_gpu_feed* f, float* film_host, bool after_end, const std::function<int()>& then = {}) {
  vpt_gpu_ctx* ctx = f->ctx;
  if (after_end) VPT_HIP(hipStreamWaitEvent(f->copy_stream, f->closed_ev, 0));
  // counts first: a job counted here has added its samples before (in its lane's order)
  feed_trace(f, after_end ? "final0" : "snap0");
  VPT_HIP(hipMemcpyAsync(f->pin_done, f->done_dev, ctx->scene.T * sizeof(uint32_t), hipMemcpyDeviceToHost, f->copy_stream));
  VPT_HIP(hipMemcpyAsync(f->pin_film, f->film, ctx->film_count * sizeof(float), hipMemcpyDeviceToHost, f->copy_stream));
  hipEvent_t copied = nullptr;
  VPT_HIP(hipEventCreateWithFlags(&copied, hipEventDisableTiming));
  hipError_t e = hipEventRecord(copied, f->copy_stream);
  int rc = VPT_OK;
  if (e == hipSuccess && then) rc = then();  // queued after the copy: runs while the host adds it
  if (e == hipSuccess) e = hipEventSynchronize(copied);
  (void)hipEventDestroy(copied);
  if (e != hipSuccess) return vpt::set_error(VPT_E_HIP, std::string("feed snapshot copy: ") + hipGetErrorString(e));
  if (rc) return rc;
  feed_trace(f, "copied");
  add_delta(f, film_host);
  feed_trace(f, after_end ? "final" : "snapshot");
  return VPT_OK;
}

// Waits for a closed feed's work; a staged feed then adds its film into film_host (when given) and clears its
// film and counts for the next use.  The feed goes back to the context's pool unless a HIP failure leaves its
// launch possibly still reading the block (then it leaks).
int feed_finish(vpt_gpu_feed* f, float* film_host) {
  bool complete = false;
  int rc = VPT_OK;
  feed_trace(f, "wait", (double)f->published);
  const hipError_t e = hipEventSynchronize(f->closed_ev);
  if (e != hipSuccess)
    rc = vpt::set_error(VPT_E_HIP, std::string("vpt_gpu_feed_destroy: ") + hipGetErrorString(e));
  else
    complete = true;
  feed_trace(f, "ended", (double)f->published, complete ? (double)__atomic_load_n(f->error, __ATOMIC_ACQUIRE) : -1.0);
  if (complete && __atomic_load_n(f->error, __ATOMIC_ACQUIRE))
    rc = vpt::set_error(VPT_E_STATE, "vpt_gpu_feed_destroy: lanes of the feed's launch gave up waiting for jobs");
  if (complete && f->stage) {
    vpt_gpu_ctx* ctx = f->ctx;
    // the final copy; then the film and counts back to zero (copy engines, queued behind the copy on the same
    // stream) while the host adds the copy; nothing shown afterwards
    auto clear = [&] {
      int r = clear_by_copy(ctx, f->film, ctx->film_count * sizeof(float), f->copy_stream);
      return r ? r : clear_by_copy(ctx, f->done_dev, ctx->scene.T * sizeof(uint32_t), f->copy_stream);
    };
    if (rc == VPT_OK && film_host) {
      rc = feed_snapshot(f, film_host, true, clear);
    } else {
      const int r = clear();
      if (rc == VPT_OK) rc = r;
    }
    if (hipStreamSynchronize(f->copy_stream) != hipSuccess && rc == VPT_OK)
      rc = vpt::set_error(VPT_E_HIP, "vpt_gpu_feed_collect: clearing the film failed");
    std::fill(f->shown.begin(), f->shown.end(), 0.0f);
    std::fill(f->shown_done.begin(), f->shown_done.end(), 0u);
    feed_trace(f, "cleared");
  }
  // a completed feed's lanes marked every published slot empty (unpublished ones still are)
  f->ring_clean = complete && rc == VPT_OK;
  if (complete) f->ctx->feed_pool.push_back(f);
  return rc;
}
}  // namespace

extern "C" {

int vpt_gpu_feed_open(vpt_gpu_ctx* ctx, float* film_device, void* hip_stream, uint64_t window, vpt_gpu_feed** out) {
  return feed_open(ctx, film_device, hip_stream, window, false, out);
}

int vpt_gpu_feed_open_staged(vpt_gpu_ctx* ctx, float* film_device, void* hip_stream, uint64_t window,
                             vpt_gpu_feed** out) {
  return feed_open(ctx, film_device, hip_stream, window, true, out);
}

int vpt_gpu_feed_prepare(vpt_gpu_ctx* ctx, uint64_t window, int staged) {
  if (!ctx) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_prepare: null context");
  int rc = ctx_device(ctx);
  if (rc) return rc;
  std::unique_ptr<vpt_gpu_feed, void (*)(vpt_gpu_feed*)> f(nullptr, feed_free);
  if ((rc = feed_get(ctx, feed_cap(ctx, window), staged != 0, f))) return rc;
  if (staged && (rc = clear_by_copy(ctx, ctx->zeros, 0, f->copy_stream))) return rc;  // (allocates the zeros)
  ctx->feed_pool.push_back(f.release());
  return VPT_OK;
}

int vpt_gpu_feed_push(vpt_gpu_feed* f, const uint64_t* jids, uint64_t n) {
  if (!f || (n && !jids)) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_push: null argument");
  if (f->closed) return vpt::set_error(VPT_E_STATE, "vpt_gpu_feed_push: the feed is closed");
  const uint64_t T = f->ctx->scene.T, mask = f->cap - 1;
  const bool count = !f->stage;  // (a staged feed's launch counts its completed jobs itself)
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t jid = jids[i];
    if (jid >> 62) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_push: job id out of range");
    // The ring's lines were last written by the lanes (their empty marks): each is a miss in the host's
    // caches, so they are fetched 32 lines ahead (r05: the pusher, not the provider, bounded C4's drain).
    if ((f->published & 7) == 0) __builtin_prefetch(f->ring + ((f->published + 256) & mask), 1);
    uint64_t* slot = f->ring + (f->published & mask);
    if (__atomic_load_n(slot, __ATOMIC_ACQUIRE) != vpt::kFeedEmpty) {
      // the window is full (cap items published and not yet started): publish what we have, then wait --
      // spinning first (slots free at the GPU's job rate, tens of millions a second: a sleep between
      // checks would hold the lanes back), sleeping once the wait is long (a launch not yet started).  The
      // limit counts from the start of this wait, not of the call.
      feed_publish(f, false);
      if (int rc = feed_launch(f)) return rc;
      const auto w0 = std::chrono::steady_clock::now();
      for (uint32_t spins = 0; __atomic_load_n(slot, __ATOMIC_ACQUIRE) != vpt::kFeedEmpty; ++spins) {
        if (spins < (1u << 16)) continue;
        std::this_thread::sleep_for(std::chrono::microseconds(20));
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count() > kFeedHostWaitS)
          return vpt::set_error(VPT_E_STATE, "vpt_gpu_feed_push: the feed's launch stopped taking jobs");
      }
      const double waited = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
      if (waited > 1.0) feed_trace(f, "slotwait", (double)f->published, waited);
    }
    *slot = jid;
    if (count) ++f->counts[jid % T];
    ++f->published;
  }
  feed_publish(f, false);
  if (f->published >= f->launch_at)
    if (int rc = feed_launch(f)) return rc;
  return VPT_OK;
}

constexpr std::chrono::milliseconds kStaleHints{10};

int vpt_gpu_feed_backlog(vpt_gpu_feed* f, uint64_t* backlog) {
  if (!f || !backlog) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_backlog: null argument");
  // the newest reported reservation (the lanes' posted writes may land out of order: keep the largest)
  uint64_t s = 0;  // the largest reported reservation (each slot only grows between two of its writes)
  for (uint64_t i = 0; i < vpt::kHintSlots; ++i) s = std::max(s, __atomic_load_n(f->started + i, __ATOMIC_RELAXED));
  const auto now = std::chrono::steady_clock::now();
  if (s > f->started_seen || f->started_moved == std::chrono::steady_clock::time_point{}) {
    f->started_seen = std::max(s, f->started_seen);
    f->started_moved = f->stale_traced = now;
  }
  *backlog = f->published > f->started_seen ? f->published - f->started_seen : 0;
  // The hints may land out of order, so the estimate can read high after a burst of reservations (a launch's
  // first lane's worth reserves within microseconds) -- and with no reservation after it to correct it, a
  // pusher waiting for that backlog to drain would wait for ever while the lanes wait for it (r05q).  A
  // wavefront that runs out of published items stores the job count it saw: one >= the published count means
  // the lanes are waiting now.
  const uint64_t waiting = __atomic_load_n(f->waiting, __ATOMIC_RELAXED);
  if (f->launched && waiting >= f->published) *backlog = 0;
  // And a host-side bound: hints that have not moved for kStaleHints while the estimate says jobs
  // are queued mean either lanes too busy to take any -- pushing more only fills the ring up to its window --
  // or an estimate stuck on a stale count: read it as empty, so the pusher never waits on it for long.
  if (f->launched && *backlog > 0 && now - f->started_moved > kStaleHints) *backlog = 0;
  if (f->launched && *backlog > 0 && now - f->started_moved > std::chrono::seconds(1) &&
      now - f->stale_traced > std::chrono::seconds(1)) {  // (diagnostics) nothing reserved for a second
    f->stale_traced = now;
    const hipError_t q = hipStreamQuery(f->stream);
    feed_trace(f, "noreserve", (double)f->published, (double)f->started_seen);
    feed_trace(f, "state", (double)__atomic_load_n(f->error, __ATOMIC_RELAXED),
               q == hipSuccess ? 1.0 : (q == hipErrorNotReady ? 0.0 : -(double)q));
  }
  return VPT_OK;
}

int vpt_gpu_feed_debug(vpt_gpu_feed* f, int op, uint64_t* value) {
  if (!f || !value || op < 0 || op > 2) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_debug: bad argument");
  if (op == 0) {
    *value = __atomic_load_n(f->waiting, __ATOMIC_RELAXED);
  } else if (op == 1) {
    __atomic_store_n(f->waiting, *value, __ATOMIC_RELAXED);
  } else {
    for (uint64_t i = 0; i < vpt::kHintSlots; ++i) __atomic_store_n(f->started + i, *value, __ATOMIC_RELAXED);
    f->started_seen = *value;
  }
  return VPT_OK;
}

int vpt_gpu_feed_close(vpt_gpu_feed* f) {
  if (!f) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_close: null feed");
  if (f->closed) return VPT_OK;
  int rc = ctx_device(f->ctx);
  if (rc) return rc;
  f->closed = true;
  feed_publish(f, true);
  feed_trace(f, "close", (double)f->published);
  rc = feed_launch(f);
  if (f->counted) {  // closed: its launch ends once its jobs are done
    --f->ctx->open_feeds;
    f->counted = false;
  }
  if (rc) return rc;
  if (f->stage) {  // the host adds the film and the counts at collect (copy engines)
    VPT_HIP(hipEventRecord(f->closed_ev, f->stream));
    return VPT_OK;
  }
  // after the launch: the pushed jobs' sample counts (read from the pinned block, final now)
  uint32_t* counts_dev = nullptr;
  VPT_HIP(hipHostGetDevicePointer((void**)&counts_dev, f->counts, 0));
  if (int r = vpt::host::launch_tile_counts(f->ctx, f->film, counts_dev, f->stream)) return r;
  VPT_HIP(hipEventRecord(f->closed_ev, f->stream));
  return VPT_OK;
}

int vpt_gpu_feed_query(vpt_gpu_feed* f, int* done, uint64_t* pushed) {
  if (!f) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_query: null feed");
  if (pushed) *pushed = f->published;
  if (done) {
    *done = 0;
    if (f->closed) {
      const hipError_t e = hipEventQuery(f->closed_ev);
      if (e == hipSuccess)
        *done = 1;
      else if (e != hipErrorNotReady)
        return vpt::set_error(VPT_E_HIP, std::string("vpt_gpu_feed_query: ") + hipGetErrorString(e));
    }
  }
  return VPT_OK;
}

int vpt_gpu_feed_destroy(vpt_gpu_feed* f) {
  if (!f) return VPT_OK;
  const int rc = vpt_gpu_feed_close(f);
  return rc ? rc : feed_finish(f, nullptr);
}

int vpt_gpu_feed_snapshot(vpt_gpu_feed* f, float* film_host) {
  if (!f || !film_host) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_snapshot: null argument");
  if (!f->stage) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_snapshot: not a staged feed (vpt_gpu_feed_open_staged)");
  int rc = ctx_device(f->ctx);
  if (rc) return rc;
  return feed_snapshot(f, film_host, false);
}

int vpt_gpu_feed_collect(vpt_gpu_feed* f, float* film_host) {
  if (!f || !film_host) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_collect: null argument");
  if (!f->stage) return vpt::set_error(VPT_E_INVALID, "vpt_gpu_feed_collect: not a staged feed (vpt_gpu_feed_open_staged)");
  const int rc = vpt_gpu_feed_close(f);
  return rc ? rc : feed_finish(f, film_host);
}

}  // extern "C"
