// dropin_mock.cpp -- TEST HARNESS (CPU only): include/vpt_run.hpp's drain / help threads over a mock of the
// C ABI's stream, film and feed calls, so the host-side protocol -- tokens taken by drivers and helpers and
// queued for the pusher thread, the run-ahead bound, the held jobs' cost tail, the film thread's snapshots,
// helpers detaching before the driver's final collect -- is checked without a GPU: every job id the provider hands out must be "rendered"
// (pushed into some open feed) exactly once, and the host film must count every sample once.  The mock
// keeps the GPU's one blocking rule: a feed's launch holds the device (every context shares one here) until
// it is closed, so a feed's work completes only once it and every feed opened before it are closed; a wait
// that cannot end that way within 5 s is reported as a deadlock.
//
//   dropin_mock drivers=<n> helpers=<n> w= h= waves= batch= flush_ms= hold= backlog= cost_tail= stop_after=
//               multi=1 devices=<n> blocks= threads= cheap=1 rate=1 ordered=1
//
// multi=1: ONE thread drives `devices` mock GPUs through vpt_gpu::drain_devices (what run() does with the
// process's GPUs); each device blocks only its own feeds.  blocks / threads: the mock launch's
// lanes (default 3 x 7).  cheap=1: a push only records its job ids (the film is counted at the snapshots), so the
// host protocol's own cost shows; rate=1 then also times the provider alone on one thread over the same frame
// and prints both token rates ("rate frame <M/s> provider <M/s>").  ordered=1: DrainOptions::ordered_frame (what run()
// sets): each mock device's frame finish checks that every job of its tile band in the frame's range was rendered
// once, by that device, and writes the band's counts over the host film as the library writes its ordered pixels.
#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "tile_provider_headless.hpp"
#include "vpt_run.hpp"

namespace {
int64_t g_w = 0, g_h = 0, g_tw = 8, g_th = 8, g_ntx = 0;
int g_blocks = 3, g_threads = 7;
bool g_cheap = false;
std::mutex g_mu;
std::vector<uint32_t> g_rendered;  // per jid: times pushed into an open feed
std::vector<int> g_device_of;      // per jid: the device that rendered it (-1: none)
std::atomic<int> g_frames{0};      // ordered frames finished
std::atomic<int> g_open_feeds{0}, g_max_open{0};
std::atomic<uint64_t> g_direct_jobs{0};  // jobs rendered by jid-range launches (small frames), not feeds
std::mutex g_dev_mu;            // the "device": feeds in open order
std::vector<struct vpt_gpu_feed*> g_dev_feeds;
}  // namespace

struct vpt_gpu_ctx {
  std::vector<float> own;
  int device = 0;
  uint64_t frame_lo = 0, frame_waves = 0;  // an open ordered frame (frame_waves > 0): jobs from frame_lo of tiles
  uint32_t frame_tl = 0, frame_th = 0;     // [frame_tl, frame_th)
};
struct vpt_gpu_feed {
  vpt_gpu_ctx* ctx;
  float* film;
  bool closed = false;
  bool staged = false;
  std::mutex mu;              // film / shown / jids: the pusher "renders" (push), the film thread snapshots
  std::vector<float> shown;   // a staged feed's film as already added to the host film
  std::vector<uint64_t> jids; // cheap=1: pushed, not yet counted into the film
  uint64_t published = 0;
  std::atomic<uint64_t> backlog_calls{0};
};

namespace {
bool complete(vpt_gpu_feed* f) {  // closed, and every feed opened before it on its device closed (its launch has run)
  std::lock_guard<std::mutex> l(g_dev_mu);
  for (vpt_gpu_feed* g : g_dev_feeds) {
    if (g->ctx->device != f->ctx->device) continue;
    if (!g->closed) return false;
    if (g == f) return true;
  }
  return true;
}
void count_job(float* film, uint64_t jid) {  // the job's 64 samples' count channel
  const int64_t T = g_ntx * ((g_h + g_th - 1) / g_th);
  const int64_t tile = (int64_t)(jid % (uint64_t)T), x0 = (tile % g_ntx) * g_tw, y0 = (tile / g_ntx) * g_th;
  for (int64_t y = y0; y < std::min(g_h, y0 + g_th); ++y)
    for (int64_t x = x0; x < std::min(g_w, x0 + g_tw); ++x) film[(y * g_w + x) * 4 + 3] += 1.0f;
}
void settle(vpt_gpu_feed* f) {  // cheap=1: the pushed jobs into the counts (under f->mu)
  if (f->jids.empty()) return;
  {
    std::lock_guard<std::mutex> l(g_mu);
    for (uint64_t j : f->jids) {
      ++g_rendered[j];
      g_device_of[j] = f->ctx->device;
    }
  }
  for (uint64_t j : f->jids) count_job(f->film, j);
  f->jids.clear();
}
int wait_complete(vpt_gpu_feed* f) {
  for (int i = 0; i < 50000 && !complete(f); ++i) std::this_thread::sleep_for(std::chrono::microseconds(100));
  if (complete(f)) return VPT_OK;
  std::printf("dropin_mock: deadlock: waited 5 s for a feed behind an open one\n");
  return VPT_E_STATE;
}
void dev_remove(vpt_gpu_feed* f) {
  std::lock_guard<std::mutex> l(g_dev_mu);
  g_dev_feeds.erase(std::find(g_dev_feeds.begin(), g_dev_feeds.end(), f));
}
void add_delta(vpt_gpu_feed* f, float* host) {  // host += film - shown; shown = film
  std::lock_guard<std::mutex> l(f->mu);
  settle(f);
  if (f->shown.empty()) f->shown.assign((size_t)(g_w * g_h * 4), 0.0f);
  for (int64_t i = 0; i < g_w * g_h * 4; ++i) {
    host[i] += f->film[i] - f->shown[i];
    f->shown[i] = f->film[i];
  }
}
}  // namespace

extern "C" {
const char* vpt_last_error(void) { return "mock"; }
int vpt_gpu_stream_create(vpt_gpu_ctx*, void** s) {
  *s = new int(0);
  return VPT_OK;
}
int vpt_gpu_stream_destroy(vpt_gpu_ctx*, void* s) {
  delete static_cast<int*>(s);
  return VPT_OK;
}
int vpt_gpu_launch_info(const vpt_gpu_ctx*, int* blocks, int* threads) {  // a small "GPU": 3 x 7 lanes by default
  *blocks = g_blocks;
  *threads = g_threads;
  return VPT_OK;
}
int vpt_gpu_find_seeds(int, uint32_t, uint32_t, uint32_t*, int, int*) { return VPT_E_HIP; }  // (run() is not mocked)
int vpt_gpu_job_space(const vpt_gpu_ctx*, uint64_t* per_wave, uint64_t* total) {
  *per_wave = (uint64_t)(g_ntx * ((g_h + g_th - 1) / g_th));
  *total = 0;
  return VPT_OK;
}
int vpt_gpu_tile_costs(vpt_gpu_ctx*, float*, uint32_t* rank) {  // the last tile costliest: a real reorder
  const uint64_t T = (uint64_t)(g_ntx * ((g_h + g_th - 1) / g_th));
  if (rank)
    for (uint64_t i = 0; i < T; ++i) rank[i] = (uint32_t)(T - 1 - i);
  return VPT_OK;
}
int vpt_gpu_feed_prepare(vpt_gpu_ctx*, uint64_t, int) { return VPT_OK; }
int vpt_gpu_film_device_ptr(vpt_gpu_ctx* c, float** film, uint64_t* count) {
  *film = c->own.data();
  *count = c->own.size();
  return VPT_OK;
}
int vpt_gpu_frame_open(vpt_gpu_ctx* c, uint64_t jid_lo, uint64_t* waves, uint32_t tile_lo, uint32_t tile_hi) {
  c->frame_waves = std::min<uint64_t>(*waves, 1u << 20);
  *waves = c->frame_waves;
  c->frame_lo = jid_lo;
  c->frame_tl = tile_lo;
  c->frame_th = tile_hi;
  return VPT_OK;
}
int vpt_gpu_frame_finish(vpt_gpu_ctx* c, uint64_t jid_end, const float* prior, float* host) {
  if (!c->frame_waves) return VPT_OK;
  c->frame_waves = 0;
  const uint64_t T = (uint64_t)(g_ntx * ((g_h + g_th - 1) / g_th));
  std::vector<float> count(T, 0.0f);
  {
    std::lock_guard<std::mutex> l(g_mu);
    for (uint64_t j = c->frame_lo; j < jid_end; ++j) {
      const uint64_t t = j % T;
      if (t < c->frame_tl || t >= c->frame_th) continue;
      if (j >= g_rendered.size() || g_rendered[j] != 1 || g_device_of[j] != c->device) {
        std::printf("dropin_mock: frame of device %d: jid %llu rendered %u times, by device %d\n", c->device,
                    (unsigned long long)j, j < g_rendered.size() ? g_rendered[j] : 0u, j < g_device_of.size() ? g_device_of[j] : -2);
        return VPT_E_STATE;
      }
      count[t] += 1.0f;
    }
  }
  for (uint64_t t = c->frame_tl; t < c->frame_th; ++t) {  // the band's pixels over the host film
    const int64_t x0 = (int64_t)(t % (uint64_t)g_ntx) * g_tw, y0 = (int64_t)(t / (uint64_t)g_ntx) * g_th;
    for (int64_t y = y0; y < std::min(g_h, y0 + g_th); ++y)
      for (int64_t x = x0; x < std::min(g_w, x0 + g_tw); ++x) {
        const size_t p = (size_t)(y * g_w + x) * 4 + 3;
        host[p] = (prior ? prior[p] : 0.0f) + count[t];
      }
  }
  ++g_frames;
  return VPT_OK;
}
int vpt_gpu_render_jobs(vpt_gpu_ctx* c, uint64_t begin, uint64_t count, float* film, void*) {  // a small frame's launch
  if (film) return VPT_E_INVALID;
  const int64_t T = g_ntx * ((g_h + g_th - 1) / g_th);
  for (uint64_t jid = begin; jid < begin + count; ++jid) {
    {
      std::lock_guard<std::mutex> l(g_mu);
      if (jid >= g_rendered.size()) return VPT_E_INVALID;
      ++g_rendered[jid];
      g_device_of[jid] = c->device;
    }
    const int64_t tile = (int64_t)(jid % (uint64_t)T), x0 = (tile % g_ntx) * g_tw, y0 = (tile / g_ntx) * g_th;
    for (int64_t y = y0; y < std::min(g_h, y0 + g_th); ++y)
      for (int64_t x = x0; x < std::min(g_w, x0 + g_tw); ++x) c->own[(y * g_w + x) * 4 + 3] += 1.0f;
  }
  g_direct_jobs += count;
  return VPT_OK;
}
int vpt_gpu_sync(vpt_gpu_ctx*) { return VPT_OK; }
int vpt_gpu_film_flush_to_host(vpt_gpu_ctx* c, float* film, float* host) {
  if (film) return VPT_E_INVALID;
  for (size_t i = 0; i < c->own.size(); ++i) {
    host[i] += c->own[i];
    c->own[i] = 0.0f;
  }
  return VPT_OK;
}
int vpt_gpu_bind_thread_near(vpt_gpu_ctx*, int* node) {
  if (node) *node = -1;
  return VPT_OK;
}
int vpt_gpu_feed_open(vpt_gpu_ctx* c, float* film, void* stream, uint64_t, vpt_gpu_feed** out) {
  if (!stream) return VPT_E_INVALID;
  *out = new vpt_gpu_feed();
  (*out)->ctx = c;
  (*out)->film = film ? film : c->own.data();
  // (shown is allocated at the first snapshot: a 1080p film's 33 MB zero-fill here would time the mock, not the
  // protocol -- the library's feeds come from a pool prepared ahead)
  {
    std::lock_guard<std::mutex> l(g_dev_mu);
    g_dev_feeds.push_back(*out);
  }
  const int n = ++g_open_feeds;
  int m = g_max_open.load();
  while (n > m && !g_max_open.compare_exchange_weak(m, n)) {
  }
  return VPT_OK;
}
int vpt_gpu_feed_push(vpt_gpu_feed* f, const uint64_t* jids, uint64_t n) {
  if (f->closed) return VPT_E_STATE;
  if (g_cheap) {
    for (uint64_t i = 0; i < n; ++i)
      if (jids[i] >= g_rendered.size()) return VPT_E_INVALID;
    std::lock_guard<std::mutex> l(f->mu);
    f->jids.insert(f->jids.end(), jids, jids + n);
    f->published += n;
    return VPT_OK;
  }
  const int64_t T = (int64_t)g_rendered.size() ? g_ntx * ((g_h + g_th - 1) / g_th) : 1;
  for (uint64_t i = 0; i < n; ++i) {
    {
      std::lock_guard<std::mutex> l(g_mu);
      if (jids[i] >= g_rendered.size()) return VPT_E_INVALID;
      ++g_rendered[jids[i]];
      g_device_of[jids[i]] = f->ctx->device;
    }
    const int64_t tile = (int64_t)(jids[i] % (uint64_t)T), x0 = (tile % g_ntx) * g_tw, y0 = (tile / g_ntx) * g_th;
    std::lock_guard<std::mutex> l(f->mu);
    for (int64_t y = y0; y < std::min(g_h, y0 + g_th); ++y)
      for (int64_t x = x0; x < std::min(g_w, x0 + g_tw); ++x) f->film[(y * g_w + x) * 4 + 3] += 1.0f;  // the count
  }
  f->published += n;
  if (n % 3 == 0) std::this_thread::yield();  // let other threads interleave
  return VPT_OK;
}
int vpt_gpu_feed_backlog(vpt_gpu_feed* f, uint64_t* b) {  // alternately "starved" and "full": both pusher branches
  if (g_cheap) {  // a GPU that takes every job at once
    *b = 0;
    return VPT_OK;
  }
  *b = (f->backlog_calls++ % 4 == 0) ? 0 : f->published;
  return VPT_OK;
}
int vpt_gpu_feed_open_staged(vpt_gpu_ctx* c, float* film, void* stream, uint64_t w, vpt_gpu_feed** out) {
  int own = 0;  // (a staged feed without a stream uses its own)
  const int rc = vpt_gpu_feed_open(c, film, stream ? stream : &own, w, out);
  if (rc == VPT_OK) (*out)->staged = true;
  return rc;
}
int vpt_gpu_feed_close(vpt_gpu_feed* f) {
  std::lock_guard<std::mutex> l(g_dev_mu);
  f->closed = true;
  return VPT_OK;
}
int vpt_gpu_feed_query(vpt_gpu_feed* f, int* done, uint64_t*) {
  *done = complete(f) ? 1 : 0;
  return VPT_OK;
}
int vpt_gpu_feed_destroy(vpt_gpu_feed* f) {
  vpt_gpu_feed_close(f);
  const int rc = wait_complete(f);
  {
    std::lock_guard<std::mutex> l(f->mu);
    settle(f);
  }
  dev_remove(f);
  --g_open_feeds;
  delete f;
  return rc;
}
int vpt_gpu_feed_snapshot(vpt_gpu_feed* f, float* host) {
  if (!f->staged) return VPT_E_INVALID;
  add_delta(f, host);
  return VPT_OK;
}
int vpt_gpu_feed_collect(vpt_gpu_feed* f, float* host) {
  if (!f->staged) return VPT_E_INVALID;
  vpt_gpu_feed_close(f);
  int rc = wait_complete(f);
  if (rc == VPT_OK) {
    add_delta(f, host);
    std::lock_guard<std::mutex> l(f->mu);
    std::fill(f->film, f->film + g_w * g_h * 4, 0.0f);
  }
  dev_remove(f);
  --g_open_feeds;
  delete f;
  return rc;
}
}

int main(int argc, char** argv) {
  std::map<std::string, long long> a{{"drivers", 1}, {"helpers", 0}, {"w", 72}, {"h", 40}, {"waves", 5},
                                     {"batch", 7}, {"flush_ms", 0}, {"hold", 0}, {"backlog", 0}, {"stop_after", 0},
                                     {"cost_tail", 1}, {"cost_chunks", 1}, {"multi", 0}, {"devices", 1},
                                     {"blocks", 3}, {"threads", 7}, {"cheap", 0}, {"rate", 0}, {"ordered", 0}};
  for (int i = 1; i < argc; ++i) {
    const char* eq = std::strchr(argv[i], '=');
    if (eq) a[std::string(argv[i], eq - argv[i])] = std::atoll(eq + 1);
  }
  g_w = a["w"];
  g_h = a["h"];
  g_ntx = (g_w + g_tw - 1) / g_tw;
  g_blocks = (int)a["blocks"];
  g_threads = (int)a["threads"];
  g_cheap = a["cheap"] != 0;
  double provider_ms = 0;
  if (a["rate"]) {  // the provider alone, one thread: the drop-in's floor (bench.py's provider_alone)
    vpt_headless::TileProvider tp0(g_w, g_h, (unsigned)a["waves"], g_tw, g_th);
    struct Counting {  // (the same per-token counter as the frame's provider below)
      vpt_headless::TileProvider& tp;
      std::atomic<uint64_t> handed{0};
      vpt_headless::TileProvider::token next() {
        handed.fetch_add(1);
        return tp.next();
      }
    } cp{tp0};
    const auto r0 = std::chrono::steady_clock::now();
    vpt_gpu::JobRuns runs;
    uint64_t n = 0;
    while (uint64_t k = vpt_gpu::take_jobs(cp, 4096, runs, [](auto&) {})) n += k;
    provider_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - r0).count();
    if (n != tp0.num_tiles() * (uint64_t)a["waves"]) return 1;
    // the same on a thread of its own (the frame's taker is one), for reference
    vpt_headless::TileProvider tp1(g_w, g_h, (unsigned)a["waves"], g_tw, g_th);
    Counting cp1{tp1};
    double ms1 = 0;
    std::thread([&] {
      const auto t1 = std::chrono::steady_clock::now();
      vpt_gpu::JobRuns r1;
      while (vpt_gpu::take_jobs(cp1, 4096, r1, [](auto&) {})) {
      }
      ms1 = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    }).join();
    std::printf("dropin_mock: provider alone %.1f ms on the main thread, %.1f ms on a new thread\n", provider_ms, ms1);
  }
  vpt_headless::TileProvider tp(g_w, g_h, (unsigned)a["waves"], g_tw, g_th);
  const uint64_t T = tp.num_tiles(), total = T * (uint64_t)a["waves"];
  g_rendered.assign(total + 8 * T, 0);  // room for jids past a stop
  g_device_of.assign(g_rendered.size(), -1);
  std::atomic<uint64_t> handed{0};
  struct Stopping {
    vpt_headless::TileProvider& tp;
    std::atomic<uint64_t>& handed;
    uint64_t stop_after;
    uint64_t last = 0;               // rate=1: the frame's token count; the call that takes it notes the time
    std::atomic<int64_t> dry_ns{0};
    vpt_headless::TileProvider::token next() {
      const uint64_t k = handed.fetch_add(1) + 1;
      if (k == stop_after) tp.stop_at_next_wave();
      if (k == last) dry_ns.store(std::chrono::steady_clock::now().time_since_epoch().count());
      return tp.next();
    }
    unsigned progress() const { return tp.progress(); }  // (drain's probe; ordered frames are sized from it)
  } sp{tp, handed, (uint64_t)a["stop_after"]};
  sp.last = a["rate"] ? total : 0;
  std::vector<float> film((size_t)(g_w * g_h * 4), 0.0f);
  const bool multi = a["multi"] != 0;
  const int drivers = multi ? 1 : (int)a["drivers"], helpers = multi ? 0 : (int)a["helpers"];
  std::vector<vpt_gpu_ctx> ctx(multi ? (size_t)a["devices"] : (size_t)drivers);
  for (size_t i = 0; i < ctx.size(); ++i) {
    ctx[i].own.assign(film.size(), 0.0f);
    ctx[i].device = multi ? (int)i : 0;  // drain(): every context on the one device, as before
  }
  std::vector<vpt_gpu_ctx*> ctxp;
  for (auto& c : ctx) ctxp.push_back(&c);
  vpt_gpu::DrainOptions opt;
  opt.flush_seconds = (double)a["flush_ms"] / 1000.0;
  opt.hold_jobs = (uint64_t)a["hold"];
  opt.backlog_jobs = (uint64_t)a["backlog"];
  opt.cost_tail = a["cost_tail"] != 0;
  opt.cost_chunks = a["cost_chunks"] != 0;
  opt.ordered_frame = a["ordered"] != 0;
  {
    std::lock_guard<std::mutex> l(vpt_gpu::detail::Helpers::get().mu);
    vpt_gpu::detail::Helpers::get().drivers += drivers;  // (run() counts them when they claim a device)
  }
  std::vector<int> rc(drivers + helpers, 0);
  std::vector<std::thread> pool;
  const auto f0 = std::chrono::steady_clock::now();
  if (multi)
    pool.emplace_back([&] { rc[0] = vpt_gpu::drain_devices(ctxp, sp, film.data(), (uint64_t)a["batch"], opt); });
  else
    for (int i = 0; i < drivers; ++i)
      pool.emplace_back([&, i] { rc[i] = vpt_gpu::drain(&ctx[i], sp, film.data(), (uint64_t)a["batch"], opt, nullptr, helpers > 0); });
  for (int i = 0; i < helpers; ++i) pool.emplace_back([&, i] { rc[drivers + i] = vpt_gpu::help(sp, (uint64_t)a["batch"]); });
  for (int i = 0; i < drivers; ++i) pool[i].join();
  const double frame_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - f0).count();
  {
    std::lock_guard<std::mutex> l(vpt_gpu::detail::Helpers::get().mu);
    vpt_gpu::detail::Helpers::get().drivers -= drivers;
    vpt_gpu::detail::Helpers::get().cv.notify_all();
  }
  for (size_t i = drivers; i < pool.size(); ++i) pool[i].join();
  for (int r : rc)
    if (r) {
      std::printf("dropin_mock: a thread returned %d\n", r);
      return 1;
    }
  // every job of the waves that ran rendered exactly once; none beyond them
  const uint64_t waves = tp.max_wave_started(), ran = T * waves;
  for (uint64_t j = 0; j < g_rendered.size(); ++j)
    if (g_rendered[j] != (j < ran ? 1u : 0u)) {
      std::printf("dropin_mock: jid %llu rendered %u times\n", (unsigned long long)j, g_rendered[j]);
      return 1;
    }
  for (size_t p = 3; p < film.size(); p += 4)
    if (film[p] != (float)waves) {
      std::printf("dropin_mock: pixel %zu counts %g samples, want %llu\n", p / 4, film[p], (unsigned long long)waves);
      return 1;
    }
  std::printf("dropin_mock: ok %llu waves, %llu jobs, max %d feeds open, %llu jobs in direct launches, %d ordered frames\n",
              (unsigned long long)waves, (unsigned long long)ran, g_max_open.load(),
              (unsigned long long)g_direct_jobs.load(), g_frames.load());
  if (a["rate"]) {  // the taker's rate: tokens / (provider dry - start); frame_ms adds the pipelines' end
    const double take_ms =
        (double)(sp.dry_ns.load() - f0.time_since_epoch().count()) * 1e3 * std::chrono::steady_clock::period::num /
        std::chrono::steady_clock::period::den;
    std::printf("dropin_mock: rate frame %.2f provider %.2f M tokens/s (taken in %.1f ms, frame %.1f ms, provider alone %.1f ms)\n",
                ran / take_ms / 1e3, ran / provider_ms / 1e3, take_ms, frame_ms, provider_ms);
  }
  return 0;
}
