// vpt_run.hpp — the reference-side drop-in for vpt::run (include/vpt/worker.hpp:11, src/worker.cpp:92-208)
// on MI355X GPUs, written against the C ABI of vpt_gpu.h only (header-only C++20).
//
//   vpt_gpu::run(cfg.worker_parameters, vol, camera, provider, film, rng);   // was vpt::run(...)
//
// is the only change src/main.cpp:63-68 needs: the same arguments, the reference's own types
// (templated, so this header needs neither Eigen nor NanoVDB), the same threads.  What run() reads
// from them, all through their public interfaces:
//   * WorkerParameters            the fields of configuration.hpp:34-44
//   * Volume                      vol.params() (VolumeParameters) and vol.grids().density() /
//                                 .temperature() / .has_temperature(): the NanoGrid<float>s themselves,
//                                 flattened by vpt_grid_from_nanovdb from their memory (&grid,
//                                 grid.gridSize() bytes).  Their leaf maxima were already fixed by the
//                                 Volume ctor (volume.cpp:162-170); vpt_gpu_create's fix is idempotent.
//   * Camera                      camera.params() (CameraParameters); the raster->world matrix is
//                                 rebuilt from them exactly as Camera::Camera does (camera.cpp:45-57)
//   * TileProvider                next() tokens: jid() and compute_rect().  The tile size is private
//                                 to the reference's TileProvider, so it is read off the first batch
//                                 of tokens (the largest rect; every token's rect is then checked
//                                 against the jid -> tile mapping of tile_provider.cpp:27-31, 95-105)
//   * Image<float,4>              film.size() and film.data().data(): H x W XYZW floats, row-major
//   * RandomNumberGenerator       its seed: rng.seed() when the type has one; the reference keeps it
//                                 private (random.hpp:86-115), so otherwise the u32 seed whose job-0
//                                 stream starts with the same two outputs is found by search (2^32
//                                 candidates of hash + pcg32_fast in one GPU launch, vpt_gpu_find_seeds:
//                                 a few ms; once per process and stream start)
// Threads: main.cpp starts num_workers threads that all call run().  The first caller drives every GPU
// of the process from one token-taking thread (drain_devices: a context and a feed pipeline per GPU, each
// batch of tokens routed to the GPU that needs it); callers that find it driving return at once -- the
// provider's one job counter makes a second taker slower, not faster (r05: 13-16x per token).  The
// contexts are built only after the caller's first batch of tokens, so a late caller that finds the
// provider drained returns without building one.  Errors: the reference exits
// through vptFATAL (exit(1), logging.hpp:16); run() prints vpt_last_error() and exits with 1 too
// (run_checked returns the code instead).
#pragma once

#include <algorithm>
#include <bit>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

#include "vpt_gpu.h"

namespace vpt_gpu {

using JobRuns = std::vector<std::pair<uint64_t, uint64_t>>;  // contiguous (jid_begin, count) runs

struct DrainOptions {
  double flush_seconds = 0.2;  // progressive film period (main.cpp's window draws at 5 FPS); <= 0: at the end only
  // Run-ahead: the jobs taken from the provider and not yet started on the GPU are at most hold_jobs (held on
  // the host, in the order taken) + backlog_jobs (pushed into the feed's ring, which the pusher keeps at least
  // that full so the lanes never wait for the host).  0 = auto: hold 2 x the launch's lanes (C3: 917 504 jobs,
  // 28 of 256 waves), backlog 1 x (C3: 458 752).  The C3 frame measured flat over hold 2 / 4 / 6 x and backlog
  // 1 / 0.5 x (366-372 ms, r05d), and 390 ms without the cost tail.
  uint64_t hold_jobs = 0;
  uint64_t backlog_jobs = 0;
  // When the provider runs dry the held jobs are pushed costliest tile first (vpt_gpu_tile_costs), so the launch
  // ends on cheap jobs -- the one-launch frame's cost tail (VPT_ORDER_COST_TAIL), over the jobs still held.
  bool cost_tail = true;
  // Before that, every push of held jobs (kChunk = 16 384 at a time, half a C3 wave) goes costliest tile first
  // -- the one-launch frame's wave-major cost order (VPT_ORDER_COST_WAVE_MAJOR), chunk by chunk.
  bool cost_chunks = true;
  // Frames the provider hands out in fewer than direct_below jobs render as jid-range launches instead of a feed
  // (detail::render_runs); 0 = auto: the launch's lanes (a feed would launch only at its close).  1: always a feed.
  uint64_t direct_below = 0;
  // The ordered frame (vpt_gpu_frame_open / _finish): the feeds' launches also store every sample, and once they are
  // collected each pixel's samples are added in wave order onto the film as it was before the frame -- the film the
  // reference's workers produce, bit for bit (the feeds' fp32 atomics only make the progressive film).  It needs one
  // taker: every job of the frame's range must reach this drain (run() sets it; drain() threads sharing a provider,
  // or helpers, must not).  A frame larger than the device's memory keeps the atomics' film.
  bool ordered_frame = false;
};

// Takes up to max_jobs tokens; on_token(token&) sees each before it is released.  Returns the count.
template <class Provider, class OnToken>
uint64_t take_jobs(Provider& tp, uint64_t max_jobs, JobRuns& runs, OnToken&& on_token) {
  runs.clear();
  uint64_t taken = 0;
  while (taken < max_jobs) {
    auto t = tp.next();  // released at the end of this iteration, before the next next()
    if (!t) break;       // waves exhausted, stop_at_next_wave() or stop_now() (tile_provider.cpp:33-34)
    on_token(t);
    const uint64_t jid = t.jid();
    if (!runs.empty() && runs.back().first + runs.back().second == jid)
      ++runs.back().second;
    else
      runs.emplace_back(jid, 1);
    ++taken;
  }
  return taken;
}

namespace detail {
// VPT_DRAIN_TRACE=1: one stderr line per pipeline event (taker done, the pusher's final hold, its close), in
// milliseconds since the first event, next to the library's VPT_FEED_TRACE lines.
inline void drain_trace(const char* what, double a = 0, double b = 0) {
  static const bool on = std::getenv("VPT_DRAIN_TRACE") && std::atoi(std::getenv("VPT_DRAIN_TRACE")) > 0;
  if (!on) return;
  static const auto t0 = std::chrono::steady_clock::now();
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::fprintf(stderr, "drain %10.2f ms %-10s %.0f %.0f\n", ms, what, a, b);
}
// The host film as it was before an ordered frame (vpt_gpu_frame_finish adds the frame's samples onto it), copied on
// a thread of its own while the frame starts; get() is nullptr when it was all zeros (+0.0), the usual fresh film.
// Joined (by any pipeline's thread, once) before anything writes the film: a small frame's launches, a pipeline's
// first snapshot, its finish.
struct PriorFilm {
  std::vector<float> v;
  bool zero = true;
  std::thread th;
  std::mutex mu;
  void start(vpt_gpu_ctx* ctx, const float* film) {
    float* dev = nullptr;
    uint64_t n = 0;
    if (vpt_gpu_film_device_ptr(ctx, &dev, &n) != VPT_OK) return;
    th = std::thread([this, film, n] {
      v.assign(film, film + n);
      zero = std::all_of(v.begin(), v.end(), [](float x) { return std::bit_cast<uint32_t>(x) == 0u; });
    });
  }
  void join() {
    std::lock_guard<std::mutex> l(mu);
    if (th.joinable()) th.join();
  }
  const float* get() {
    join();
    return zero ? nullptr : v.data();
  }
  ~PriorFilm() { join(); }
};
}  // namespace detail

inline std::mutex& film_mutex() {  // the host film is shared by every caller
  static std::mutex mu;
  return mu;
}

// One drain() call's pipeline: one staged feed (one launch of the production kernel for the whole drain, no
// launch drain between batches), a pusher thread that feeds it from the jobs the takers queue, and a film
// thread that adds the launch's progress into the caller's film every flush_seconds.  The takers (the driving
// thread and help() threads) only take tokens and queue their job ids: the provider's next() is the drop-in's
// host-side bound (C4: 66 M tokens/s on one thread of the GPU box vs ~83 M jobs/s the GPU renders), so nothing else runs on
// that thread.
class FeedPipeline {
 public:
  // An ordered frame (DrainOptions::ordered_frame): the jobs from jid_lo on of tiles [tile_lo, tile_hi), at most
  // `waves` waves (the library may grant fewer), added in wave order onto the film before the frame at finish().
  struct Frame {
    uint64_t jid_lo = 0, waves = 0;
    uint32_t tile_lo = 0, tile_hi = 0;
    detail::PriorFilm* prior = nullptr;  // the film before the frame (joined before this pipeline writes the film)
  };
  std::atomic<int> helpers{0};  // help() threads attached (see detail::Helpers)
  explicit FeedPipeline(vpt_gpu_ctx* ctx) : ctx_(ctx) {}
  ~FeedPipeline() {
    stop_threads();
    if (feed_) (void)vpt_gpu_feed_destroy(feed_);
    uint64_t none = 0;
    if (frame_on_ && !feed_) (void)vpt_gpu_frame_open(ctx_, 0, &none, 0, 0);  // (a frame left open by an error path)
  }
  int start(float* film_host, const DrainOptions& opt, const Frame* frame = nullptr) {
    film_host_ = film_host;
    prior_ = frame ? frame->prior : nullptr;
    if (frame) {  // before the feed opens: the frame's memory is allocated now (vpt_gpu_frame_open)
      uint64_t T = 0, total = 0, waves = frame->waves;
      if (int rc = vpt_gpu_job_space(ctx_, &T, &total)) return rc;
      if (vpt_gpu_frame_open(ctx_, frame->jid_lo, &waves, frame->tile_lo, frame->tile_hi) == VPT_OK) {
        frame_ = *frame;
        frame_on_ = true;
        frame_end_ = (frame->jid_lo / T + waves) * T;  // jobs from here on store nothing: the atomics' film stands
        pushed_end_ = frame->jid_lo;
      }
      detail::drain_trace("frame", frame_on_ ? (double)waves : -1.0, (double)frame->jid_lo);
    }
    flush_ = opt.flush_seconds;
    int blocks = 0, threads = 0;
    if (int rc = vpt_gpu_launch_info(ctx_, &blocks, &threads)) return rc;
    const uint64_t lanes = (uint64_t)blocks * (uint64_t)threads;
    lanes_ = lanes;
    hold_max_ = opt.hold_jobs ? opt.hold_jobs : 2 * lanes;
    backlog_ = opt.backlog_jobs ? opt.backlog_jobs : lanes;
    cost_chunks_ = opt.cost_chunks;
    if (opt.cost_tail || opt.cost_chunks) {  // cost classes per tile, before the feed holds the device (the cost pass syncs)
      uint64_t T = 0, total = 0;
      if (int rc = vpt_gpu_job_space(ctx_, &T, &total)) return rc;
      std::vector<uint32_t> rank(T);
      if (int rc = vpt_gpu_tile_costs(ctx_, nullptr, rank.data())) return rc;
      cls_.assign(T, 0);
      for (uint64_t i = 0; i < T; ++i) cls_[rank[i]] = (uint8_t)((i * kClasses) / T);  // 0: costliest
    }
    cost_tail_ = opt.cost_tail;
    // the ring holds the backlog plus the lanes' reservations; the feed's own stream
    if (int rc = vpt_gpu_feed_open_staged(ctx_, nullptr, nullptr, backlog_ + lanes, &feed_)) return rc;
    pusher_ = std::thread([this] { pusher_main(); });
    if (flush_ > 0) film_ = std::thread([this] { film_main(); });
    return VPT_OK;
  }
  // A taker's batch of job ids: queued for the pusher.  Blocks while the run-ahead bound is reached.
  int add(const JobRuns& runs) {
    uint64_t n = 0;
    for (const auto& r : runs) n += r.second;
    std::unique_lock<std::mutex> l(mu_);
    if (err_ == VPT_OK && queued_ + held_ >= hold_max_) {  // the run-ahead bound: wait for the lanes
      const auto w0 = std::chrono::steady_clock::now();
      taker_cv_.wait(l, [&] { return err_ != VPT_OK || queued_ + held_ < hold_max_; });
      blocked_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();
    }
    if (err_ != VPT_OK) return err_;
    queue_.insert(queue_.end(), runs.begin(), runs.end());
    queued_ += n;
    added_.fetch_add(n, std::memory_order_relaxed);
    return VPT_OK;
  }
  // Jobs given to this pipeline and not yet started on the GPU: queued and held on the host, plus the feed's
  // backlog as the pusher last read it (drain_devices routes each batch to the GPU with the fewest).
  uint64_t pending() {
    std::lock_guard<std::mutex> l(mu_);
    return queued_ + held_ + backlog_seen_.load(std::memory_order_relaxed);
  }
  uint64_t added() const { return added_.load(std::memory_order_relaxed); }  // jobs given to add()
  uint64_t lanes() const { return lanes_; }  // the launch's lanes: it starts once that many jobs are pushed
  // No more add(): the pusher pushes what it holds and closes the feed (finish() then waits for the launch).
  // drain_devices ends every GPU's input first, so no pipeline's last push waits for another one's launch.
  void end_input() {
    std::lock_guard<std::mutex> l(mu_);
    no_more_ = true;
  }
  // No more jobs: the pusher pushes what it holds and closes the feed; then the rest of the film is added.
  int finish() {
    end_input();
    if (pusher_.joinable()) pusher_.join();
    stop_threads();  // no snapshot starts once the feed is closed: the collect adds the rest
    detail::drain_trace("taker_blocked_ms", blocked_s_ * 1e3);
    int rc = err_;
    if (feed_) {
      vpt_gpu_feed* f = feed_;
      feed_ = nullptr;
      // The wait happens before the film lock: another caller's launch may be waiting for this device's CUs,
      // which this feed's launch holds until that caller -- maybe blocked on the lock -- closes its feed.
      int frc = vpt_gpu_feed_close(f);
      for (int done = 0; frc == VPT_OK && !done;)
        if ((frc = vpt_gpu_feed_query(f, &done, nullptr)) == VPT_OK && !done)
          std::this_thread::sleep_for(std::chrono::microseconds(100));
      if (prior_) prior_->join();
      if (frc == VPT_OK) {
        std::lock_guard<std::mutex> lock(film_mutex());
        // An ordered frame rewrites its tiles' pixels whole (this feed rendered no others): the feed's last
        // delta is not added first, its film only cleared for the next use.  Else the collect adds it.
        const bool order = frame_on_ && rc == VPT_OK && pushed_end_ <= frame_end_;
        frc = order ? vpt_gpu_feed_destroy(f) : vpt_gpu_feed_collect(f, film_host_);
        if (frame_on_) {  // the frame's tiles in wave order (or the frame closed: the atomics' film stands)
          if (order && frc == VPT_OK) {
            frc = vpt_gpu_frame_finish(ctx_, pushed_end_, frame_.prior ? frame_.prior->get() : nullptr, film_host_);
          } else {
            uint64_t none = 0;
            (void)vpt_gpu_frame_open(ctx_, 0, &none, 0, 0);
          }
          detail::drain_trace("frame_done", (double)pushed_end_, (double)frame_end_);
        }
      } else {
        (void)vpt_gpu_feed_destroy(f);
        uint64_t none = 0;
        if (frame_on_) (void)vpt_gpu_frame_open(ctx_, 0, &none, 0, 0);  // (closed: the atomics' film stands)
      }
      if (rc == VPT_OK) rc = frc;
    }
    return rc;
  }

 private:
  static constexpr int kClasses = 256;
  static constexpr uint64_t kChunk = 16384;  // jobs per push

  void fail(int rc) {
    std::lock_guard<std::mutex> l(mu_);
    if (err_ == VPT_OK) err_ = rc;
    taker_cv_.notify_all();
  }
  int push(const uint64_t* ids, uint64_t n) { return n ? vpt_gpu_feed_push(feed_, ids, n) : VPT_OK; }
  void note_end(const JobRuns& rs) {  // (the pusher's: one past the largest job id pushed, for the frame)
    for (const auto& r : rs) pushed_end_ = std::max(pushed_end_, r.first + r.second);
  }
  // The jobs taken and not yet pushed, as contiguous (jid, count) runs in the order taken (the pusher's): the
  // takers hand over runs (a batch of tokens is one or two), and the pusher expands them into job ids only as
  // it pushes them -- one pass over the ids, no division per job (r06: the pusher, not the taker, set the
  // drop-in's pace once a frame's jobs outran what it could expand, sort and push per second).
  struct Held {
    JobRuns runs;
    size_t head = 0;
    uint64_t n = 0;
    void add(const JobRuns& rs) {
      for (const auto& r : rs) {
        if (!r.second) continue;
        if (head < runs.size() && runs.back().first + runs.back().second == r.first)
          runs.back().second += r.second;
        else
          runs.push_back(r);
        n += r.second;
      }
    }
    // The first (up to) k jobs into out; their count.
    uint64_t take(uint64_t k, JobRuns& out) {
      out.clear();
      uint64_t got = 0;
      while (got < k && head < runs.size()) {
        auto& r = runs[head];
        const uint64_t c = std::min(k - got, r.second);
        out.emplace_back(r.first, c);
        r.first += c;
        r.second -= c;
        got += c;
        if (!r.second) ++head;
      }
      n -= got;
      if (head == runs.size()) {
        runs.clear();
        head = 0;
      } else if (head > 4096 && head * 2 > runs.size()) {
        runs.erase(runs.begin(), runs.begin() + (ptrdiff_t)head);
        head = 0;
      }
      return got;
    }
  };
  // A chunk's n jobs into ids_: in the order taken, or costliest tile class first (a counting sort; the order
  // taken within a class: consecutive items are different tiles of one wave).  Each job's tile is stepped along
  // its run (jid + 1 is tile + 1, mod T).
  const uint64_t* emit(const JobRuns& chunk, uint64_t n, bool sort) {
    ids_.resize(n);
    uint64_t* out = ids_.data();
    if (!sort) {
      for (const auto& r : chunk)
        for (uint64_t k = 0; k < r.second; ++k) *out++ = r.first + k;
      return ids_.data();
    }
    const uint64_t T = cls_.size();
    uint64_t start[kClasses + 1] = {};
    for (const auto& r : chunk)
      for (uint64_t k = 0, t = r.first % T; k < r.second; ++k, t = t + 1 == T ? 0 : t + 1) ++start[cls_[t] + 1];
    for (int c = 0; c < kClasses; ++c) start[c + 1] += start[c];
    for (const auto& r : chunk)
      for (uint64_t k = 0, t = r.first % T; k < r.second; ++k, t = t + 1 == T ? 0 : t + 1) out[start[cls_[t]]++] = r.first + k;
    return ids_.data();
  }
  // Pushes held jobs, oldest first, while the feed's backlog is below its mark -- and, until the launch has
  // started (it starts once a lane's worth of jobs is pushed, vpt_gpu_feed_push), below the lanes.
  int top_up(Held& hold) {
    uint64_t b = 0;
    if (int rc = vpt_gpu_feed_backlog(feed_, &b)) return rc;
    struct Seen {  // (the backlog after this call's pushes, for pending())
      std::atomic<uint64_t>& to;
      const uint64_t& b;
      ~Seen() { to.store(b, std::memory_order_relaxed); }
    } seen{backlog_seen_, b};
    const uint64_t mark = pushed_ < lanes_ ? std::max(backlog_, lanes_) : backlog_;
    while (hold.n > 0 && b < mark) {
      // (the launch's first lane's worth goes unsorted: every lane takes one of those jobs at once, so their order
      // changes nothing, and sorting them would delay the launch -- ~3 ms of C3's 458 752)
      const bool sort = cost_chunks_ && !cls_.empty() && pushed_ >= lanes_;
      const uint64_t n = hold.take(kChunk, chunk_);
      note_end(chunk_);
      if (int rc = push(emit(chunk_, n, sort), n)) return rc;
      b += n;
      pushed_ += n;
    }
    return VPT_OK;
  }
  void pusher_main() {
    (void)vpt_gpu_bind_thread_near(ctx_, nullptr);  // the ring is in the GPU's node's memory
    Held hold;  // taken, not pushed, in the order taken
    auto last_push = std::chrono::steady_clock::now();
    JobRuns batch;
    for (;;) {
      bool last;
      {
        std::lock_guard<std::mutex> l(mu_);
        batch.swap(queue_);
        queue_.clear();
        held_ += queued_;
        queued_ = 0;
        last = no_more_;  // (set after the takers' last add: everything is in batch now)
      }
      // nothing new: the lanes take jobs meanwhile (the backlog check below); a timed condition-variable wait
      // would do the same, but ThreadSanitizer (gcc 11) does not model pthread_cond_clockwait
      if (batch.empty() && !last) std::this_thread::sleep_for(std::chrono::microseconds(50));
      hold.add(batch);
      batch.clear();
      if (last) break;
      const uint64_t before = hold.n, pushed_before = pushed_;
      if (int rc = top_up(hold)) return fail(rc);
      if (pushed_ != pushed_before) {
        last_push = std::chrono::steady_clock::now();
      } else if (std::chrono::steady_clock::now() - last_push > std::chrono::seconds(1)) {
        detail::drain_trace("nopush", (double)hold.n, (double)pushed_);  // (diagnostics)
        last_push = std::chrono::steady_clock::now();
      }
      if (hold.n != before) {
        std::lock_guard<std::mutex> l(mu_);
        held_ = hold.n;
        taker_cv_.notify_all();
      }
    }
    // The provider is dry: the held jobs, costliest tile class first (jid order within a class: consecutive
    // items are different tiles of one wave), then the end of the feed.
    detail::drain_trace("final_hold", (double)hold.n, (double)pushed_);
    const uint64_t n = hold.take(hold.n, chunk_);
    note_end(chunk_);
    const uint64_t* rest = emit(chunk_, n, cost_tail_ && !cls_.empty());
    for (uint64_t i = 0; i < n; i += kChunk)
      if (int rc = push(rest + i, std::min<uint64_t>(kChunk, n - i))) return fail(rc);
    if (int rc = vpt_gpu_feed_close(feed_)) return fail(rc);
    detail::drain_trace("closed");
    std::lock_guard<std::mutex> l(mu_);
    held_ = 0;
  }
  void film_main() {
    (void)vpt_gpu_bind_thread_near(ctx_, nullptr);  // the pinned film copies are there too
    auto next = std::chrono::steady_clock::now() + std::chrono::duration<double>(flush_);
    while (!film_stop_.load()) {
      if (std::chrono::steady_clock::now() < next) {  // (slices of 1 ms: stop_threads() ends the wait)
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
        continue;
      }
      const auto period = std::chrono::duration_cast<std::chrono::steady_clock::duration>(std::chrono::duration<double>(flush_));
      next += period;
      if (prior_) prior_->join();  // (the film before the frame is copied before it changes)
      {
        std::lock_guard<std::mutex> lock(film_mutex());
        if (int rc = vpt_gpu_feed_snapshot(feed_, film_host_)) return fail(rc);
      }
      // a snapshot that overran its period skips the missed ones: back-to-back snapshots would hold the film
      // lock (and the feed's) nearly all the time
      const auto now = std::chrono::steady_clock::now();
      if (next <= now) next = now + period;
    }
  }
  void stop_threads() {
    film_stop_.store(true);
    if (film_.joinable()) film_.join();
    if (pusher_.joinable()) {  // (an error path: let the pusher end)
      {
        std::lock_guard<std::mutex> l(mu_);
        no_more_ = true;
      }
      pusher_.join();
    }
  }

  vpt_gpu_ctx* ctx_;
  float* film_host_ = nullptr;
  Frame frame_;
  detail::PriorFilm* prior_ = nullptr;  // (joined before this pipeline writes the film)
  bool frame_on_ = false;
  uint64_t frame_end_ = 0, pushed_end_ = 0;  // (pushed_end_: the pusher's, read after it has ended)
  double flush_ = 0.2;
  uint64_t hold_max_ = 0, backlog_ = 0, lanes_ = 0;
  uint64_t pushed_ = 0;  // (the pusher's)
  vpt_gpu_feed* feed_ = nullptr;
  std::vector<uint8_t> cls_;  // per tile: cost class (0 = costliest)
  bool cost_tail_ = true, cost_chunks_ = true;
  std::vector<uint64_t> ids_;  // (the pusher's: a push's job ids)
  JobRuns chunk_;              // (the pusher's: a push's runs)
  std::thread pusher_, film_;
  std::mutex mu_;  // queue_, queued_, held_, no_more_, err_
  std::condition_variable taker_cv_;
  JobRuns queue_;
  uint64_t queued_ = 0, held_ = 0;
  double blocked_s_ = 0;  // the takers' waits on the run-ahead bound (VPT_DRAIN_TRACE)
  bool no_more_ = false;
  int err_ = VPT_OK;
  std::atomic<bool> film_stop_{false};
  std::atomic<uint64_t> added_{0}, backlog_seen_{0};
};

namespace detail {
// Threads on one provider: each GPU is driven by the one thread that claimed it; other threads may take
// tokens too and queue their job ids into a driving thread's pipeline (help()).  run() does not use it: with
// the restated TileProvider, contended next() calls are slower than one thread's (r05: 1 thread 64-67 M tokens/s,
// 2 threads 3.8-5.3 M/s on the GPU box's EPYC; 42 / 29 / 28 M/s for 1 / 2 / 4 threads on an 8-core Xeon: the
// provider's one job counter); a provider whose next() scales across threads could.
struct Helpers {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<FeedPipeline*> pipes;  // pipelines that accept helpers
  int drivers = 0;                   // driving threads that have not finished (their callers count them)
  size_t next = 0;
  static Helpers& get() {
    static Helpers h;
    return h;
  }
};

}  // namespace detail

// Renders every job `tp` hands out on `ctx` and adds it into the caller's reference-layout film
// (float[H][W][4], Image<float,4>) as it goes.  Returns VPT_OK or the first error code (vpt_last_error() has
// the message).  Several threads may call it with one `tp` and one `film_host`, each with its own context.
//
// TileProvider::next() blocks until the same tile's previous wave has been released
// (src/tile_provider.cpp:40-60), so a thread that holds a token while calling next() deadlocks on itself as
// soon as the job counter has moved one wave past that token -- which, with other threads taking jobs, can
// happen at any batch size.  drain() therefore holds no token across next(): each token is released as soon
// as its job id is recorded.  Every recorded job is rendered (no token is dropped), and the GPU film needs no
// tile exclusivity: its adds are fp32 atomics.
//
// The job ids reach the GPU through one staged feed (vpt_gpu_feed_*): one running launch of the production
// kernel takes them as they are pushed, so
//   * nothing drains until the provider is dry (a launch lasts as long as its longest job);
//   * run-ahead is bounded: the takers wait while opt.hold_jobs taken jobs are held, and the pusher keeps
//     opt.backlog_jobs in the ring, so the provider's job counter (progress(), eta(), what
//     stop_at_next_wave() cuts) leads the GPU by at most those plus the jobs in flight -- as the reference's
//     workers each hold the token they render;
//   * the launch ends on cheap jobs: the jobs held when the provider runs dry go costliest tile first;
//   * the film is progressive (main.cpp:101-132 shows it at 5 FPS): every flush_seconds the film thread adds
//     what the launch has completed into film_host (the copy engines read the device film beside the launch),
//     under a mutex shared by all callers; the final film is the launch's.
// `first`: job runs already taken by the caller (queued first).  `share`: other threads of run() may queue
// into this pipeline while it drains (detail::Helpers); drain returns once they have detached.
// drain(): tokens taken before a provider with progress() is asked how large its frame is.
constexpr uint64_t kDirectProbe = 65536;

namespace detail {
inline void append_runs(JobRuns& to, const JobRuns& from) {
  for (const auto& r : from)
    if (!to.empty() && to.back().first + to.back().second == r.first)
      to.back().second += r.second;
    else
      to.push_back(r);
}
// A frame the provider hands out in fewer jobs than the launch has lanes: a feed's launch would start only at its
// close anyway (it waits for a lane's worth), on the throughput kernel.  Rendered instead as jid-range launches,
// which render() sizes as latency-bound or partly filled ones (C1: 4 096 jobs, 49-70 ms through a feed vs the
// 20.8-ms one-launch frame), then added into the caller's film.
inline int render_runs(vpt_gpu_ctx* ctx, const JobRuns& runs, float* film_host) {
  for (const auto& r : runs)
    if (int rc = vpt_gpu_render_jobs(ctx, r.first, r.second, nullptr, nullptr)) return rc;
  if (int rc = vpt_gpu_sync(ctx)) return rc;
  std::lock_guard<std::mutex> lock(film_mutex());
  return vpt_gpu_film_flush_to_host(ctx, nullptr, film_host);
}
// The same on several GPUs: the runs cut into contiguous parts of about equal job counts, one per context, all
// launched before any is waited for (C2's 262 144 jobs: a launch per GPU of 1 / N of them).
inline int render_runs_split(const std::vector<vpt_gpu_ctx*>& ctxs, const JobRuns& runs, float* film_host) {
  uint64_t total = 0;
  for (const auto& r : runs) total += r.second;
  const uint64_t n = ctxs.size(), per = (total + n - 1) / n;
  std::vector<JobRuns> parts(n);
  size_t k = 0;
  uint64_t in_part = 0;
  for (auto r : runs)
    while (r.second > 0) {
      const uint64_t c = std::min(r.second, per - in_part);
      parts[k].emplace_back(r.first, c);
      r.first += c;
      r.second -= c;
      if ((in_part += c) == per && k + 1 < n) {
        ++k;
        in_part = 0;
      }
    }
  for (size_t i = 0; i < n; ++i)
    for (const auto& r : parts[i])
      if (int rc = vpt_gpu_render_jobs(ctxs[i], r.first, r.second, nullptr, nullptr)) return rc;
  for (size_t i = 0; i < n; ++i) {
    if (int rc = vpt_gpu_sync(ctxs[i])) return rc;
    std::lock_guard<std::mutex> lock(film_mutex());
    if (int rc = vpt_gpu_film_flush_to_host(ctxs[i], nullptr, film_host)) return rc;
  }
  return VPT_OK;
}
// The jobs taken before a pipeline starts (`first`, then up to the launch's lanes -- opt.direct_below): true
// when the provider ran dry before that, a small frame (rendered by jid-range launches instead of a feed).
// A provider with the reference's progress() (percent of its jobs handed out, tile_provider.hpp:72-74) tells a
// large frame after a few batches: the pipeline then starts at once, its pusher filling the ring while the
// rest of the launch's first lane's worth is taken.  (Starting the launch itself earlier than a lane's worth
// was measured 5-15x slower: tools/experiments/r05_wave_cas_early_launch.patch.)
template <class Provider>
int take_head(vpt_gpu_ctx* ctx, Provider& tp, uint64_t batch_jobs, const DrainOptions& opt, const JobRuns* first,
              JobRuns& head, bool& small) {
  small = false;
  head.clear();
  int blocks = 0, threads = 0;
  if (int rc = vpt_gpu_launch_info(ctx, &blocks, &threads)) return rc;
  const uint64_t direct = opt.direct_below ? opt.direct_below : (uint64_t)blocks * (uint64_t)threads;
  uint64_t have = 0;
  if (first) {
    head = *first;
    for (const auto& r : head) have += r.second;
  }
  const uint64_t probe = std::min<uint64_t>(direct, kDirectProbe);
  JobRuns runs;
  while (have < direct) {
    const uint64_t n = take_jobs(tp, std::min<uint64_t>(std::max<uint64_t>(1, batch_jobs), direct - have), runs, [](auto&) {});
    if (n == 0) {  // the provider is dry: a small frame
      small = true;
      return VPT_OK;
    }
    append_runs(head, runs);
    have += n;
    if constexpr (requires { tp.progress(); }) {
      if (have >= probe && have < direct) {
        const uint64_t pct = (uint64_t)tp.progress();  // floor: the frame has >= have * 100 / (pct + 1) jobs
        if (pct == 0 || have * 100 / (pct + 1) >= direct) break;
      }
    }
  }
  return VPT_OK;
}
}  // namespace detail

namespace detail {
// An ordered frame is sized from the provider's progress() (percent of its jobs handed out, floored): until it
// reads >= 1 the frame's size has no useful bound, so tokens are taken on until it does (1 % of the frame: C3 83 K
// tokens, ~1 ms; C5 1.3 M, ~20 ms) or the provider runs dry (`dry`: the frame is what was taken) -- at most
// kSizeTokens of them (a frame of more than 400 M jobs is then sized by the device's memory).
constexpr uint64_t kSizeTokens = 4u << 20;
template <class Provider>
int take_until_sized(Provider& tp, uint64_t batch_jobs, JobRuns& head, bool& dry) {
  dry = false;
  if constexpr (requires { tp.progress(); }) {
    JobRuns more;
    uint64_t taken = 0;
    while (tp.progress() == 0 && taken < kSizeTokens) {
      const uint64_t n = take_jobs(tp, std::max<uint64_t>(1, batch_jobs), more, [](auto&) {});
      if (!n) {
        dry = true;
        break;
      }
      taken += n;
      append_runs(head, more);
    }
  }
  return VPT_OK;
}
// The frame of the jobs taken from `head` on: its first job, and how many waves it can span -- all taken (dry), or
// bounded by progress() (the frame ends before taken * 100 / pct jobs), else as many as the device holds
// (vpt_gpu_frame_open grants what fits).
template <class Provider>
FeedPipeline::Frame frame_of(Provider& tp, const JobRuns& head, uint64_t T, uint32_t tile_lo, uint32_t tile_hi,
                             PriorFilm* prior, bool dry = false) {
  FeedPipeline::Frame fr;
  fr.jid_lo = head.empty() ? 0 : head.front().first;
  uint64_t end = 0;
  for (const auto& r : head) {
    fr.jid_lo = std::min(fr.jid_lo, r.first);
    end = std::max(end, r.first + r.second);
  }
  fr.waves = ~0ULL >> 8;
  if (dry && T > 0 && end > fr.jid_lo) {
    fr.waves = (end - 1) / T - fr.jid_lo / T + 1;
  } else if constexpr (requires { tp.progress(); }) {
    if (const uint64_t pct = (uint64_t)tp.progress(); pct > 0 && T > 0)
      fr.waves = (end * 100 / pct - 1) / T - fr.jid_lo / T + 1;  // (end = the provider's job counter)
  }
  fr.tile_lo = tile_lo;
  fr.tile_hi = tile_hi;
  fr.prior = prior;
  return fr;
}
// n bands of consecutive tiles [cut[i], cut[i + 1]) of about equal estimated cost, each at least one tile (T >= n).
inline std::vector<uint32_t> cost_bands(const std::vector<float>& cost, size_t n) {
  const uint64_t T = cost.size();
  std::vector<uint32_t> cut(n + 1, 0);
  double total = 0;
  for (float c : cost) total += std::max(0.0f, c);
  double acc = 0;
  uint64_t t = 0;
  for (size_t i = 1; i < n; ++i) {
    const double goal = total * (double)i / (double)n;
    while (t < T && acc + std::max(0.0f, cost[t]) <= goal) acc += std::max(0.0f, cost[t++]);
    t = std::max<uint64_t>(t, (uint64_t)cut[i - 1] + 1);  // non-empty bands
    t = std::min<uint64_t>(t, T - (n - i));                // room for the rest
    cut[i] = (uint32_t)t;
  }
  cut[n] = (uint32_t)T;
  return cut;
}
// Runs of job ids cut at the bands' tile boundaries (jid % T), each piece appended to its band's runs.
inline void split_bands(const JobRuns& rs, uint64_t T, const std::vector<uint32_t>& cut, std::vector<JobRuns>& parts) {
  for (auto r : rs)
    while (r.second > 0) {
      const uint64_t t = r.first % T;
      const size_t b = (size_t)(std::upper_bound(cut.begin(), cut.end(), (uint32_t)t) - cut.begin()) - 1;
      const uint64_t len = std::min<uint64_t>(r.second, (uint64_t)cut[b + 1] - t);
      JobRuns& p = parts[b];
      if (!p.empty() && p.back().first + p.back().second == r.first)
        p.back().second += len;
      else
        p.emplace_back(r.first, len);
      r.first += len;
      r.second -= len;
    }
}
}  // namespace detail

template <class Provider>
int drain(vpt_gpu_ctx* ctx, Provider& tp, float* film_host, uint64_t batch_jobs, const DrainOptions& opt = {},
          const JobRuns* first = nullptr, bool share = false) {
  const bool ordered = opt.ordered_frame && !share;
  detail::PriorFilm prior;
  if (ordered) prior.start(ctx, film_host);
  JobRuns head;  // the jobs taken before the pipeline starts
  if (!share) {  // (a shared pipeline takes helpers' jobs: it always runs)
    bool small = false;
    detail::drain_trace("drain");
    if (int rc = detail::take_head(ctx, tp, batch_jobs, opt, first, head, small)) return rc;
    if (small) {
      prior.join();  // (before the launches' films are added)
      return detail::render_runs(ctx, head, film_host);
    }
    first = &head;
  }
  detail::drain_trace("head_taken");
  FeedPipeline pipe(ctx);
  FeedPipeline::Frame frame;
  if (ordered) {
    uint64_t T = 0, total = 0;
    bool dry = false;
    if (int rc = vpt_gpu_job_space(ctx, &T, &total)) return rc;
    if (int rc = detail::take_until_sized(tp, batch_jobs, head, dry)) return rc;
    frame = detail::frame_of(tp, head, T, 0, (uint32_t)T, &prior, dry);
  }
  int rc = pipe.start(film_host, opt, ordered ? &frame : nullptr);
  if (rc == VPT_OK && first) rc = pipe.add(*first);
  detail::drain_trace("started");
  detail::Helpers& hub = detail::Helpers::get();
  if (share && rc == VPT_OK) {
    std::lock_guard<std::mutex> l(hub.mu);
    hub.pipes.push_back(&pipe);
    hub.cv.notify_all();
  }
  JobRuns runs;
  uint64_t taken = 0;
  for (uint64_t n; rc == VPT_OK && (n = take_jobs(tp, std::max<uint64_t>(1, batch_jobs), runs, [](auto&) {}));) {
    taken += n;
    rc = pipe.add(runs);
  }
  detail::drain_trace("taker_done", (double)taken);
  if (share) {  // no new helper attaches; the attached ones queue their last jobs, then detach
    {
      std::lock_guard<std::mutex> l(hub.mu);
      auto it = std::find(hub.pipes.begin(), hub.pipes.end(), &pipe);
      if (it != hub.pipes.end()) hub.pipes.erase(it);
    }
    while (pipe.helpers.load() > 0) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  const int frc = pipe.finish();
  return rc ? rc : frc;
}

// A helper thread (run() does not start any, see run_checked): takes tokens batch_jobs at a time and queues
// their job ids into a driving thread's pipeline, until the provider is exhausted (or no thread drives a GPU).
template <class Provider>
int help(Provider& tp, uint64_t batch_jobs) {
  detail::Helpers& hub = detail::Helpers::get();
  FeedPipeline* pipe = nullptr;
  {
    std::unique_lock<std::mutex> l(hub.mu);
    hub.cv.wait(l, [&] { return !hub.pipes.empty() || hub.drivers == 0; });
    if (hub.pipes.empty()) return VPT_OK;
    pipe = hub.pipes[hub.next++ % hub.pipes.size()];
    ++pipe->helpers;  // under hub.mu: its driver cannot have stopped accepting helpers
  }
  int rc = VPT_OK;
  JobRuns runs;
  while (rc == VPT_OK && take_jobs(tp, std::max<uint64_t>(1, batch_jobs), runs, [](auto&) {})) rc = pipe->add(runs);
  --pipe->helpers;  // the last touch: its driver may finish and destroy the pipeline from here on
  return rc;
}

// One taker for every GPU of the process.  The reference's caller starts num_workers threads that
// all call run() on one provider (main.cpp:63-68), and every next() is a fetch_add on one job counter plus a
// seq_cst token store and notify_all (tile_provider.cpp:28, tile_provider.hpp:22-27): on the GPU box's EPYC one
// thread takes 64-67 M tokens/s, two threads together 3.8-5.3 M/s.  So the drop-in takes tokens on ONE thread
// and feeds every GPU from it: one FeedPipeline (staged feed, pusher and film threads) per context, each batch
// routed to the GPU that needs it -- first to each GPU in turn until its launch has a lane's worth (a feed's
// launch starts then), afterwards to the GPU with the fewest jobs given and not yet started (FeedPipeline::
// pending); with the ordered frame (what run() sets) each job goes to the GPU that owns its tile (cost-balanced
// bands of tiles, so every pixel's samples are ordered on one GPU).  The provider's token rate is the frame's floor: C3's 8.3 M tokens take 124 ms on one thread, so
// the 8-GPU drop-in frame is ~125-145 ms however fast the GPUs are; north_star's >= 6x at 8 GPUs
// is reachable through the C ABI's jid ranges (distributed.py, bench.py), not through a TileProvider.
// One context: exactly drain().  Small frames (the provider dry before a lane's worth): jid-range launches
// split across the GPUs.
template <class Provider>
int drain_devices(const std::vector<vpt_gpu_ctx*>& ctxs, Provider& tp, float* film_host, uint64_t batch_jobs,
                  const DrainOptions& opt = {}, const JobRuns* first = nullptr) {
  if (ctxs.empty()) return VPT_E_INVALID;
  if (ctxs.size() == 1) return drain(ctxs[0], tp, film_host, batch_jobs, opt, first);
  detail::PriorFilm prior;
  if (opt.ordered_frame) prior.start(ctxs[0], film_host);
  JobRuns head;
  bool small = false;
  if (int rc = detail::take_head(ctxs[0], tp, batch_jobs, opt, first, head, small)) return rc;
  if (small) {
    prior.join();  // (before the launches' films are added)
    // (parts on several GPUs would add into the film one after another, not in wave order: an ordered frame's
    // small frame renders on the first GPU)
    return opt.ordered_frame ? detail::render_runs(ctxs[0], head, film_host) : detail::render_runs_split(ctxs, head, film_host);
  }
  std::vector<std::unique_ptr<FeedPipeline>> pipes;
  int rc = VPT_OK;
  // An ordered frame: each GPU owns a band of tiles (about equal estimated cost, vpt_gpu_tile_costs) and renders
  // every job of its tiles, so each pixel's samples are on one GPU and its frame pass orders them.
  std::vector<uint32_t> cut;
  uint64_t T = 0;
  bool dry = false;
  if (opt.ordered_frame) {
    uint64_t total = 0;
    if ((rc = vpt_gpu_job_space(ctxs[0], &T, &total))) return rc;
    if ((rc = detail::take_until_sized(tp, batch_jobs, head, dry))) return rc;
    std::vector<float> cost(T);
    if ((rc = vpt_gpu_tile_costs(ctxs[0], cost.data(), nullptr))) return rc;
    cut = detail::cost_bands(cost, ctxs.size());
  }
  for (size_t i = 0; i < ctxs.size(); ++i) {
    pipes.push_back(std::make_unique<FeedPipeline>(ctxs[i]));
    FeedPipeline::Frame frame;
    if (opt.ordered_frame) frame = detail::frame_of(tp, head, T, cut[i], cut[i + 1], &prior, dry);
    if (rc == VPT_OK) rc = pipes.back()->start(film_host, opt, opt.ordered_frame ? &frame : nullptr);
  }
  std::vector<JobRuns> parts(opt.ordered_frame ? ctxs.size() : 0);
  auto add_bands = [&](const JobRuns& rs) -> int {  // (ordered frames) each job to the GPU that owns its tile
    for (auto& p : parts) p.clear();
    detail::split_bands(rs, T, cut, parts);
    for (size_t i = 0; i < parts.size(); ++i)
      if (!parts[i].empty())
        if (int r = pipes[i]->add(parts[i])) return r;
    return VPT_OK;
  };
  if (rc == VPT_OK) rc = opt.ordered_frame ? add_bands(head) : pipes[0]->add(head);  // (one GPU's launch starts now)
  auto route = [&]() -> size_t {
    for (size_t i = 0; i < pipes.size(); ++i)
      if (pipes[i]->added() < pipes[i]->lanes()) return i;
    size_t best = 0;
    uint64_t least = ~0ULL;
    for (size_t i = 0; i < pipes.size(); ++i)
      if (const uint64_t p = pipes[i]->pending(); p < least) {
        least = p;
        best = i;
      }
    return best;
  };
  JobRuns runs;
  uint64_t taken = 0;
  for (uint64_t n; rc == VPT_OK && (n = take_jobs(tp, std::max<uint64_t>(1, batch_jobs), runs, [](auto&) {}));) {
    taken += n;
    rc = opt.ordered_frame ? add_bands(runs) : pipes[route()]->add(runs);
  }
  detail::drain_trace("taker_done", (double)taken);
  for (auto& p : pipes) p->end_input();  // every GPU's last jobs go out before any launch is waited for
  for (auto& p : pipes)
    if (const int frc = p->finish(); rc == VPT_OK) rc = frc;
  return rc;
}

namespace detail {

// hash(seed, jid) (include/vpt/hash.hpp:20-67) and pcg32_fast's output (pcg_random.hpp, xsh_rs)
inline uint64_t job_state(uint64_t seed, uint64_t jid) {
  const uint64_t m = 0xc6a4a7935bd1e995ULL;
  uint64_t h = seed ^ (8ULL * m), k = jid * m;
  k ^= k >> 47;
  k *= m;
  h ^= k;
  h *= m;
  h ^= h >> 47;
  h *= m;
  h ^= h >> 47;
  return h | 3ULL;
}
inline uint32_t pcg_out(uint64_t s) { return (uint32_t)((s ^ (s >> 22)) >> (22 + (uint32_t)(s >> 61))); }
constexpr uint64_t kPcgMult = 6364136223846793005ULL;

// The u32 seeds whose job-0 stream starts with outputs (a, b); normally exactly one.  device >= 0: one launch
// over all 2^32 candidates (vpt_gpu_find_seeds, a few ms); device < 0 (no GPU, the host tests): host threads,
// 1-3 s.
inline int seeds_for(uint32_t a, uint32_t b, int device, std::vector<uint32_t>& out) {
  out.clear();
  if (device >= 0) {
    uint32_t found[8];
    int n = 0;
    if (int rc = vpt_gpu_find_seeds(device, a, b, found, 8, &n)) return rc;
    out.assign(found, found + std::min(n, 8));
    if (n > 8) out.resize(9, 0);  // (more than we keep: ambiguous anyway)
    return VPT_OK;
  }
  const unsigned n = std::max(1u, std::min(64u, std::thread::hardware_concurrency()));
  std::vector<std::vector<uint32_t>> found(n);
  std::vector<std::thread> pool;
  for (unsigned t = 0; t < n; ++t)
    pool.emplace_back([&, t] {
      const uint64_t lo = (1ULL << 32) * t / n, hi = (1ULL << 32) * (t + 1) / n;
      for (uint64_t s = lo; s < hi; ++s) {
        const uint64_t st = job_state(s, 0);
        if (pcg_out(st) == a && pcg_out(st * kPcgMult) == b) found[t].push_back((uint32_t)s);
      }
    });
  for (auto& th : pool) th.join();
  for (auto& f : found) out.insert(out.end(), f.begin(), f.end());
  return VPT_OK;
}

template <class RNG>
int rng_seed(const RNG& rng, uint32_t& seed, int device = -1) {
  if constexpr (requires { rng.seed(); }) {
    seed = (uint32_t)rng.seed();
    return VPT_OK;
  } else {
    RNG r = rng;  // passed by value to run() as well: its state is ours to use
    r.begin_job(0);
    const uint32_t a = r.template uniform<uint32_t>(), b = r.template uniform<uint32_t>();
    static std::mutex mu;
    static std::map<std::pair<uint32_t, uint32_t>, std::vector<uint32_t>> cache;
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find({a, b});
    if (it == cache.end()) {
      std::vector<uint32_t> found;
      if (int rc = seeds_for(a, b, device, found)) return rc;
      it = cache.emplace(std::make_pair(a, b), std::move(found)).first;
    }
    if (it->second.size() != 1) return VPT_E_STATE;
    seed = it->second[0];
    return VPT_OK;
  }
}

// The process's one driving run() call: the first caller takes every token and drives every GPU
// (drain_devices); callers that find it taken return at once, as the reference's surplus workers would find the
// provider dry.  Released when that call returns (a later frame's run() may lead).
struct Leader {
  static std::mutex& mu() {
    static std::mutex m;
    return m;
  }
  static bool& busy() {
    static bool b = false;
    return b;
  }
  bool leads = false;
  Leader() {
    std::lock_guard<std::mutex> l(mu());
    if (!busy()) busy() = leads = true;
  }
  ~Leader() {
    if (!leads) return;
    std::lock_guard<std::mutex> l(mu());
    busy() = false;
  }
  Leader(const Leader&) = delete;
  Leader& operator=(const Leader&) = delete;
};

template <class V3>
void copy3(float* dst, const V3& v) {
  for (int i = 0; i < 3; ++i) dst[i] = (float)v[i];
}

// (jid, {x0, y0, w, h}) of the tokens of a first batch.  The tile size is the largest rect
// (compute_tile_rect clips only the last column / row, tile_provider.cpp:95-105); false when some
// rect does not follow the jid -> (tile = jid % T, rect) mapping that size implies.
using TokenRects = std::vector<std::pair<uint64_t, std::array<int64_t, 4>>>;
inline bool tile_size_from_rects(const TokenRects& rects, int64_t W, int64_t H, int64_t& tw, int64_t& th) {
  tw = th = 0;
  for (const auto& e : rects) {
    tw = std::max(tw, e.second[2]);
    th = std::max(th, e.second[3]);
  }
  if (tw <= 0 || th <= 0) return false;
  const int64_t ntx = (W + tw - 1) / tw, nty = (H + th - 1) / th;
  const uint64_t T = (uint64_t)(ntx * nty);
  for (const auto& e : rects) {
    const uint64_t tile = e.first % T;
    const int64_t x0 = (int64_t)(tile % (uint64_t)ntx) * tw, y0 = (int64_t)(tile / (uint64_t)ntx) * th;
    if (e.second[0] != x0 || e.second[1] != y0 || e.second[2] != std::min(tw, W - x0) || e.second[3] != std::min(th, H - y0))
      return false;
  }
  return true;
}

struct OwnedDesc {
  vpt_grid_desc* d = nullptr;
  ~OwnedDesc() {
    if (d) vpt_grid_free(d);
  }
};
struct OwnedGrids {
  vpt_host_grids* g = nullptr;
  ~OwnedGrids() { vpt_grids_free(g); }
};

// VPT_DEVICES=n: use at most n of the process's HIP devices (A/B runs); default all of them.
inline int device_limit(int n) {
  const char* e = std::getenv("VPT_DEVICES");
  return e && std::atoi(e) > 0 ? std::min(n, std::atoi(e)) : n;
}

}  // namespace detail

// What the last run() that drove the GPUs spent where (ms), as main.cpp:65-84 times the whole call -- for
// reports (the bench's `first_call`).  Written by that call's thread; read after it has returned.
struct RunPhases {
  int devices = 0;
  double first_batch_ms = 0;  // the first batch of tokens (the tile size is read off it)
  double hip_ms = 0;          // the HIP runtime's start (the process's first HIP call: the device count) and
  double seed_ms = 0;         // the RandomNumberGenerator's private seed, recovered on the GPU -- both on a helper
                              // thread, beside:
  double nanogrid_ms = 0;     // the NanoGrid<float>s read into grid descriptions (vpt_grid_from_nanovdb) and
  double flatten_ms = 0;      // the grids flattened + the density's majorants fixed (vpt_grids_flatten)
  double wait_ms = 0;         // then the wait for the helper thread
  double contexts_ms = 0;     // vpt_gpu_create_from + feed memory + tile costs on every GPU (in parallel)
  double feeds_ms = 0;        // the share of contexts_ms after vpt_gpu_create_from: feed memory + tile costs
  double setup_ms[5] = {};    // the first GPU's context: flatten + majorant fix (= flatten_ms), upload, the rest,
                              // tile costs, bind
  double frame_ms = 0;        // drain_devices: the frame itself
  double total_ms = 0;        // the whole run() call
};
inline RunPhases& run_phases() {
  static RunPhases p;
  return p;
}

// vpt::run with the reference's signature; returns VPT_OK or an error code (see run()).
template <class WorkerParameters, class Volume, class Camera, class TileProvider, class Image, class RNG>
int run_checked(const WorkerParameters& params, const Volume& vol, const Camera& camera, TileProvider& tp, Image& film,
                RNG rng, uint64_t first_batch = 4096) {
  const detail::Leader lead;
  // Another worker thread drives every GPU and takes every token: return (taking tokens for it was measured
  // 13-16x slower per token -- the provider's one job counter -- r05, vpt_run.hpp Helpers).
  if (!lead.leads) return VPT_OK;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  auto t = t0;
  auto lap = [&](double& into) {
    const auto now = clk::now();
    into = std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
  };
  RunPhases ph;
  const auto size = film.size();
  const int64_t W = (int64_t)size.x(), H = (int64_t)size.y();
  // First batch of tokens: the tile size is the largest rect (tile_provider.cpp:95-105 clips only the
  // last column / row), then every rect must match the jid -> (tile, rect) mapping it implies.
  JobRuns runs;
  detail::TokenRects rects;
  const uint64_t taken = take_jobs(tp, first_batch, runs, [&](auto& tok) {
    const auto r = tok.compute_rect();
    rects.push_back({(uint64_t)tok.jid(), {(int64_t)r.start.x(), (int64_t)r.start.y(), (int64_t)r.size.x(), (int64_t)r.size.y()}});
  });
  if (taken == 0) return VPT_OK;  // the provider is dry: nothing to build
  int64_t tw = 0, th = 0;
  if (!detail::tile_size_from_rects(rects, W, H, tw, th)) {
    std::fprintf(stderr, "vpt_gpu::run: token rects do not follow one tile size (%lld x %lld)\n", (long long)tw,
                 (long long)th);
    return VPT_E_STATE;
  }
  lap(ph.first_batch_ms);

  // the film in wave order, bit-identical to the reference's (VPT_DROPIN_ORDERED=0: the feeds' atomics alone)
  DrainOptions dopt;
  const char* ord = std::getenv("VPT_DROPIN_ORDERED");
  dopt.ordered_frame = !(ord && std::atoi(ord) == 0);
  if (const char* db = std::getenv("VPT_DROPIN_DIRECT_BELOW"))  // (tests: 1 = a feed even for a small frame)
    dopt.direct_below = (uint64_t)std::atoll(db);
  // An ordered frame is sized from progress() (detail::take_until_sized): the tokens up to 1 % of the frame are
  // taken on a thread of their own beside the setup below, so one GPU's frame memory is allocated with its context.
  bool dry = false;
  std::thread sizer;
  if (dopt.ordered_frame) sizer = std::thread([&] { (void)detail::take_until_sized(tp, 4096, runs, dry); });
  struct Join {
    std::thread& t;
    ~Join() {
      if (t.joinable()) t.join();
    }
  } join_sizer{sizer};

  // The HIP runtime's start and the seed recovery (one GPU launch) run on a helper thread while this one reads
  // the NanoGrids and flattens them (host work): their phases overlap.
  vpt_configuration cfg;
  std::memset(&cfg, 0, sizeof cfg);
  int ndev = 0, gpu_rc = VPT_OK;
  std::thread gpu_side([&] {
    auto g0 = clk::now();
    if (vpt_gpu_device_count(&ndev) || ndev <= 0) {
      std::fprintf(stderr, "vpt_gpu::run: no HIP device (the integrator has no CPU fallback)\n");
      gpu_rc = VPT_E_HIP;
      return;
    }
    ph.hip_ms = std::chrono::duration<double, std::milli>(clk::now() - g0).count();
    g0 = clk::now();
    if ((gpu_rc = detail::rng_seed(rng, cfg.seed, 0)))  // (vpt_last_error is per thread: say it here)
      std::fprintf(stderr, "vpt_gpu::run: the RandomNumberGenerator's seed could not be determined (%s)\n", vpt_last_error());
    ph.seed_ms = std::chrono::duration<double, std::milli>(clk::now() - g0).count();
  });
  const auto& grids = vol.grids();
  detail::OwnedDesc dens, temp;
  int grid_rc = vpt_grid_from_nanovdb(&grids.density(), (size_t)grids.density().gridSize(), &dens.d);
  if (grid_rc == VPT_OK && grids.has_temperature())
    grid_rc = vpt_grid_from_nanovdb(&grids.temperature(), (size_t)grids.temperature().gridSize(), &temp.d);
  lap(ph.nanogrid_ms);
  detail::OwnedGrids flat;
  if (grid_rc == VPT_OK) grid_rc = vpt_grids_flatten(dens.d, temp.d, &flat.g);
  lap(ph.flatten_ms);
  if (grid_rc)  // (vpt_last_error is per thread: say it here)
    std::fprintf(stderr, "vpt_gpu::run: the grids could not be read (%s)\n", vpt_last_error());
  gpu_side.join();
  lap(ph.wait_ms);
  if (grid_rc) return grid_rc;
  if (gpu_rc) return gpu_rc;
  ndev = detail::device_limit(ndev);
  cfg.num_waves = 1;  // the provider decides which waves run; the context renders any job id
  cfg.num_workers = 1;
  cfg.output_size[0] = W;
  cfg.output_size[1] = H;
  cfg.tile_size[0] = tw;
  cfg.tile_size[1] = th;
  const auto& cp = camera.params();
  detail::copy3(cfg.camera_parameters.position, cp.position);
  detail::copy3(cfg.camera_parameters.look, cp.look);
  detail::copy3(cfg.camera_parameters.up, cp.up);
  cfg.camera_parameters.vfov_deg = cp.vfov_deg;
  cfg.camera_parameters.imaging_ratio = cp.imaging_ratio;
  vpt_worker_params& wp = cfg.worker_parameters;
  wp.single_pixel_enabled = params.single_pixel.enabled ? 1 : 0;
  wp.single_pixel_coord[0] = (int64_t)params.single_pixel.coord.x();
  wp.single_pixel_coord[1] = (int64_t)params.single_pixel.coord.y();
  wp.use_jitter = params.use_jitter ? 1 : 0;
  detail::copy3(wp.infinite_light_xyz, params.infinite_light.xyz);
  wp.infinite_light_multiplier = params.infinite_light.multiplier;
  detail::copy3(wp.distant_light_xyz, params.distant_light.xyz);
  wp.distant_light_multiplier = params.distant_light.multiplier;
  detail::copy3(wp.distant_light_inv_direction, params.distant_light.inv_direction);
  wp.max_depth = params.max_depth;
  const auto& vp = vol.params();
  cfg.volume_parameters = vpt_volume_params{vp.henyey_greenstein_g, vp.le_scale,          vp.sigma_a,
                                            vp.sigma_s,             vp.temperature_offset, vp.temperature_scale};


  // A context per GPU: the grids flattened and majorant-fixed once (above), uploaded to every device in parallel
  // (vpt_gpu_create_from); the feed's pinned ring and copy buffers and the tile costs of its cost tail are setup
  // too, like the grid upload.
  std::vector<vpt_gpu_ctx*> ctxs((size_t)ndev, nullptr);
  struct Ctxs {
    std::vector<vpt_gpu_ctx*>& c;
    ~Ctxs() {
      for (auto* x : c)
        if (x) vpt_gpu_destroy(x);
    }
  } guard{ctxs};
  std::vector<int> devices((size_t)ndev);
  for (int d = 0; d < ndev; ++d) devices[(size_t)d] = d;
  if (int rc = vpt_gpu_create_from(&cfg, flat.g, nullptr, devices.data(), ndev, ctxs.data())) return rc;
  const auto t_feeds = clk::now();
  std::vector<int> crc((size_t)ndev, VPT_OK);
  if (sizer.joinable()) sizer.join();
  auto prepare = [&](int d) {
    int rc = vpt_gpu_feed_prepare(ctxs[(size_t)d], 0, 1);
    if (rc == VPT_OK) rc = vpt_gpu_tile_costs(ctxs[(size_t)d], nullptr, nullptr);
    if (rc == VPT_OK && dopt.ordered_frame && ndev == 1) {  // the frame's memory now (drain's frame then reuses it)
      uint64_t T = 0, total = 0, none = 0;
      if ((rc = vpt_gpu_job_space(ctxs[0], &T, &total)) == VPT_OK) {
        FeedPipeline::Frame fr = detail::frame_of(tp, runs, T, 0, (uint32_t)T, nullptr, dry);
        int blocks = 0, threads = 0;
        (void)vpt_gpu_launch_info(ctxs[0], &blocks, &threads);
        const bool small = fr.waves < (~0ULL >> 8) && fr.waves * T < (uint64_t)blocks * (uint64_t)threads;  // (no feed)
        if (!small && vpt_gpu_frame_open(ctxs[0], fr.jid_lo, &fr.waves, 0, (uint32_t)T) == VPT_OK)
          (void)vpt_gpu_frame_open(ctxs[0], 0, &none, 0, 0);
      }
    }
    if (rc != VPT_OK)  // (vpt_last_error is per thread: say it here)
      std::fprintf(stderr, "vpt_gpu::run: device %d: %s\n", d, vpt_last_error());
    crc[(size_t)d] = rc;
  };
  if (ndev == 1) {
    prepare(0);
  } else {
    std::vector<std::thread> pool;
    for (int d = 0; d < ndev; ++d) pool.emplace_back(prepare, d);
    for (auto& th2 : pool) th2.join();
  }
  for (int rc : crc)
    if (rc) return rc;
  ph.feeds_ms = std::chrono::duration<double, std::milli>(clk::now() - t_feeds).count();
  lap(ph.contexts_ms);
  (void)vpt_gpu_setup_timings(ctxs[0], ph.setup_ms, 5);
  ph.devices = ndev;
  float* film_host = reinterpret_cast<float*>(film.data().data());  // H x W x (X, Y, Z, W)
  // the first batch is queued first; then 4096 tokens per batch (a token is one 8x8 job: 64 samples)
  // The host copies of the grids (the devices hold theirs) are kept until the next run() or the process's exit,
  // as the reference's Volume keeps its grids: unmapping ~1 GB of pages took 58-97 ms on the box, and slowed the
  // frame by 46-92 ms when done beside it (r06o, r06p: mmap-lock contention).  One run() drives the GPUs at a time
  // (Leader), so the slot is never shared; flat now holds the previous call's copies, released at this call's end.
  static detail::OwnedGrids kept;
  std::swap(kept.g, flat.g);
  const int rc = drain_devices(ctxs, tp, film_host, 4096, dopt, &runs);
  lap(ph.frame_ms);
  ph.total_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  run_phases() = ph;
  return rc;
}

template <class WorkerParameters, class Volume, class Camera, class TileProvider, class Image, class RNG>
void run(const WorkerParameters& params, const Volume& vol, const Camera& camera, TileProvider& tp, Image& film,
         RNG rng) {
  if (int rc = run_checked(params, vol, camera, tp, film, rng)) {
    std::fprintf(stderr, "[FATAL] vpt_gpu::run failed (%d): %s\n", rc, vpt_last_error());
    std::exit(1);  // vptFATAL (include/vpt/logging.hpp:16)
  }
}

}  // namespace vpt_gpu
