// tile_provider_headless.hpp — TEST HARNESS: the reference's work distributor, restated without
// Eigen so that run_gpu.hpp (the documented drop-in for vpt::run) can be compiled and driven here.
//
// Semantics restated from the reference (/root/reference, read as text):
//   * job ids from one relaxed fetch_add; wave = 1 + jid / T, tile = jid % T   (src/tile_provider.cpp:27-31)
//   * a job of a wave that was never started, or after stop_now(), yields the invalid token (:33-34)
//   * wave gating: the job waits until the same tile's previous wave has been released, i.e. its
//     token destroyed (:40-60; the token destructor, include/vpt/tile_provider.hpp:22-27)
//   * waves start lazily under a mutex and never beyond requested_waves (:70-90)
//   * compute_tile_rect clips the tile to the image (:95-105); stop_at_next_wave caps the requested
//     waves at the highest wave started so far (:107-110)
//   * progress = jobs handed out / (requested_waves * T) (include/vpt/tile_provider.hpp:66-69)
// The token is non-copyable and non-movable, as in the reference, so callers must consume it in
// place (C++17 guaranteed elision makes `auto t = tp.next();` valid).
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <limits>
#include <mutex>
#include <vector>

namespace vpt_headless {

// image_rect_t (include/vpt/image.hpp:31-38): start and size with Eigen's x() / y()
struct Point {
  int64_t px, py;
  int64_t x() const { return px; }
  int64_t y() const { return py; }
};
struct Rect {
  Point start, size;
};

class TileProvider {
 public:
  using tile_index_t = unsigned int;
  using wave_index_t = unsigned int;

  class token {
   public:
    token(const token&) = delete;
    token& operator=(const token&) = delete;
    token(token&&) = delete;
    token& operator=(token&&) = delete;
    ~token() {
      if (!valid()) return;
      // the tile's `wave` is done: the next wave of this tile may now be handed out
      owner_.tile_wave_[tile_].store(wave_);
      owner_.tile_wave_[tile_].notify_all();
    }
    bool valid() const { return tile_ != kInvalid; }
    explicit operator bool() const { return valid(); }
    size_t wave() const { return wave_; }
    size_t jid() const { return jid_; }
    Rect compute_rect() { return owner_.compute_tile_rect(tile_); }

   private:
    friend class TileProvider;
    static constexpr tile_index_t kInvalid = std::numeric_limits<tile_index_t>::max();
    token(TileProvider& owner, tile_index_t tile, wave_index_t wave, size_t jid)
        : owner_(owner), tile_(tile), wave_(wave), jid_(jid) {}
    TileProvider& owner_;
    tile_index_t tile_;
    wave_index_t wave_;
    size_t jid_;
  };

  TileProvider(int64_t img_w, int64_t img_h, wave_index_t waves, int64_t tile_w, int64_t tile_h)
      : img_w_(img_w), img_h_(img_h), tile_w_(tile_w), tile_h_(tile_h),
        ntx_((img_w + tile_w - 1) / tile_w), nty_((img_h + tile_h - 1) / tile_h),
        requested_waves_(waves), tile_wave_((size_t)(ntx_ * nty_)) {
    for (auto& w : tile_wave_) w.store(0);
  }

  token next() {
    const size_t jid = job_idx_.fetch_add(1, std::memory_order_relaxed);
    const size_t T = tile_wave_.size();
    const wave_index_t wave = (wave_index_t)(1 + jid / T);
    const tile_index_t tile = (tile_index_t)(jid % T);
    if (force_stop_.load() || !start_wave(wave)) return token(*this, token::kInvalid, 0, 0);
    // wait until this tile's previous wave has been released (by whichever thread holds it)
    for (;;) {
      if (force_stop_.load()) return token(*this, token::kInvalid, 0, 0);
      const wave_index_t done = tile_wave_[tile].load(std::memory_order_relaxed);
      if (done == wave - 1) break;
      tile_wave_[tile].wait(done, std::memory_order_relaxed);
    }
    return token(*this, tile, wave, jid);
  }

  void stop_at_next_wave() {
    std::lock_guard<std::mutex> lock(wave_mu_);
    requested_waves_ = max_wave_idx_.load();
  }
  void stop_now() {
    force_stop_.store(true);
    for (auto& w : tile_wave_) w.notify_all();
  }
  unsigned progress() const { return (unsigned)(progress_ratio() * 100.0f); }
  float progress_ratio() const {
    std::lock_guard<std::mutex> lock(wave_mu_);
    return (float)job_idx_.load() / (float)((size_t)requested_waves_ * tile_wave_.size());
  }
  size_t num_tiles() const { return tile_wave_.size(); }
  wave_index_t max_wave_started() const { return max_wave_idx_.load(); }

  Rect compute_tile_rect(tile_index_t tile) const {
    const int64_t x0 = (int64_t)(tile % (tile_index_t)ntx_) * tile_w_;
    const int64_t y0 = (int64_t)(tile / (tile_index_t)ntx_) * tile_h_;
    const int64_t w = img_w_ - x0 < tile_w_ ? img_w_ - x0 : tile_w_;
    const int64_t h = img_h_ - y0 < tile_h_ ? img_h_ - y0 : tile_h_;
    return Rect{Point{x0, y0}, Point{w, h}};
  }

 private:
  bool start_wave(wave_index_t wave) {
    if (wave <= max_wave_idx_.load()) return true;  // already running
    std::lock_guard<std::mutex> lock(wave_mu_);
    if (wave <= max_wave_idx_.load()) return true;
    if (wave > requested_waves_) return false;
    max_wave_idx_.store(wave);
    return true;
  }

  int64_t img_w_, img_h_, tile_w_, tile_h_, ntx_, nty_;
  mutable std::mutex wave_mu_;
  wave_index_t requested_waves_;
  std::atomic<wave_index_t> max_wave_idx_{0};
  std::atomic<bool> force_stop_{false};
  std::atomic<size_t> job_idx_{0};
  std::vector<std::atomic<wave_index_t>> tile_wave_;
};

}  // namespace vpt_headless
