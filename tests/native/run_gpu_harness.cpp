// run_gpu_harness.cpp — TEST HARNESS: main.cpp:46-87 headless over the restated TileProvider, with
// the reference-side drop-in of include/vpt_run.hpp in place of vpt::run.  N host threads share one
// provider and one host film, which is written to a file for tests/test_gpu_integration.py to compare
// with the oracle.
//
//   run_gpu_harness config=<scene.json> out=<film.f32> [mode=drain|run w= h= waves= threads= batch=
//                   grid_n= kind= dist= temperature=0|1 stop_after=<jobs> nvdb=<file.nvdb> gridbuf=<file> taker_node=<n>
//                   tempbuf=<file> hold= backlog= flush_ms= cost_tail= cost_chunks= helpers= grid_blocks= sample_ms= frames= warmup=]
//
// mode=drain (default): each thread owns a context made with vpt_gpu_create and calls
//   vpt_gpu::drain(ctx, tp, film, batch).  The volume is nvdb= (vpt_grid_read_nvdb: "density", and
//   "temperature" when present) or the product library's synthetic stand-in (cloud density, plus the
//   40*base temperature grid with temperature=1).
// multi=1 (mode=drain): one thread drives every context through vpt_gpu::drain_devices, as run() drives the GPUs.
// mode=seed: the private seed recovered from the RNG's job-0 stream (device=-1: host threads; else that GPU).
// mode=run: each thread calls vpt_gpu::run(params, vol, camera, tp, film, rng) with the reference's
//   own argument types (tests/native/reference_types_headless.hpp), exactly as main.cpp:63-68 calls
//   vpt::run; the volume is the NanoGrid<float> bytes of gridbuf= (and tempbuf=), the seed is private
//   to the RandomNumberGenerator.
// The camera looks at the volume from (0, 0, -dist) unless dist=0 (then the scene file's camera).
// stop_after: after that many jobs thread 0 calls tp.stop_at_next_wave() (tile_provider.cpp:107-110).
// hold / backlog / flush_ms / cost_tail: vpt_gpu::DrainOptions of mode=drain; helpers: threads that take tokens for the drain
// threads (vpt_gpu::help, as run()'s threads that find every GPU driven); grid_blocks: vpt_gpu_set_tuning's grid override.
// mode=tokens (no GPU): the provider alone -- `threads` threads take every token of the frame and release it at once, the
// drop-in's host-side floor (r05) -- printed as tokens_ms and M tokens/s.
// sample_ms: a thread samples, every sample_ms, the jobs handed out and the samples in the host film (what
// main.cpp's 5-FPS window shows: film_to_image(film) and provider.progress(), main.cpp:101-132) and prints
// them as "sample <ms> <waves handed out> <waves in the film>".  The render time is printed as render_ms.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <array>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include <pthread.h>
#include <sched.h>

#include "reference_types_headless.hpp"
#include "tile_provider_headless.hpp"
#include "vpt_run.hpp"

namespace {

// A provider that forwards to the restated TileProvider and, once, stops at the next wave.  It counts the
// tokens only when something reads the count (stop_after, sample_ms): a counter's atomic add per token would
// time this frame ~20 ms slower than the frames=/warmup= frames, which take the provider as it is (C4, r05).
struct StoppingProvider {
  vpt_headless::TileProvider& tp;
  uint64_t stop_after;
  bool count;
  std::atomic<uint64_t> handed{0};
  vpt_headless::TileProvider::token next() {
    if (count && handed.fetch_add(1) + 1 == stop_after) tp.stop_at_next_wave();
    return tp.next();
  }
  unsigned progress() const { return tp.progress(); }
};

int fail(const char* what) {
  std::fprintf(stderr, "run_gpu_harness: %s: %s\n", what, vpt_last_error());
  return 1;
}

std::vector<char> slurp(const std::string& path) {
  std::ifstream in(path, std::ios::binary);
  return std::vector<char>((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
}

vpt_headless::Vector3f v3(const float* f) { return vpt_headless::Vector3f{{f[0], f[1], f[2]}}; }

// taker_node=N: the driving threads (the takers) run on NUMA node N's CPUs (/sys cpulist); -1: wherever
void pin_to_node(long long node) {
  if (node < 0) return;
  std::ifstream in("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string list;
  if (!std::getline(in, list)) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (size_t pos = 0; pos < list.size();) {
    size_t end = list.find(',', pos);
    if (end == std::string::npos) end = list.size();
    const std::string r = list.substr(pos, end - pos);
    const size_t dash = r.find('-');
    const int a = std::atoi(r.c_str()), b = dash == std::string::npos ? a : std::atoi(r.c_str() + dash + 1);
    for (int c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET(c, &set);
    pos = end + 1;
  }
  (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
}

}  // namespace

int main(int argc, char** argv) {
  std::setvbuf(stdout, nullptr, _IOLBF, 0);  // (lines survive a run killed at its time limit)
  std::map<std::string, std::string> a;
  for (int i = 1; i < argc; ++i) {
    const char* eq = std::strchr(argv[i], '=');
    if (!eq) {
      std::fprintf(stderr, "run_gpu_harness: bad argument %s\n", argv[i]);
      return 2;
    }
    a[std::string(argv[i], eq - argv[i])] = eq + 1;
  }
  auto num = [&](const char* k, long long d) { return a.count(k) ? std::atoll(a[k].c_str()) : d; };
  if (!a.count("config") || !a.count("out")) {
    std::fprintf(stderr, "run_gpu_harness: config= and out= are required\n");
    return 2;
  }
  vpt_configuration cfg;
  if (vpt_config_read(a["config"].c_str(), &cfg)) return fail("vpt_config_read");
  cfg.output_size[0] = num("w", cfg.output_size[0]);
  cfg.output_size[1] = num("h", cfg.output_size[1]);
  cfg.num_waves = (uint32_t)num("waves", cfg.num_waves);
  const int grid_n = (int)num("grid_n", 64);
  const float dist = (float)num("dist", 800 * grid_n / 512);
  if (dist != 0.0f) {
    const float cam[9] = {0, 0, -dist, 0, 0, 0, 0, 1, 0};
    std::memcpy(cfg.camera_parameters.position, cam, 3 * sizeof(float));
    std::memcpy(cfg.camera_parameters.look, cam + 3, 3 * sizeof(float));
    std::memcpy(cfg.camera_parameters.up, cam + 6, 3 * sizeof(float));
  }
  const int threads = (int)num("threads", 2);
  const uint64_t batch = (uint64_t)num("batch", 1000);
  const std::string mode = a.count("mode") ? a["mode"] : "drain";

  // main.cpp:46-55: provider and film; then num_workers threads (main.cpp:62-68)
  vpt_headless::TileProvider tp(cfg.output_size[0], cfg.output_size[1], cfg.num_waves, cfg.tile_size[0],
                                cfg.tile_size[1]);
  StoppingProvider sp{tp, (uint64_t)num("stop_after", 0), num("stop_after", 0) > 0 || num("sample_ms", 0) > 0};
  vpt_headless::Image<float, 4> film(cfg.output_size[0], cfg.output_size[1]);
  std::vector<int> rc(threads, 0);

  // the 5-FPS window of main.cpp:101-132, headless: what a viewer would see while the GPU renders
  const long long sample_ms = num("sample_ms", 0);
  std::atomic<bool> rendering{true};
  std::vector<std::array<double, 3>> samples;
  const auto t0 = std::chrono::steady_clock::now();
  auto sampler = [&] {
    const double T = (double)tp.num_tiles(), px = (double)cfg.output_size[0] * (double)cfg.output_size[1];
    while (rendering.load()) {
      double w = 0.0;
      for (size_t i = 3; i < film.px.size() * 4; i += 4) w += (double)reinterpret_cast<const float*>(film.px.data())[i];
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      samples.push_back({ms, (double)sp.handed.load() / T, w / px});
      std::this_thread::sleep_for(std::chrono::milliseconds(sample_ms));
    }
  };
  std::thread sampler_thread;

  if (mode == "seed") {  // the drop-in's seed recovery: the RNG's seed is private (device=-1: host threads, no GPU)
    vpt_headless::RandomNumberGenerator rng(cfg.seed);
    uint32_t seed = 0;
    int ndev = 0;
    if (num("device", -1) >= 0 && (vpt_gpu_device_count(&ndev) || ndev <= 0)) return fail("no HIP device");  // (runtime start: not timed)
    const auto s0 = std::chrono::steady_clock::now();
    const int r = vpt_gpu::detail::rng_seed(rng, seed, (int)num("device", -1));
    std::printf("run_gpu_harness: seed %d %u %.1f ms\n", r, seed,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - s0).count());
    return 0;
  }
  if (mode == "tiles") {  // the drop-in's tile-size derivation from a first batch of `batch` tokens (no GPU)
    vpt_gpu::detail::TokenRects rects;
    vpt_gpu::JobRuns runs;
    vpt_gpu::take_jobs(sp, batch, runs, [&](auto& t) {
      const auto r = t.compute_rect();
      rects.push_back({(uint64_t)t.jid(), {r.start.x(), r.start.y(), r.size.x(), r.size.y()}});
    });
    int64_t tw = 0, th = 0;
    const bool ok = vpt_gpu::detail::tile_size_from_rects(rects, cfg.output_size[0], cfg.output_size[1], tw, th);
    std::printf("run_gpu_harness: tiles %d %lld %lld %zu\n", ok ? 1 : 0, (long long)tw, (long long)th, runs.size());
    return 0;
  }
  if (mode == "tokens") {
    std::vector<std::thread> pool;
    std::vector<uint64_t> got(threads, 0);
    const auto r0 = std::chrono::steady_clock::now();
    for (int i = 0; i < threads; ++i)
      pool.emplace_back([&, i] {
        vpt_gpu::JobRuns runs;
        while (uint64_t n = vpt_gpu::take_jobs(sp, 4096, runs, [](auto&) {})) got[i] += n;
      });
    for (auto& t : pool) t.join();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - r0).count();
    uint64_t n = 0;
    for (uint64_t g : got) n += g;
    std::printf("run_gpu_harness: tokens_ms %.1f, %llu tokens, %.1f M tokens/s, %d threads\n", ms, (unsigned long long)n,
                n / ms / 1e3, threads);
    return 0;
  }
  if (mode == "run") {
    // The reference's objects, built from the same configuration as main.cpp builds them.
    const std::vector<char> gbuf = slurp(a["gridbuf"]), tbuf = a.count("tempbuf") ? slurp(a["tempbuf"]) : std::vector<char>();
    if (gbuf.size() < 672) return fail("gridbuf");
    const vpt_worker_params& w = cfg.worker_parameters;
    vpt_headless::WorkerParameters params{{w.single_pixel_enabled != 0, {{w.single_pixel_coord[0], w.single_pixel_coord[1]}}},
                                          w.use_jitter != 0,
                                          {v3(w.infinite_light_xyz), w.infinite_light_multiplier},
                                          {v3(w.distant_light_xyz), w.distant_light_multiplier, v3(w.distant_light_inv_direction)},
                                          w.max_depth};
    const vpt_volume_params& v = cfg.volume_parameters;
    vpt_headless::Volume vol{{reinterpret_cast<const vpt_headless::NanoGridF*>(gbuf.data()),
                              tbuf.empty() ? nullptr : reinterpret_cast<const vpt_headless::NanoGridF*>(tbuf.data())},
                             {v.henyey_greenstein_g, v.le_scale, v.sigma_a, v.sigma_s, v.temperature_offset, v.temperature_scale}};
    const vpt_camera_params& c = cfg.camera_parameters;
    vpt_headless::Camera camera{{v3(c.position), v3(c.look), v3(c.up), c.vfov_deg, c.imaging_ratio}};
    std::vector<std::thread> pool;
    if (sample_ms > 0) sampler_thread = std::thread(sampler);
    for (int i = 0; i < threads; ++i)
      pool.emplace_back([&, i] {
        vpt_headless::RandomNumberGenerator rng(cfg.seed);
        rc[i] = vpt_gpu::run_checked(params, vol, camera, sp, film, rng);  // vpt::run(...) in main.cpp
      });
    for (auto& t : pool) t.join();
    for (int i = 0; i < threads; ++i)
      if (rc[i]) return fail("vpt_gpu::run");
    // frames=k: k - 1 more frames in this process, each with a fresh provider and film, as a caller that renders
    // again would (the later calls release the previous call's host grid copies); `out` gets the last film
    for (long long f = 1; f < num("frames", 1); ++f) {
      vpt_headless::TileProvider tp2(cfg.output_size[0], cfg.output_size[1], cfg.num_waves, cfg.tile_size[0],
                                     cfg.tile_size[1]);
      vpt_headless::Image<float, 4> film2(cfg.output_size[0], cfg.output_size[1]);
      const auto f0 = std::chrono::steady_clock::now();
      std::vector<std::thread> pool2;
      for (int i = 0; i < threads; ++i)
        pool2.emplace_back([&, i] {
          vpt_headless::RandomNumberGenerator rng(cfg.seed);
          rc[i] = vpt_gpu::run_checked(params, vol, camera, tp2, film2, rng);
        });
      for (auto& t : pool2) t.join();
      for (int i = 0; i < threads; ++i)
        if (rc[i]) return fail("vpt_gpu::run (a later frame)");
      std::printf("run_gpu_harness: frame %lld total_ms=%.1f\n", f,
                  std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - f0).count());
      film.px = film2.px;
    }
    // what the call cost, as main.cpp:65-84 times it (the whole run(); its phases)
    const vpt_gpu::RunPhases& ph = vpt_gpu::run_phases();
    std::printf("run_gpu_harness: phases devices=%d total_ms=%.1f hip_ms=%.1f first_batch_ms=%.1f seed_ms=%.1f "
                "nanogrid_ms=%.1f flatten_ms=%.1f wait_ms=%.1f contexts_ms=%.1f feeds_ms=%.1f flatten_fix_ms=%.1f upload_ms=%.1f ctx_rest_ms=%.1f tile_costs_ms=%.1f "
                "bind_ms=%.1f frame_ms=%.1f\n",
                ph.devices, ph.total_ms, ph.hip_ms, ph.first_batch_ms, ph.seed_ms, ph.nanogrid_ms, ph.flatten_ms, ph.wait_ms, ph.contexts_ms,
                ph.feeds_ms, ph.setup_ms[0], ph.setup_ms[1], ph.setup_ms[2], ph.setup_ms[3], ph.setup_ms[4], ph.frame_ms);
  } else {
    vpt_grid_desc *dens = nullptr, *temp = nullptr;
    if (a.count("nvdb")) {
      if (vpt_grid_read_nvdb(a["nvdb"].c_str(), "density", &dens) || !dens) return fail("vpt_grid_read_nvdb density");
      if (vpt_grid_read_nvdb(a["nvdb"].c_str(), "temperature", &temp)) return fail("vpt_grid_read_nvdb temperature");
    } else {
      dens = vpt_synth_grid((int)num("kind", 1), grid_n);  // kind 0: C2's constant cube
      temp = num("temperature", 0) ? vpt_synth_grid(2, grid_n) : nullptr;
      if (!dens || (num("temperature", 0) && !temp)) return fail("vpt_synth_grid");
    }
    std::vector<vpt_gpu_ctx*> ctx(threads, nullptr);
    const int ndev = (int)num("devices", 1);
    // multi=1: one thread drives all `threads` contexts (vpt_gpu::drain_devices, what run() does with the
    // process's GPUs); contexts go to devices i % devices
    const bool multi = num("multi", 0) != 0;
    for (int i = 0; i < threads; ++i)
      if (vpt_gpu_create(&cfg, dens, temp, nullptr, i % ndev, &ctx[i])) return fail("vpt_gpu_create");
    float* fh = reinterpret_cast<float*>(film.data().data());
    vpt_gpu::DrainOptions opt;
    opt.hold_jobs = (uint64_t)num("hold", (long long)opt.hold_jobs);
    opt.backlog_jobs = (uint64_t)num("backlog", (long long)opt.backlog_jobs);
    opt.cost_tail = num("cost_tail", opt.cost_tail ? 1 : 0) != 0;
    opt.cost_chunks = num("cost_chunks", opt.cost_chunks ? 1 : 0) != 0;
    opt.direct_below = (uint64_t)num("direct_below", (long long)opt.direct_below);
    opt.flush_seconds = (double)num("flush_ms", (long long)(opt.flush_seconds * 1000)) / 1000.0;
    opt.ordered_frame = num("ordered", 0) != 0;  // (one taker only: multi=1, or one drain thread without helpers)
    if (num("grid_blocks", 0) > 0)
      for (auto* c : ctx)
        if (vpt_gpu_set_tuning(c, 0, -1, (int)num("grid_blocks", 0), 0, -1)) return fail("vpt_gpu_set_tuning");
    for (auto* c : ctx)  // setup outside the timed render, as run_checked does it: the tile-cost pass, the feed's memory
      if (vpt_gpu_tile_costs(c, nullptr, nullptr) || vpt_gpu_feed_prepare(c, 0, 1) || vpt_gpu_sync(c)) return fail("warm-up");
    // frames=N: N - 1 more frames first, each with a fresh provider and film (main.cpp renders one frame per
    // process: these time the same drain again, on the contexts already built), one render_ms line each;
    // warmup=M: M more such frames before them, untimed (a GPU coming out of idle clocks up over the first ones)
    const long long warm = num("warmup", 0);
    for (long long fr = 1 - warm; fr < num("frames", 1); ++fr) {
      vpt_headless::TileProvider tp2(cfg.output_size[0], cfg.output_size[1], cfg.num_waves, cfg.tile_size[0], cfg.tile_size[1]);
      vpt_headless::Image<float, 4> film2(cfg.output_size[0], cfg.output_size[1]);
      float* fh2 = reinterpret_cast<float*>(film2.data().data());
      const auto r0 = std::chrono::steady_clock::now();
      std::vector<std::thread> pool;
      if (multi)
        pool.emplace_back([&] {
          pin_to_node(num("taker_node", -1));
          rc[0] = vpt_gpu::drain_devices(ctx, tp2, fh2, batch, opt);
        });
      else
        for (int i = 0; i < threads; ++i)
          pool.emplace_back([&, i] {
            pin_to_node(num("taker_node", -1));
            rc[i] = vpt_gpu::drain(ctx[i], tp2, fh2, batch, opt);
          });
      for (auto& t : pool) t.join();
      for (int i = 0; i < threads; ++i)
        if (rc[i]) return fail("vpt_gpu::drain");
      std::printf("run_gpu_harness: %s %.1f\n", fr < 1 ? "warmup_ms" : "render_ms",
                  std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - r0).count());
    }
    {
      const auto r0 = std::chrono::steady_clock::now();
      if (sample_ms > 0) sampler_thread = std::thread(sampler);
      std::vector<std::thread> pool;
      // helpers=N: N more threads take tokens for the drivers (vpt_gpu::help, as run()'s non-driving threads do)
      const int helpers = multi ? 0 : (int)num("helpers", 0);
      if (multi)  // (pool[0] .. pool[threads - 1] are joined below: the other slots are empty threads)
        for (int i = 0; i < threads; ++i)
          pool.emplace_back([&, i] {
            pin_to_node(num("taker_node", -1));
            if (i == 0) rc[0] = vpt_gpu::drain_devices(ctx, sp, fh, batch, opt);
          });
      else
        for (int i = 0; i < threads; ++i)
          pool.emplace_back([&, i] {
            pin_to_node(num("taker_node", -1));
            rc[i] = vpt_gpu::drain(ctx[i], sp, fh, batch, opt, nullptr, helpers > 0);
          });
      std::vector<int> hrc(helpers, 0);
      {
        // the drivers register their pipelines as they start; helpers wait for one (Helpers::drivers counts
        // the devices claimed by run(), which drain mode bypasses: count the drivers here instead)
        std::lock_guard<std::mutex> l(vpt_gpu::detail::Helpers::get().mu);
        vpt_gpu::detail::Helpers::get().drivers += helpers > 0 ? threads : 0;
      }
      for (int i = 0; i < helpers; ++i) pool.emplace_back([&, i] { hrc[i] = vpt_gpu::help(sp, batch); });
      for (int i = 0; i < threads; ++i) pool[i].join();
      {
        std::lock_guard<std::mutex> l(vpt_gpu::detail::Helpers::get().mu);
        vpt_gpu::detail::Helpers::get().drivers -= helpers > 0 ? threads : 0;
        vpt_gpu::detail::Helpers::get().cv.notify_all();
      }
      for (size_t i = threads; i < pool.size(); ++i) pool[i].join();
      for (int r : hrc)
        if (r) return fail("vpt_gpu::help");
      std::printf("run_gpu_harness: render_ms %.1f\n",
                  std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - r0).count());
    }
    for (int i = 0; i < threads; ++i)
      if (rc[i]) {  // (the message was set on the worker thread: vpt_last_error is per thread)
        std::fprintf(stderr, "run_gpu_harness: vpt_gpu::drain on thread %d returned %d\n", i, rc[i]);
        return 1;
      }
    for (auto* c : ctx) vpt_gpu_destroy(c);
    vpt_grid_free(dens);
    if (temp) vpt_grid_free(temp);
  }

  rendering.store(false);
  if (sampler_thread.joinable()) sampler_thread.join();
  for (const auto& e : samples) std::printf("sample %.1f %.3f %.3f\n", e[0], e[1], e[2]);

  FILE* f = std::fopen(a["out"].c_str(), "wb");
  const size_t n = film.px.size() * 4;
  if (!f || std::fwrite(film.px.data(), sizeof(float), n, f) != n) return fail("write film");
  std::fclose(f);
  std::printf("run_gpu_harness: %s, %d threads, %u waves started, %llu jobs handed out\n", mode.c_str(), threads,
              tp.max_wave_started(),
              (unsigned long long)(sp.count ? sp.handed.load() : (uint64_t)tp.num_tiles() * tp.max_wave_started()));
  return 0;
}
