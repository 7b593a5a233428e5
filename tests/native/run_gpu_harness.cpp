// run_gpu_harness.cpp — TEST HARNESS: main.cpp:46-87 headless, with run_gpu (the documented drop-in
// for vpt::run) in place of run, over the restated TileProvider.  N host threads each own one GPU
// context and drain one shared provider into one shared host film, which is written to a file for
// tests/test_gpu_integration.py to compare with the oracle.
//
//   run_gpu_harness config=<scene.json> out=<film.f32> [w= h= waves= threads= batch= grid_n= dist=
//                   temperature=0|1 stop_after=<jobs>]
//
// The volume is the product library's synthetic stand-in (vpt_synth_grid: cloud density, plus the
// 40*base temperature grid with temperature=1); the camera looks at it from (0, 0, -dist).
// stop_after: after that many jobs thread 0 calls tp.stop_at_next_wave() (tile_provider.cpp:107-110).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "run_gpu.hpp"
#include "tile_provider_headless.hpp"

namespace {

// A provider that forwards to the restated TileProvider and, once, stops at the next wave.
struct StoppingProvider {
  vpt_headless::TileProvider& tp;
  uint64_t stop_after;
  std::atomic<uint64_t> handed{0};
  vpt_headless::TileProvider::token next() {
    if (handed.fetch_add(1) + 1 == stop_after) tp.stop_at_next_wave();
    return tp.next();
  }
};

int fail(const char* what) {
  std::fprintf(stderr, "run_gpu_harness: %s: %s\n", what, vpt_last_error());
  return 1;
}

}  // namespace

int main(int argc, char** argv) {
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
  const float cam[9] = {0, 0, -dist, 0, 0, 0, 0, 1, 0};
  std::memcpy(cfg.camera_parameters.position, cam, 3 * sizeof(float));
  std::memcpy(cfg.camera_parameters.look, cam + 3, 3 * sizeof(float));
  std::memcpy(cfg.camera_parameters.up, cam + 6, 3 * sizeof(float));
  const int threads = (int)num("threads", 2);
  const uint64_t batch = (uint64_t)num("batch", 1000);

  vpt_grid_desc* dens = vpt_synth_grid(1, grid_n);
  vpt_grid_desc* temp = num("temperature", 0) ? vpt_synth_grid(2, grid_n) : nullptr;
  if (!dens || (num("temperature", 0) && !temp)) return fail("vpt_synth_grid");

  // main.cpp:46-55: provider and film; then one worker per context (main.cpp:62-68)
  vpt_headless::TileProvider tp(cfg.output_size[0], cfg.output_size[1], cfg.num_waves, cfg.tile_size[0],
                                cfg.tile_size[1]);
  StoppingProvider sp{tp, (uint64_t)num("stop_after", 0)};
  std::vector<float> film((size_t)(cfg.output_size[0] * cfg.output_size[1] * 4), 0.0f);
  std::vector<vpt_gpu_ctx*> ctx(threads, nullptr);
  const int ndev = (int)num("devices", 1);
  for (int i = 0; i < threads; ++i)
    if (vpt_gpu_create(&cfg, dens, temp, nullptr, i % ndev, &ctx[i])) return fail("vpt_gpu_create");
  std::vector<int> rc(threads, 0);
  {
    std::vector<std::thread> pool;
    for (int i = 0; i < threads; ++i)
      pool.emplace_back([&, i] { rc[i] = run_gpu(ctx[i], sp, film.data(), batch); });
    for (auto& t : pool) t.join();
  }
  for (int i = 0; i < threads; ++i)
    if (rc[i]) return fail("run_gpu");
  for (auto* c : ctx) vpt_gpu_destroy(c);
  vpt_synth_free(dens);
  if (temp) vpt_synth_free(temp);

  FILE* f = std::fopen(a["out"].c_str(), "wb");
  if (!f || std::fwrite(film.data(), sizeof(float), film.size(), f) != film.size()) return fail("write film");
  std::fclose(f);
  std::printf("run_gpu_harness: %d threads, %u waves started, %llu jobs handed out\n", threads, tp.max_wave_started(),
              (unsigned long long)sp.handed.load());
  return 0;
}
