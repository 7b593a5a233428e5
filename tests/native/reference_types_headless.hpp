// reference_types_headless.hpp — TEST HARNESS: the reference types vpt::run takes, restated without
// Eigen or NanoVDB with the members and accessors include/vpt_run.hpp reads, so that the drop-in
// vpt_gpu::run can be compiled and called exactly as src/main.cpp:63-68 calls vpt::run.
//
//   WorkerParameters / CameraParameters / VolumeParameters   include/vpt/configuration.hpp:14-59
//   Volume (params(), grids())                               include/vpt/volume.hpp:78-104
//   VolumeGrids (density(), temperature(), has_temperature()) include/vpt/volume_grids.hpp:12-33
//   NanoGrid<float>: the grid's own bytes, gridSize() = GridData::mGridSize (u64 at byte 32)
//   Camera (params())                                        include/vpt/camera.hpp:12-30
//   Image<float, 4> (size(), data().data())                  include/vpt/image.hpp:40-60
//   RandomNumberGenerator: begin_job + uniform<T>, the seed kept private as in random.hpp:86-115
// Eigen vectors become small structs with operator[] / x() / y() (the calls vpt_run.hpp makes).
#pragma once

#include <cstdint>
#include <cstring>
#include <type_traits>
#include <vector>

namespace vpt_headless {

struct Vector3f {
  float v[3];
  float operator[](int i) const { return v[i]; }
};
struct Index2 {
  int64_t v[2];
  int64_t x() const { return v[0]; }
  int64_t y() const { return v[1]; }
};

struct CameraParameters {
  Vector3f position, look, up;
  float vfov_deg, imaging_ratio;
};
struct InfiniteLightParameters {
  Vector3f xyz;
  float multiplier;
};
struct DistantLightParameters {
  Vector3f xyz;
  float multiplier;
  Vector3f inv_direction;
};
struct WorkerParameters {
  struct SinglePixelMode {
    bool enabled;
    Index2 coord;
  } single_pixel;
  bool use_jitter;
  InfiniteLightParameters infinite_light;
  DistantLightParameters distant_light;
  unsigned int max_depth;
};
struct VolumeParameters {
  float henyey_greenstein_g, le_scale, sigma_a, sigma_s, temperature_offset, temperature_scale;
};

// nanovdb::NanoGrid<float>: only ever referenced in place, over the grid's bytes.
struct NanoGridF {
  uint64_t gridSize() const {
    uint64_t n;
    std::memcpy(&n, reinterpret_cast<const char*>(this) + 32, 8);
    return n;
  }
};

struct VolumeGrids {
  const NanoGridF* d = nullptr;
  const NanoGridF* t = nullptr;
  const NanoGridF& density() const { return *d; }
  const NanoGridF& temperature() const { return *t; }
  bool has_temperature() const { return t != nullptr; }
};

struct Volume {
  VolumeGrids g;
  VolumeParameters p;
  const VolumeParameters& params() const { return p; }
  const VolumeGrids& grids() const { return g; }
};

struct Camera {
  CameraParameters p;
  const CameraParameters& params() const { return p; }
};

struct Pixel4 {
  float c[4];
};
template <typename T, int N>
struct Image;
template <>
struct Image<float, 4> {
  int64_t w, h;
  std::vector<Pixel4> px;
  Image(int64_t w_, int64_t h_) : w(w_), h(h_), px((size_t)(w_ * h_), Pixel4{{0, 0, 0, 0}}) {}
  Index2 size() const { return Index2{{w, h}}; }
  struct Map {
    Pixel4* p;
    Pixel4* data() const { return p; }
  };
  Map data() { return Map{px.data()}; }
};

// hash + pcg32_fast + uniform<T> (include/vpt/hash.hpp:20-67, random.hpp:86-115); no seed accessor.
class RandomNumberGenerator {
 public:
  explicit RandomNumberGenerator(uint32_t seed) : m_seed(seed) {}
  void begin_job(size_t jid) {
    const uint64_t m = 0xc6a4a7935bd1e995ULL;
    uint64_t h = (uint64_t)m_seed ^ (8ULL * m), k = (uint64_t)jid * m;
    k ^= k >> 47;
    k *= m;
    h ^= k;
    h *= m;
    h ^= h >> 47;
    h *= m;
    h ^= h >> 47;
    m_state = h | 3ULL;
  }
  template <typename T>
  T uniform() {
    const uint64_t old = m_state;
    m_state = old * 6364136223846793005ULL;
    const uint32_t u = (uint32_t)((old ^ (old >> 22)) >> (22 + (uint32_t)(old >> 61)));
    if constexpr (std::is_same_v<T, uint32_t>) {
      return u;
    } else {
      const float v = (float)u * 0x1p-32f;
      return v < 0x1.fffffep-1f ? v : 0x1.fffffep-1f;
    }
  }

 private:
  uint64_t m_state = 0;
  uint32_t m_seed;
};

}  // namespace vpt_headless
