// vpt_oracle.cpp — CPU restatement of Shibodd/volume_path_tracer's hot path.
//
// TEST INFRASTRUCTURE ONLY (the parity oracle and the timed CPU baseline).  Nothing in the
// product (volume_path_tracer_amd/) links or calls this file.  Each block restates one reference
// function; the citation is /root/reference/<file>:<line>.
//
// Float discipline: built with -O3 -ffp-contract=off and no fast-math, like the reference's
// Release build (CMakeLists.txt:26-44 sets no -march, so x86-64 baseline: no FMA contraction).
// Transcendentals are glibc's, as in the reference (std::log/std::sin/std::cos on float).
// Eigen's fixed-size reductions are restated as x0 + (x1 + x2) (Eigen redux_novec_unroller);
// NanoVDB Vec3::lengthSqr as (x*x + y*y) + z*z; NanoVDB Map products with explicit fmaf.
// NanoVDB/Eigen are not in /root/reference (empty submodule / system dep): parity unpinned there.

#include "vpt_oracle.h"

// Mutation builds (test infrastructure for the scattering anchor, tests/test_analytic_scatter.py,
// which must reject each; `make mutants` builds build/libvpt_oracle_mut<N>.so):
//   1  NEE phase with pbrt's sign (den = 1 + g^2 - 2g w.wi instead of utils.hpp:62's + with the forward w)
//   2  HG sampling about -w (pbrt's minus sign restored, random.hpp:64)
//   3  one depth increment per scatter (worker.cpp:169's depth++ dropped)
//   4  environment light only on escape (not on the depth-bound exit, worker.cpp:130,198-200)
#ifndef VPTO_MUTANT
#define VPTO_MUTANT 0
#endif

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

namespace {

// ------------------------------------------------------------------------------------------
// RNG: include/vpt/hash.hpp:20-67, include/vpt/random.hpp:86-115,
//      external/pcg-cpp/include/pcg/pcg_random.hpp (pcg32_fast = mcg_xsh_rs_64_32, :1535,1673)
// ------------------------------------------------------------------------------------------

// hash(seed, jid): key = one 8-byte word (jid), MurmurHash64A over 8 bytes (hash.hpp:20-51,55-67).
uint64_t murmur64a_one_word(uint64_t seed, uint64_t k) {
  const uint64_t m = 0xc6a4a7935bd1e995ULL;
  const int r = 47;
  uint64_t h = seed ^ (8ULL * m);
  k *= m;
  k ^= k >> r;
  k *= m;
  h ^= k;
  h *= m;
  h ^= h >> r;
  h *= m;
  h ^= h >> r;
  return h;
}

struct Rng {
  uint64_t state = 0;
  // RandomNumberGenerator::begin_job (random.hpp:93-95) -> pcg32_fast::seed(h): state = h | 3.
  void begin_job(uint32_t seed, uint64_t jid) { state = murmur64a_one_word(seed, jid) | 3ULL; }
  // pcg32_fast operator(): output_previous, xsh_rs 64->32 (pcg_random.hpp:389-400,459,762-786).
  uint32_t next_u32() {
    uint64_t old = state;
    state = state * 6364136223846793005ULL;
    uint32_t rshift = (uint32_t)(old >> 61);
    old ^= old >> 22;
    return (uint32_t)(old >> (22 + rshift));
  }
  // uniform<float>() (random.hpp:107-111).
  float uniform() {
    const float one_minus_eps = 0x1.fffffep-1f;
    float v = (float)next_u32() * 0x1p-32f;
    return std::min<float>(one_minus_eps, v);
  }
};

// ------------------------------------------------------------------------------------------
// Small vector helpers with Eigen / NanoVDB operation order.
// ------------------------------------------------------------------------------------------
struct V3 {
  float x, y, z;
};
inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
inline V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 mul(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
inline V3 smul(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
// Eigen squaredNorm / dot for size 3: redux_novec_unroller -> x0 + (x1 + x2).
inline float eigen_dot(V3 a, V3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
inline float eigen_sqnorm(V3 a) { return a.x * a.x + (a.y * a.y + a.z * a.z); }
// Eigen normalized(): n / sqrt(squaredNorm()) if > 0.
inline V3 eigen_normalized(V3 a) {
  float z = eigen_sqnorm(a);
  if (z > 0.0f) {
    float s = std::sqrt(z);
    return v3(a.x / s, a.y / s, a.z / s);
  }
  return a;
}
inline V3 eigen_cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// NanoVDB Vec3::length(): Sqrt(x*x + y*y + z*z) evaluated left to right.
inline float nvdb_length(V3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }

// NanoVDB math::matMult(mat, xyz) = fmaf(x0,m0, fmaf(x1,m1, x2*m2)) per row;
// matMult(mat, vec, xyz) = fmaf(x0,m0, fmaf(x1,m1, fmaf(x2,m2, v0))).
inline V3 mat_mult(const float* m, V3 p) {
  return v3(std::fmaf(p.x, m[0], std::fmaf(p.y, m[1], p.z * m[2])),
            std::fmaf(p.x, m[3], std::fmaf(p.y, m[4], p.z * m[5])),
            std::fmaf(p.x, m[6], std::fmaf(p.y, m[7], p.z * m[8])));
}
inline V3 mat_mult_vec(const float* m, const float* v, V3 p) {
  return v3(std::fmaf(p.x, m[0], std::fmaf(p.y, m[1], std::fmaf(p.z, m[2], v[0]))),
            std::fmaf(p.x, m[3], std::fmaf(p.y, m[4], std::fmaf(p.z, m[5], v[1]))),
            std::fmaf(p.x, m[6], std::fmaf(p.y, m[7], std::fmaf(p.z, m[8], v[2]))));
}

inline int32_t nvdb_floor(float x) { return (int32_t)std::floor(x); }

// ------------------------------------------------------------------------------------------
// NanoVDB NanoGrid<float> semantics (third-party; restated): tree + ReadAccessor queries
// used at volume.cpp:13,21,29,152 and by SampleFromVoxels.
// ------------------------------------------------------------------------------------------
struct Leaf {
  int32_t origin[3];
  float v[512];
  uint64_t mask[8];
  float max;
};
struct Lower {  // InternalNode<Leaf, 4>: 16^3 slots of 8^3
  int32_t origin[3];
  std::vector<int32_t> child;  // 4096, leaf index or -1
  std::vector<float> tile;
  std::vector<uint8_t> active;
  float max = 0.0f;  // build statistic (NodeInfo::maximum), see Grid::update_stats
  bool max_any = false;
};
struct Upper {  // InternalNode<Lower, 5>: 32^3 slots of 128^3
  int32_t origin[3];
  std::vector<int32_t> child;  // 32768, lower index or -1
  std::vector<float> tile;
  std::vector<uint8_t> active;
  float max = 0.0f;
  bool max_any = false;
};
struct RootTile {
  int32_t upper = -1;  // child upper index, or -1 for a value tile
  float value = 0.0f;
  bool active = false;
};

inline uint32_t leaf_offset(int32_t i, int32_t j, int32_t k) {
  return ((uint32_t)(i & 7) << 6) | ((uint32_t)(j & 7) << 3) | (uint32_t)(k & 7);
}
inline uint32_t lower_offset(int32_t i, int32_t j, int32_t k) {
  return ((uint32_t)((i & 127) >> 3) << 8) | ((uint32_t)((j & 127) >> 3) << 4) | (uint32_t)((k & 127) >> 3);
}
inline uint32_t upper_offset(int32_t i, int32_t j, int32_t k) {
  return ((uint32_t)((i & 4095) >> 7) << 10) | ((uint32_t)((j & 4095) >> 7) << 5) | (uint32_t)((k & 4095) >> 7);
}
using Key = std::tuple<int32_t, int32_t, int32_t>;
inline Key root_key(int32_t i, int32_t j, int32_t k) { return Key(i & ~4095, j & ~4095, k & ~4095); }

struct Grid {
  float mat[9], inv_mat[9], vec[3];
  float background;
  int32_t bbox_min[3], bbox_max[3];
  std::vector<Leaf> leaves;
  std::vector<Lower> lowers;
  std::vector<Upper> uppers;
  std::map<Key, RootTile> root;
  float root_max = 0.0f;

  // NanoVDB's build statistics of the internal nodes and the root (tools/GridStats.h, restated):
  // maximum over the children's maxima and the active tile values; 0 when a node has none.  Taken
  // from the stored leaf maxima, i.e. before fix_majorants_for_interpolation rewrites them.
  void update_stats() {
    auto acc = [](float& m, bool& any, float x) {
      m = any ? std::max(m, x) : x;
      any = true;
    };
    for (Lower& l : lowers) {
      bool any = false;
      float m = 0.0f;
      for (int n = 0; n < 4096; ++n) {
        if (l.child[n] >= 0) acc(m, any, leaves[l.child[n]].max);
        else if (l.active[n]) acc(m, any, l.tile[n]);
      }
      l.max = m;
      l.max_any = any;
    }
    for (Upper& u : uppers) {
      bool any = false;
      float m = 0.0f;
      for (int n = 0; n < 32768; ++n) {
        if (u.child[n] >= 0) {
          if (lowers[u.child[n]].max_any) acc(m, any, lowers[u.child[n]].max);
        } else if (u.active[n]) {
          acc(m, any, u.tile[n]);
        }
      }
      u.max = m;
      u.max_any = any;
    }
    bool any = false;
    float m = 0.0f;
    for (const auto& kv : root) {
      if (kv.second.upper >= 0) {
        if (uppers[kv.second.upper].max_any) acc(m, any, uppers[kv.second.upper].max);
      } else if (kv.second.active) {
        acc(m, any, kv.second.value);
      }
    }
    root_max = m;
  }

  // ReadAccessor::getNodeInfo(ijk): dim and maximum of the deepest node holding ijk.
  void node_info(int32_t i, int32_t j, int32_t k, uint32_t& dim, float& maximum) const {
    auto it = root.find(root_key(i, j, k));
    if (it == root.end() || it->second.upper < 0) {
      dim = 4096u;  // RootNode: NodeInfo{LEVEL, ChildT::dim(), ...}
      maximum = root_max;
      return;
    }
    const Upper& up = uppers[it->second.upper];
    const int32_t lo_idx = up.child[upper_offset(i, j, k)];
    if (lo_idx < 0) {
      dim = 4096u;
      maximum = up.max;
      return;
    }
    const Lower& lo = lowers[lo_idx];
    const int32_t lf_idx = lo.child[lower_offset(i, j, k)];
    if (lf_idx < 0) {
      dim = 128u;
      maximum = lo.max;
      return;
    }
    dim = 8u;
    maximum = leaves[lf_idx].max;  // after fix_majorants_for_interpolation (it writes the grid)
  }

  // Node walk. level_out: 0 leaf, 1 lower-tile, 2 upper-tile, 3 root tile/background.
  struct Hit {
    const Leaf* leaf;
    float value;
    bool active;
    uint32_t dim;  // ReadAccessor::getDim
  };
  Hit query(int32_t i, int32_t j, int32_t k) const {
    auto it = root.find(root_key(i, j, k));
    if (it == root.end()) return Hit{nullptr, background, false, 4096u};  // ChildNodeType::dim()
    const RootTile& rt = it->second;
    if (rt.upper < 0) return Hit{nullptr, rt.value, rt.active, 4096u};   // 1 << ChildT::TOTAL
    const Upper& up = uppers[rt.upper];
    uint32_t nu = upper_offset(i, j, k);
    int32_t lo_idx = up.child[nu];
    if (lo_idx < 0) return Hit{nullptr, up.tile[nu], up.active[nu] != 0, 128u};
    const Lower& lo = lowers[lo_idx];
    uint32_t nl = lower_offset(i, j, k);
    int32_t lf_idx = lo.child[nl];
    if (lf_idx < 0) return Hit{nullptr, lo.tile[nl], lo.active[nl] != 0, 8u};
    const Leaf& lf = leaves[lf_idx];
    uint32_t n = leaf_offset(i, j, k);
    return Hit{&lf, lf.v[n], ((lf.mask[n >> 6] >> (n & 63)) & 1ULL) != 0, 1u};
  }
  float getValue(int32_t i, int32_t j, int32_t k) const { return query(i, j, k).value; }
  const Leaf* probeLeaf(int32_t i, int32_t j, int32_t k) const { return query(i, j, k).leaf; }
  bool probeValue(int32_t i, int32_t j, int32_t k, float& v) const {
    Hit h = query(i, j, k);
    v = h.value;
    return h.active;
  }
  uint32_t getDim(int32_t i, int32_t j, int32_t k) const { return query(i, j, k).dim; }

  V3 worldToIndexF(V3 w) const { return mat_mult(inv_mat, v3(w.x - vec[0], w.y - vec[1], w.z - vec[2])); }
  V3 worldToIndexDirF(V3 d) const { return mat_mult(inv_mat, d); }
  V3 indexToWorldF(V3 p) const { return mat_mult_vec(mat, vec, p); }
};

// A tiny ReadAccessor-style cache (leaf / lower / upper by aligned origin) so that the CPU
// baseline pays NanoVDB-like query costs.  Values returned are identical to Grid::query.
struct Accessor {
  const Grid* g;
  int32_t leaf_key[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
  const Leaf* leaf = nullptr;
  explicit Accessor(const Grid* grid) : g(grid) {}
  float getValue(int32_t i, int32_t j, int32_t k) {
    int32_t ki = i & ~7, kj = j & ~7, kk = k & ~7;
    if (leaf && ki == leaf_key[0] && kj == leaf_key[1] && kk == leaf_key[2]) return leaf->v[leaf_offset(i, j, k)];
    Grid::Hit h = g->query(i, j, k);
    if (h.leaf) {
      leaf = h.leaf;
      leaf_key[0] = ki;
      leaf_key[1] = kj;
      leaf_key[2] = kk;
    }
    return h.value;
  }
};

// NanoVDB math::SampleFromVoxels<Acc, 1, true> (trilinear with stencil cache).
struct Trilinear {
  Accessor acc;
  int32_t pos[3] = {0, 0, 0};
  bool valid = false;  // reference: mPos starts at (0,0,0) with mVal unset (UB); we always fetch first
  float val[2][2][2];
  uint64_t* refresh_counter = nullptr;
  explicit Trilinear(const Grid* g) : acc(g) {}
  float operator()(V3 xyz) {
    // Floor(xyz) modifies xyz into the fractional part and returns the cell.
    float fi = std::floor(xyz.x), fj = std::floor(xyz.y), fk = std::floor(xyz.z);
    xyz.x -= fi;
    xyz.y -= fj;
    xyz.z -= fk;
    int32_t i = (int32_t)fi, j = (int32_t)fj, k = (int32_t)fk;
    if (!valid || i != pos[0] || j != pos[1] || k != pos[2]) {
      valid = true;
      pos[0] = i;
      pos[1] = j;
      pos[2] = k;
      if (refresh_counter) ++*refresh_counter;
      for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b)
          for (int c = 0; c < 2; ++c) val[a][b][c] = acc.getValue(i + a, j + b, k + c);
    }
    auto lerp = [](float a, float b, float w) { return a + w * (b - a); };
    return lerp(lerp(lerp(val[0][0][0], val[0][0][1], xyz.z), lerp(val[0][1][0], val[0][1][1], xyz.z), xyz.y),
                lerp(lerp(val[1][0][0], val[1][0][1], xyz.z), lerp(val[1][1][0], val[1][1][1], xyz.z), xyz.y),
                xyz.x);
  }
};

// NanoVDB math::Ray<float> (restated): eye, dir, invDir = 1/dir, timespan [t0, t1].
struct NRay {
  V3 eye, dir, inv;
  float t0, t1;
  NRay(V3 e, V3 d, float a = 1e-5f, float b = std::numeric_limits<float>::max())
      : eye(e), dir(d), inv(v3(1 / d.x, 1 / d.y, 1 / d.z)), t0(a), t1(b) {}
  V3 at(float t) const { return v3(eye.x + dir.x * t, eye.y + dir.y * t, eye.z + dir.z * t); }
  // Ray::worldToIndexF(grid)
  NRay worldToIndexF(const Grid& g) const {
    V3 e = g.worldToIndexF(eye);
    V3 d = g.worldToIndexDirF(dir);
    float len = nvdb_length(d), inv_len = 1.0f / len;
    float nt1 = t1;
    if (nt1 < std::numeric_limits<float>::max()) nt1 *= len;
    return NRay(e, mul(d, inv_len), len * t0, nt1);
  }
  // Ray::clip(CoordBBox): slab test against [min, max+1].
  bool clip(const int32_t* bmin, const int32_t* bmax) {
    float a0 = t0, a1 = t1;
    const float* e = &eye.x;
    const float* iv = &inv.x;
    for (int i = 0; i < 3; ++i) {
      float a = (float)bmin[i], b = (float)(bmax[i] + 1);
      a = (a - e[i]) * iv[i];
      b = (b - e[i]) * iv[i];
      if (a > b) std::swap(a, b);
      if (a > a0) a0 = a;
      if (b < a1) a1 = b;
      if (a0 > a1) return false;
    }
    t0 = a0;
    t1 = a1;
    return true;
  }
};

// NanoVDB math::HDDA<Ray<float>, Coord> (restated).
struct HDDA {
  int32_t dim;
  float T0, T1;
  float next[3], delta[3];
  int32_t voxel[3], step[3];
  void init(const NRay& ray, int32_t d) {
    dim = d;
    T0 = ray.t0;
    T1 = ray.t1;
    V3 pos = ray.at(T0);
    const float p[3] = {pos.x, pos.y, pos.z};
    const float dr[3] = {ray.dir.x, ray.dir.y, ray.dir.z};
    const float iv[3] = {ray.inv.x, ray.inv.y, ray.inv.z};
    for (int a = 0; a < 3; ++a) voxel[a] = nvdb_floor(p[a]) & (~(d - 1));
    for (int a = 0; a < 3; ++a) {
      if (dr[a] == 0.0f) {
        next[a] = std::numeric_limits<float>::max();
        step[a] = 0;
      } else if (iv[a] > 0) {
        step[a] = 1;
        next[a] = T0 + ((float)(voxel[a] + d) - p[a]) * iv[a];
        delta[a] = iv[a];
      } else {
        step[a] = -1;
        next[a] = T0 + ((float)voxel[a] - p[a]) * iv[a];
        delta[a] = -iv[a];
      }
    }
  }
  bool update(const NRay& ray, int32_t d) {
    if (dim == d) return false;
    dim = d;
    V3 pos = ray.at(T0);
    const float p[3] = {pos.x, pos.y, pos.z};
    const float iv[3] = {ray.inv.x, ray.inv.y, ray.inv.z};
    for (int a = 0; a < 3; ++a) voxel[a] = nvdb_floor(p[a]) & (~(d - 1));
    for (int a = 0; a < 3; ++a) {
      if (step[a] == 0) continue;
      next[a] = T0 + ((float)voxel[a] - p[a]) * iv[a];
      if (step[a] > 0) next[a] += (float)d * iv[a];
    }
    return true;
  }
  bool step_() {
    int a = (next[0] < next[1] && next[0] < next[2]) ? 0 : (next[1] < next[2] ? 1 : 2);  // MinIndex
    T0 = next[a];
    next[a] += (float)dim * delta[a];
    voxel[a] += dim * step[a];
    return T0 <= T1;
  }
};

// ------------------------------------------------------------------------------------------
// RayMajorantIterator: src/volume.cpp:11-98, include/vpt/volume.hpp:24-76
// ------------------------------------------------------------------------------------------
struct Segment {
  float t0, t1, d_maj;
};

struct RayMajorantIterator {
  const Grid* g;
  NRay ray;
  float scale;
  float majorant;
  HDDA dda;
  uint64_t* step_counter = nullptr;

  static uint32_t hdda_dim(const Grid& g, int32_t i, int32_t j, int32_t k) {  // volume.cpp:11-14
    return std::max<uint32_t>(8, g.getDim(i, j, k));
  }
  RayMajorantIterator(const NRay& r, const Grid* grid)  // volume.cpp:90-98
      : g(grid), ray(r) {
    scale = 1 / nvdb_length(grid->worldToIndexDirF(r.dir));
    majorant = std::numeric_limits<float>::quiet_NaN();
    V3 s = ray.at(ray.t0);
    dda.init(ray, (int32_t)hdda_dim(*grid, nvdb_floor(s.x), nvdb_floor(s.y), nvdb_floor(s.z)));
  }
  void update_current_majorant() {  // volume.cpp:18-36
    const int32_t* ijk = dda.voxel;
    Grid::Hit h = g->query(ijk[0], ijk[1], ijk[2]);
    if (h.leaf) {
      majorant = h.leaf->max;
      return;
    }
    if (h.active) {
      majorant = h.value;
      return;
    }
    majorant = 0.0f;
  }
  bool next(Segment& ans) {  // volume.cpp:38-76
    if (dda.T0 >= dda.T1) return false;
    ans.t0 = dda.T0;
    if (std::isnan(majorant)) update_current_majorant();
    do {
      ans.d_maj = majorant;
      if (step_counter) ++*step_counter;
      if (!dda.step_()) {
        ans.t1 = dda.T1;
        return true;
      }
      V3 la = ray.at(dda.T0 + 1.0001f);
      uint32_t nd = hdda_dim(*g, nvdb_floor(la.x), nvdb_floor(la.y), nvdb_floor(la.z));
      dda.update(ray, (int32_t)nd);
      update_current_majorant();
    } while (majorant == ans.d_maj);
    ans.t1 = dda.T0;
    return true;
  }
};

// Volume::intersect (volume.cpp:78-88).
bool volume_intersect(const Grid& g, V3 origin, V3 direction, NRay& out_index_ray) {
  NRay w(origin, direction);
  NRay i = w.worldToIndexF(g);
  if (!i.clip(g.bbox_min, g.bbox_max)) return false;
  out_index_ray = i;
  return true;
}

// ------------------------------------------------------------------------------------------
// MajorantTransmittanceSampler: src/majorant_transmittance_sampler.cpp:7-81
// ------------------------------------------------------------------------------------------
struct MediumProperties {
  V3 point;  // world
  float sigma_maj;
  float density;
};

struct MajorantTransmittanceSampler {
  float sigma_t;
  Rng& rng;
  RayMajorantIterator it;
  const Grid* g;
  Trilinear density;
  bool has_seg = false;
  Segment seg{};
  vpt_counters* cnt;

  MajorantTransmittanceSampler(const RayMajorantIterator& iter, Rng& r, const Grid* grid, float st,
                               vpt_counters* c)
      : sigma_t(st), rng(r), it(iter), g(grid), density(grid), cnt(c) {
    if (cnt) {
      it.step_counter = &cnt->dda_steps;
      density.refresh_counter = &cnt->stencils;
    }
  }
  // m_T_maj (:51,:73) is never read (T_maj() has no callers): omitted.
  bool next(MediumProperties& out) {
    while (true) {
      if (!has_seg) {
        if (!it.next(seg)) return false;
        if (cnt) ++cnt->segments;
        if (seg.d_maj <= 0) continue;  // :32-35, no draw
        has_seg = true;
      }
      float sigma_maj = seg.d_maj * sigma_t;
      float u = rng.uniform();
      if (cnt) {
        ++cnt->draws;
        ++cnt->rng_draws;
      }
      float dt_m = -std::log(1 - u) / sigma_maj;  // sample_exponential, random.hpp:20-22
      float t = seg.t0 + dt_m / it.scale;
      if (t < seg.t1) {
        seg.t0 = t;
        V3 p_index = it.ray.at(t);
        V3 p_world = g->indexToWorldF(p_index);
        if (cnt) ++cnt->density_evals;
        float d = density(p_index);
        if (d <= 0.0f) continue;
        out.point = p_world;
        out.sigma_maj = sigma_maj;
        out.density = d;
        return true;
      } else {
        has_seg = false;
      }
    }
  }
};

// ------------------------------------------------------------------------------------------
// Sampling helpers: include/vpt/random.hpp:20-84, include/vpt/utils.hpp:39-66
// ------------------------------------------------------------------------------------------
void coordinate_system(V3 v1, V3& v2, V3& v3o) {  // utils.hpp:39-51
  float sign = std::copysign(1.0f, v1.z);
  float a = -1.0f / (sign + v1.z);
  float b = v1.x * v1.y * a;
  v2.x = 1.0f + sign * a * std::pow(v1.x, 2.0f);
  v2.y = sign * b;
  v2.z = -sign * v1.x;
  v3o.x = b;
  v3o.y = sign + a * std::pow(v1.y, 2.0f);
  v3o.z = -v1.y;
}

V3 sample_henyey_greenstein(V3 w, float u0, float u1, float g) {  // random.hpp:56-84
  float g2 = std::pow(g, 2.0f);
  float cos_theta;
  if (std::abs(g) < 1e-3f)
    cos_theta = 1 - 2 * u0;
  else
    cos_theta = 1.0f / (2.0f * g) * (1.0f + g2 - std::pow((1.0f - g2) / (1.0f + g - 2.0f * g * u0), 2.0f));
  if (VPTO_MUTANT == 2) cos_theta = -cos_theta;
  float sin_theta = std::sqrt(std::max(0.0f, 1.0f - std::pow(cos_theta, 2.0f)));
  float phi = 2.0f * 3.14159274f * u1;  // 2.0f * float(pi) * u
  float sc = std::clamp(sin_theta, -1.0f, 1.0f);
  V3 local = v3(sc * std::cos(phi), sc * std::sin(phi), std::clamp(cos_theta, -1.0f, 1.0f));
  local = eigen_normalized(local);  // local.normalize()
  V3 x, y;
  coordinate_system(w, x, y);
  // local.x() * x + local.y() * y + local.z() * z
  return v3((local.x * x.x + local.y * y.x) + local.z * w.x, (local.x * x.y + local.y * y.y) + local.z * w.y,
            (local.x * x.z + local.y * y.z) + local.z * w.z);
}

float henyey_greenstein(float cos_theta, float g) {  // utils.hpp:61-66
  float den = 1.0f + g * g + 2.0f * g * cos_theta;
  const float inv_4_pi = (float)(0.318309886183790671537767526745028724 / 4.0);
  return inv_4_pi * (1.0f - g * g) / (den * std::sqrt(std::max(0.0f, den)));
}

enum class ScatterEvent { Null, Absorption, Scatter };

ScatterEvent sample_discrete3(float w0, float w1, float w2, float u) {  // random.hpp:30-47
  float total = ((0.0f + w0) + w1) + w2;
  u = u * total;
  u -= w0;
  if (u <= 0) return ScatterEvent::Null;
  u -= w1;
  if (u <= 0) return ScatterEvent::Absorption;
  u -= w2;
  if (u <= 0) return ScatterEvent::Scatter;
  return ScatterEvent::Scatter;
}

// ------------------------------------------------------------------------------------------
// Blackbody: src/spectral.cpp:7-20, include/vpt/spectral.hpp:62-75, src/precompute_blackbody.cpp
// ------------------------------------------------------------------------------------------
float planck_law(float lambda_m, float temperature_k) {
  if (temperature_k <= 0.0f) return 0.0f;
  const float c = 299792458.f;
  const float h = 6.62606957e-34f;
  const float kb = 1.3806488e-23f;
  const float num = 2 * h * c * c;
  float lambda5 = (float)std::pow((double)lambda_m, 5.0);  // std::pow(float, int) -> double
  float e = std::exp((h * c) / (lambda_m * kb * temperature_k));
  float den = lambda5 * (e - 1);
  return num / den;
}

V3 spectrum_to_xyz(const float* cie, float y_integral, float temperature) {
  float acc[3] = {0.0f, 0.0f, 0.0f};
  for (int c = 0; c < 3; ++c) {
    float integral = 0.0f;
    for (int i = 0; i < 471; ++i)
      integral += cie[i * 3 + c] * planck_law(static_cast<float>(360 + i) * 1e-9f, temperature);
    acc[c] = integral;
  }
  return v3(acc[0] / y_integral, acc[1] / y_integral, acc[2] / y_integral);
}

inline float idx_to_temp(int idx) { return (idx - 1) * 100.0f; }

V3 blackbody_radiation_xyz(const float* table, const float* cie, float y_integral, float t) {
  if (!std::isfinite(t)) {
    float n = std::numeric_limits<float>::quiet_NaN();
    return v3(n, n, n);
  }
  if (t <= 0.0f) return v3(0, 0, 0);
  const float TEMP_MAX = (500 - 1) * 100.0f;
  if (t >= TEMP_MAX) return spectrum_to_xyz(cie, y_integral, t);
  int dn = static_cast<int>(t / 100.0f);
  while (t <= idx_to_temp(dn - 1)) --dn;
  while (t >= idx_to_temp(dn + 1)) ++dn;
  float dn_temp = idx_to_temp(dn);
  // Row 500 does not exist in the reference (out-of-bounds read for T in [49800, 49900)); the
  // table handed to the oracle carries a zero row there.
  const float* a = table + dn * 3;
  if (t == dn_temp) return v3(a[0], a[1], a[2]);
  float w = (t - idx_to_temp(dn)) / 100.0f;
  const float* b = a + 3;
  return v3(a[0] + (b[0] - a[0]) * w, a[1] + (b[1] - a[1]) * w, a[2] + (b[2] - a[2]) * w);
}

// ------------------------------------------------------------------------------------------
// Camera: src/camera.cpp:5-57, include/vpt/camera.hpp:14-23 (Eigen Affine3f products restated)
// ------------------------------------------------------------------------------------------
struct CameraM {
  float L[9];  // raster_to_world_dir.linear(), row-major
  float t[3];  // raster_to_world_dir.translation()
  V3 position;
};

CameraM make_camera(const vpt_configuration& cfg) {
  const vpt_camera_params& p = cfg.camera_parameters;
  const float W = (float)cfg.output_size[0], H = (float)cfg.output_size[1];
  float ar = W / H;
  float vfov_rad = 3.14159274f * p.vfov_deg / 180.0f;  // float(pi) * vfov / 180
  V3 pos = v3(p.position[0], p.position[1], p.position[2]);
  V3 look = v3(p.look[0], p.look[1], p.look[2]);
  V3 up = v3(p.up[0], p.up[1], p.up[2]);
  // camera_to_world (camera.cpp:5-19): columns left, new_up, dir.
  V3 dir = eigen_normalized(sub(look, pos));
  V3 left = eigen_cross(eigen_normalized(up), dir);
  V3 new_up = eigen_cross(dir, left);
  float C[9] = {left.x, new_up.x, dir.x, left.y, new_up.y, dir.y, left.z, new_up.z, dir.z};
  // screen_to_camera (camera.cpp:34-43): diag(ar*tan, tan, 0), translation (0,0,1).
  float tv = std::tan(vfov_rad / 2);
  float S[9] = {ar * tv, 0, 0, 0, tv, 0, 0, 0, 0};
  float St[3] = {0.0f, 0.0f, 1.0f};
  // raster_to_screen (camera.cpp:21-32): diag(-(1/(W/2)), -(1/(H/2)), 0), translation (1,1,0).
  float hx = W / 2.0f, hy = H / 2.0f;
  float R[9] = {-(1.0f / hx), 0, 0, 0, -(1.0f / hy), 0, 0, 0, 0};
  float Rt[3] = {1.0f, 1.0f, 0.0f};
  // Eigen lazy product coefficient: a_i0*b_0j + (a_i1*b_1j + a_i2*b_2j).
  auto prod = [](const float* A, const float* B, float* O) {
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        O[i * 3 + j] = A[i * 3 + 0] * B[0 * 3 + j] + (A[i * 3 + 1] * B[1 * 3 + j] + A[i * 3 + 2] * B[2 * 3 + j]);
  };
  auto prodv = [](const float* A, const float* v, float* o) {
    for (int i = 0; i < 3; ++i) o[i] = A[i * 3 + 0] * v[0] + (A[i * 3 + 1] * v[1] + A[i * 3 + 2] * v[2]);
  };
  // screen_to_world_dir = c2w.linear() * s2c: linear C*S, translation C*St (camera.cpp:55).
  float SWl[9], SWt[3];
  prod(C, S, SWl);
  prodv(C, St, SWt);
  // raster_to_world_dir = s2w * r2s (Affine*Affine): linear SWl*R, translation SWl*Rt + SWt.
  CameraM cam;
  prod(SWl, R, cam.L);
  float tmp[3];
  prodv(SWl, Rt, tmp);
  for (int i = 0; i < 3; ++i) cam.t[i] = tmp[i] + SWt[i];
  cam.position = pos;
  return cam;
}

// Camera::generate_ray (camera.hpp:14-23): dir = normalized(M * (x+0.5+jx, y+0.5+jy, 0)).
V3 camera_dir(const CameraM& cam, int64_t x, int64_t y, float jx, float jy) {
  float rx = ((float)x + 0.5f) + jx;
  float ry = ((float)y + 0.5f) + jy;
  float v[3] = {rx, ry, 0.0f};
  float d[3];
  for (int i = 0; i < 3; ++i)
    d[i] = cam.t[i] + (cam.L[i * 3 + 0] * v[0] + (cam.L[i * 3 + 1] * v[1] + cam.L[i * 3 + 2] * v[2]));
  return eigen_normalized(v3(d[0], d[1], d[2]));
}

// ------------------------------------------------------------------------------------------
// The worker: src/worker.cpp:52-208
// ------------------------------------------------------------------------------------------
struct Scene {
  const vpt_configuration* cfg;
  const Grid* density;
  const Grid* temperature;
  const float* bb;
  const float* cie;
  float y_integral;
  CameraM cam;
  uint64_t ntx, nty, T;
};

V3 sample_Ld(const Scene& S, Rng& rng, V3 pos, V3 w, vpt_counters* cnt) {  // worker.cpp:52-90
  const vpt_worker_params& P = S.cfg->worker_parameters;
  const vpt_volume_params& VP = S.cfg->volume_parameters;
  V3 wi = eigen_normalized(v3(P.distant_light_inv_direction[0], P.distant_light_inv_direction[1],
                              P.distant_light_inv_direction[2]));
  V3 Li = v3(P.distant_light_xyz[0] * P.distant_light_multiplier, P.distant_light_xyz[1] * P.distant_light_multiplier,
             P.distant_light_xyz[2] * P.distant_light_multiplier);
  if (Li.x == 0.0f && Li.y == 0.0f && Li.z == 0.0f) return Li;
  float sigma_t = VP.sigma_a + VP.sigma_s;
  float T_ray = 1.0f;
  NRay ir(v3(0, 0, 0), v3(1, 0, 0));
  if (volume_intersect(*S.density, pos, wi, ir)) {
    if (cnt) ++cnt->shadow_rays;
    RayMajorantIterator it(ir, S.density);
    MajorantTransmittanceSampler sampler(it, rng, S.density, sigma_t, cnt);
    MediumProperties props;
    while (sampler.next(props)) {
      float sigma_n = std::max(0.0f, props.sigma_maj - sigma_t * props.density);
      T_ray *= sigma_n / props.sigma_maj;
      if (T_ray <= 0.05f) {
        float q = 0.75f;
        if (cnt) ++cnt->rng_draws;
        if (rng.uniform() < q)
          T_ray = 0.0f;
        else
          T_ray /= 1 - q;
      }
      if (T_ray <= 0.0f) return v3(0, 0, 0);
    }
  }
  float p = henyey_greenstein(VPTO_MUTANT == 1 ? -eigen_dot(w, wi) : eigen_dot(w, wi), VP.henyey_greenstein_g);
  return v3(p * T_ray * Li.x, p * T_ray * Li.y, p * T_ray * Li.z);
}

// One (tile, wave) job: the body of `while (auto tok = tp.next())` (worker.cpp:104-207).
// Logger<true> (worker.cpp:16-48) as records instead of log.csv lines.
struct EventSink {
  vpt_event* out;
  uint64_t cap;
  uint64_t n = 0;
  uint32_t seq = 0;
  void log(uint64_t jid, uint32_t pixel, uint32_t type, const V3* a, const V3* b, float x) {
    const uint32_t sq = seq++;
    if (n < cap) {
      vpt_event& e = out[n];
      e.jid = jid;
      e.pixel = pixel;
      e.seq = sq;
      e.type = type;
      const float av[3] = {a ? a->x : 0.0f, a ? a->y : 0.0f, a ? a->z : 0.0f};
      const float bv[3] = {b ? b->x : x, b ? b->y : 0.0f, b ? b->z : 0.0f};
      for (int i = 0; i < 3; ++i) {
        e.v[i] = av[i];
        e.v[3 + i] = bv[i];
      }
      e.v[6] = 0.0f;
    }
    ++n;
  }
};

void run_job(const Scene& S, uint64_t jid, float* film, float* records, uint64_t record_base,
             vpt_counters* cnt, EventSink* log = nullptr, bool pixel_mode = false) {
  if (log) log->seq = 0;
  const vpt_configuration& cfg = *S.cfg;
  const vpt_worker_params& P = cfg.worker_parameters;
  const vpt_volume_params& VP = cfg.volume_parameters;
  const int64_t W = cfg.output_size[0], H = cfg.output_size[1];
  const int64_t tw = cfg.tile_size[0], th = cfg.tile_size[1];
  uint64_t tile = jid % S.T;
  // TileProvider::compute_tile_rect (tile_provider.cpp:95-105)
  int64_t x0 = (int64_t)(tile % S.ntx) * tw, y0 = (int64_t)(tile / S.ntx) * th;
  int64_t rw = std::min(W - x0, tw), rh = std::min(H - y0, th);

  Rng rng;
  rng.begin_job(cfg.seed, jid);
  const float sigma_t = VP.sigma_a + VP.sigma_s;
  std::unique_ptr<Trilinear> temp_sampler;
  if (S.temperature) temp_sampler.reset(new Trilinear(S.temperature));
  if (temp_sampler && cnt) temp_sampler->refresh_counter = &cnt->temp_stencils;

  for (int64_t y = 0; y < rh; ++y) {
    for (int64_t x = 0; x < rw; ++x) {
      int64_t px = x0 + x, py = y0 + y;
      if (P.single_pixel_enabled) {
        if (P.single_pixel_coord[0] != px || P.single_pixel_coord[1] != py) continue;
      }
      // throughput mode (not the reference): one stream per pixel, hash(seed, jid * area + pixel)
      if (pixel_mode) rng.begin_job(cfg.seed, jid * (uint64_t)(tw * th) + (uint64_t)(y * rw + x));
      float jx = rng.uniform();
      float jy = rng.uniform();
      if (cnt) cnt->rng_draws += 2;
      float js = P.use_jitter ? 0.5f : 0.0f;
      jx *= js;
      jy *= js;
      V3 r_o = S.cam.position;
      V3 r_d = camera_dir(S.cam, px, py, jx, jy);
      const uint32_t pix = (uint32_t)(y * rw + x);
      if (log) log->log(jid, pix, VPT_EV_NEW_RAY, &r_o, &r_d, 0.0f);
      V3 L = v3(0, 0, 0);
      bool terminated = false;
      bool escaped = false;  // mutant 4 only
      for (unsigned int depth = 0; depth < P.max_depth; ++depth) {
        bool scattered = false;
        NRay ir(v3(0, 0, 0), v3(1, 0, 0));
        if (!volume_intersect(*S.density, r_o, r_d, ir)) {
          escaped = true;
          break;
        }
        RayMajorantIterator it(ir, S.density);
        MajorantTransmittanceSampler sampler(it, rng, S.density, sigma_t, cnt);
        MediumProperties props;
        while (sampler.next(props)) {
          if (log) log->log(jid, pix, VPT_EV_SAMPLED_POINT, &props.point, nullptr, props.density);
          float p_a = (VP.sigma_a * props.density) / props.sigma_maj;
          float p_s = (VP.sigma_s * props.density) / props.sigma_maj;
          float p_n = std::max<float>(1.0f - p_a - p_s, 0.0f);
          if (temp_sampler) {
            V3 tc = S.temperature->worldToIndexF(props.point);
            float temp_adim = (*temp_sampler)(tc);
            float temp_K = temp_adim * VP.temperature_scale + VP.temperature_offset;
            V3 bb = blackbody_radiation_xyz(S.bb, S.cie, S.y_integral, temp_K);
            float s = p_a * VP.le_scale;
            L = add(L, v3(s * bb.x, s * bb.y, s * bb.z));
          }
          float ue = rng.uniform();
          if (cnt) ++cnt->rng_draws;
          ScatterEvent ev = sample_discrete3(p_n, p_a, p_s, ue);
          if (ev == ScatterEvent::Null) {
            if (log) log->log(jid, pix, VPT_EV_NULL, nullptr, nullptr, 0.0f);
            continue;
          } else if (ev == ScatterEvent::Scatter) {
            if ((VPTO_MUTANT == 3 ? depth : depth++) >= P.max_depth) {
              if (log) log->log(jid, pix, VPT_EV_SCATTER_TERMINATED, nullptr, nullptr, 0.0f);
              terminated = true;
              break;
            }
            if (cnt) ++cnt->scatters;
            L = add(L, sample_Ld(S, rng, props.point, r_d, cnt));
            float u0 = rng.uniform();
            float u1 = rng.uniform();
            if (cnt) cnt->rng_draws += 2;
            V3 nd = sample_henyey_greenstein(r_d, u0, u1, VP.henyey_greenstein_g);
            r_o = props.point;
            r_d = nd;
            if (log) log->log(jid, pix, VPT_EV_SCATTER, &r_o, &r_d, 0.0f);
            scattered = true;
            break;
          } else {
            if (log) log->log(jid, pix, VPT_EV_ABSORBED, nullptr, nullptr, 0.0f);
            terminated = true;
            break;
          }
        }
        if (!scattered) {
          escaped = !terminated;
          break;
        }
      }
      if (!terminated && (VPTO_MUTANT != 4 || escaped)) {
        L = add(L, v3(P.infinite_light_xyz[0] * P.infinite_light_multiplier,
                      P.infinite_light_xyz[1] * P.infinite_light_multiplier,
                      P.infinite_light_xyz[2] * P.infinite_light_multiplier));
      }
      float* f = film + (py * W + px) * 4;
      f[3] += 1.0f;
      const float ir = cfg.camera_parameters.imaging_ratio;
      f[0] += ir * L.x;
      f[1] += ir * L.y;
      f[2] += ir * L.z;
      if (records) {
        float* r = records + (record_base * (uint64_t)(tw * th) + (uint64_t)(y * rw + x)) * 3;
        r[0] = L.x;
        r[1] = L.y;
        r[2] = L.z;
      }
      if (cnt) ++cnt->samples;
    }
  }
}

Scene make_scene(const vpt_configuration* cfg, const Grid* d, const Grid* t, const float* bb, const float* cie,
                 float yint) {
  Scene S;
  S.cfg = cfg;
  S.density = d;
  S.temperature = t;
  S.bb = bb;
  S.cie = cie;
  S.y_integral = yint;
  S.cam = make_camera(*cfg);
  auto ceildiv = [](int64_t x, int64_t y) { return x / y + (x % y != 0); };
  S.ntx = (uint64_t)ceildiv(cfg->output_size[0], cfg->tile_size[0]);
  S.nty = (uint64_t)ceildiv(cfg->output_size[1], cfg->tile_size[1]);
  S.T = S.ntx * S.nty;
  return S;
}

// ------------------------------------------------------------------------------------------
// TileProvider: src/tile_provider.cpp:14-111, include/vpt/tile_provider.hpp:15-106
// ------------------------------------------------------------------------------------------
struct TileProvider {
  std::mutex mtx;
  unsigned requested_waves;
  std::atomic<unsigned> max_wave_idx{0};
  std::atomic<bool> force_stop{false};
  std::atomic<size_t> job_idx{0};
  std::vector<std::atomic<unsigned>> tile_wave;
  TileProvider(unsigned waves, size_t ntiles) : requested_waves(waves), tile_wave(ntiles) {
    for (auto& a : tile_wave) a.store(0);
  }
  bool wave_should_be_processed(unsigned idx) {
    if (idx <= max_wave_idx.load(std::memory_order_relaxed)) return true;
    std::unique_lock<std::mutex> lock(mtx);
    if (idx <= max_wave_idx.load()) return true;
    if (idx > requested_waves) return false;
    max_wave_idx.store(idx);
    return true;
  }
  // next(): returns false for the invalid token; otherwise tile/wave/jid.
  bool next(unsigned& tile, unsigned& wave, size_t& jid) {
    size_t j = job_idx.fetch_add(1, std::memory_order_relaxed);
    unsigned w = 1 + (unsigned)(j / tile_wave.size());
    unsigned t = (unsigned)(j % tile_wave.size());
    if (force_stop || !wave_should_be_processed(w)) return false;
    while (!force_stop) {
      unsigned tw = tile_wave[t].load(std::memory_order_relaxed);
      if (tw == w - 1) break;
      tile_wave[t].wait(tw, std::memory_order_relaxed);
    }
    if (force_stop) return false;
    tile = t;
    wave = w;
    jid = j;
    return true;
  }
  void release(unsigned tile, unsigned wave) {  // ~token()
    tile_wave[tile].store(wave);
    tile_wave[tile].notify_all();
  }
};

void add_counters(vpt_counters* dst, const vpt_counters& s) {
  dst->samples += s.samples;
  dst->dda_steps += s.dda_steps;
  dst->segments += s.segments;
  dst->draws += s.draws;
  dst->stencils += s.stencils;
  dst->density_evals += s.density_evals;
  dst->temp_stencils += s.temp_stencils;
  dst->scatters += s.scatters;
  dst->shadow_rays += s.shadow_rays;
  dst->rng_draws += s.rng_draws;
}

// ------------------------------------------------------------------------------------------
// Synthetic stand-in volumes, independent of the product generator.
// ------------------------------------------------------------------------------------------
struct OwnedDesc {
  vpt_grid_desc d;
  std::vector<int32_t> origin;
  std::vector<float> values;
  std::vector<uint64_t> mask;
  std::vector<float> maxv;
};

double synth_value(int kind, int n, int i, int j, int k) {
  if (kind == 0) return 1.0;
  double half = n / 2.0;
  double px = (i + 0.5) / half - 1.0, py = (j + 0.5) / half - 1.0, pz = (k + 0.5) / half - 1.0;
  double r = std::sqrt(px * px + py * py + pz * pz);
  double base = std::min(1.0, std::max(0.0, (0.85 - r) / 0.35));
  if (kind == 2) return 40.0 * base;
  return base * (0.5 + 0.5 * std::sin(11.0 * px + 2.0) * std::sin(13.0 * py + 1.0) * std::sin(17.0 * pz + 3.0));
}

}  // namespace

// ==========================================================================================
// extern "C" API
// ==========================================================================================
struct vpto_grid {
  Grid g;
};

extern "C" {

uint64_t vpto_hash(uint64_t seed, uint64_t jid) { return murmur64a_one_word(seed, jid); }

void vpto_rng_u32(uint32_t seed, uint64_t jid, uint32_t* out, int n) {
  Rng r;
  r.begin_job(seed, jid);
  for (int i = 0; i < n; ++i) out[i] = r.next_u32();
}
void vpto_rng_f32(uint32_t seed, uint64_t jid, float* out, int n) {
  Rng r;
  r.begin_job(seed, jid);
  for (int i = 0; i < n; ++i) out[i] = r.uniform();
}

float vpto_planck(float lambda_m, float t) { return planck_law(lambda_m, t); }

void vpto_blackbody_table(const float* cie, float y_integral, float* out) {
  for (int i = 0; i < 500; ++i) {  // init_blackbody_radiation_xyz (precompute_blackbody.cpp:18-22)
    V3 v = spectrum_to_xyz(cie, y_integral, idx_to_temp(i));
    out[i * 3 + 0] = v.x;
    out[i * 3 + 1] = v.y;
    out[i * 3 + 2] = v.z;
  }
}

void vpto_blackbody_xyz(const float* table, const float* cie, float y_integral, float t, float* out3) {
  std::vector<float> padded(501 * 3, 0.0f);
  std::memcpy(padded.data(), table, 500 * 3 * sizeof(float));
  V3 v = blackbody_radiation_xyz(padded.data(), cie, y_integral, t);
  out3[0] = v.x;
  out3[1] = v.y;
  out3[2] = v.z;
}

vpto_grid* vpto_grid_create(const vpt_grid_desc* d) {
  std::unique_ptr<vpto_grid> G(new vpto_grid());
  Grid& g = G->g;
  std::memcpy(g.mat, d->map_mat, sizeof g.mat);
  std::memcpy(g.inv_mat, d->map_inv_mat, sizeof g.inv_mat);
  std::memcpy(g.vec, d->map_vec, sizeof g.vec);
  g.background = d->background;
  std::memcpy(g.bbox_min, d->index_bbox_min, sizeof g.bbox_min);
  std::memcpy(g.bbox_max, d->index_bbox_max, sizeof g.bbox_max);
  std::map<Key, int32_t> lower_of, upper_of;
  auto get_upper = [&](int32_t i, int32_t j, int32_t k) -> int32_t {
    Key key(i & ~4095, j & ~4095, k & ~4095);
    auto it = upper_of.find(key);
    if (it != upper_of.end()) return it->second;
    Upper u;
    u.origin[0] = std::get<0>(key);
    u.origin[1] = std::get<1>(key);
    u.origin[2] = std::get<2>(key);
    u.child.assign(32768, -1);
    u.tile.assign(32768, g.background);
    u.active.assign(32768, 0);
    g.uppers.push_back(std::move(u));
    int32_t idx = (int32_t)g.uppers.size() - 1;
    upper_of[key] = idx;
    RootTile& rt = g.root[key];
    rt.upper = idx;
    return idx;
  };
  auto get_lower = [&](int32_t i, int32_t j, int32_t k) -> int32_t {
    Key key(i & ~127, j & ~127, k & ~127);
    auto it = lower_of.find(key);
    if (it != lower_of.end()) return it->second;
    int32_t ui = get_upper(i, j, k);
    Lower l;
    l.origin[0] = std::get<0>(key);
    l.origin[1] = std::get<1>(key);
    l.origin[2] = std::get<2>(key);
    l.child.assign(4096, -1);
    l.tile.assign(4096, g.background);
    l.active.assign(4096, 0);
    g.lowers.push_back(std::move(l));
    int32_t idx = (int32_t)g.lowers.size() - 1;
    lower_of[key] = idx;
    g.uppers[ui].child[upper_offset(i, j, k)] = idx;
    return idx;
  };
  for (uint64_t u = 0; u < d->upper_count; ++u)
    get_upper(d->upper_origin[u * 3], d->upper_origin[u * 3 + 1], d->upper_origin[u * 3 + 2]);
  for (uint64_t u = 0; u < d->lower_count; ++u)
    get_lower(d->lower_origin[u * 3], d->lower_origin[u * 3 + 1], d->lower_origin[u * 3 + 2]);
  g.leaves.resize(d->leaf_count);
  for (uint64_t n = 0; n < d->leaf_count; ++n) {
    Leaf& lf = g.leaves[n];
    for (int a = 0; a < 3; ++a) lf.origin[a] = d->leaf_origin[n * 3 + a];
    std::memcpy(lf.v, d->leaf_values + n * 512, 512 * sizeof(float));
    if (d->leaf_value_mask)
      std::memcpy(lf.mask, d->leaf_value_mask + n * 8, 8 * sizeof(uint64_t));
    else
      std::memset(lf.mask, 0xff, sizeof lf.mask);
    lf.max = d->leaf_max[n];
    int32_t li = get_lower(lf.origin[0], lf.origin[1], lf.origin[2]);
    g.lowers[li].child[lower_offset(lf.origin[0], lf.origin[1], lf.origin[2])] = (int32_t)n;
  }
  for (uint64_t t = 0; t < d->tile_count; ++t) {
    int32_t i = d->tile_origin[t * 3], j = d->tile_origin[t * 3 + 1], k = d->tile_origin[t * 3 + 2];
    int lvl = d->tile_level[t];
    float v = d->tile_value[t];
    bool act = d->tile_active[t] != 0;
    if (lvl == 1) {
      Lower& l = g.lowers[get_lower(i, j, k)];
      uint32_t o = lower_offset(i, j, k);
      l.tile[o] = v;
      l.active[o] = act;
    } else if (lvl == 2) {
      Upper& u = g.uppers[get_upper(i, j, k)];
      uint32_t o = upper_offset(i, j, k);
      u.tile[o] = v;
      u.active[o] = act;
    } else {
      RootTile& rt = g.root[root_key(i, j, k)];
      rt.value = v;
      rt.active = act;
    }
  }
  g.update_stats();
  return G.release();
}

void vpto_grid_destroy(vpto_grid* g) { delete g; }

uint64_t vpto_grid_fix_majorants(vpto_grid* G) {  // volume.cpp:104-160 (order = 1)
  Grid& g = G->g;
  std::vector<float> fixed(g.leaves.size());
  for (size_t n = 0; n < g.leaves.size(); ++n) {
    const Leaf& leaf = g.leaves[n];
    float m = leaf.max;
    const int32_t* o = leaf.origin;
    int32_t lmin[3] = {o[0], o[1], o[2]}, lmax[3] = {o[0] + 7, o[1] + 7, o[2] + 7};
    int32_t amin[3] = {lmin[0] - 1, lmin[1] - 1, lmin[2] - 1}, amax[3] = {lmax[0] + 1, lmax[1] + 1, lmax[2] + 1};
    for (int i = -1; i <= 1; ++i)
      for (int j = -1; j <= 1; ++j)
        for (int k = -1; k <= 1; ++k) {
          if (i == 0 && j == 0 && k == 0) continue;
          int32_t nmin[3] = {lmin[0] + i * 8, lmin[1] + j * 8, lmin[2] + k * 8};
          int32_t nmax[3] = {lmax[0] + i * 8, lmax[1] + j * 8, lmax[2] + k * 8};
          for (int a = 0; a < 3; ++a) {
            nmin[a] = std::max(nmin[a], amin[a]);
            nmax[a] = std::min(nmax[a], amax[a]);
          }
          for (int32_t x = nmin[0]; x <= nmax[0]; ++x)
            for (int32_t y = nmin[1]; y <= nmax[1]; ++y)
              for (int32_t z = nmin[2]; z <= nmax[2]; ++z) m = std::max(m, g.getValue(x, y, z));
        }
    fixed[n] = m;
  }
  for (size_t n = 0; n < g.leaves.size(); ++n) g.leaves[n].max = fixed[n];  // leaf.setMax
  return g.leaves.size();
}

void vpto_grid_leaf_max(const vpto_grid* G, float* out) {
  for (size_t n = 0; n < G->g.leaves.size(); ++n) out[n] = G->g.leaves[n].max;
}
float vpto_grid_get_value(const vpto_grid* G, int32_t i, int32_t j, int32_t k) { return G->g.getValue(i, j, k); }
uint32_t vpto_grid_get_dim(const vpto_grid* G, int32_t i, int32_t j, int32_t k) { return G->g.getDim(i, j, k); }
float vpto_grid_sample(const vpto_grid* G, float x, float y, float z) {
  Trilinear t(&G->g);
  return t(v3(x, y, z));
}

void vpto_camera_matrix(const vpt_configuration* cfg, float* lin9, float* trans3) {
  CameraM c = make_camera(*cfg);
  std::memcpy(lin9, c.L, sizeof c.L);
  std::memcpy(trans3, c.t, sizeof c.t);
}
void vpto_camera_ray(const vpt_configuration* cfg, int64_t x, int64_t y, float jx, float jy, float* o, float* d) {
  CameraM c = make_camera(*cfg);
  V3 dir = camera_dir(c, x, y, jx, jy);
  o[0] = c.position.x;
  o[1] = c.position.y;
  o[2] = c.position.z;
  d[0] = dir.x;
  d[1] = dir.y;
  d[2] = dir.z;
}

int vpto_trace_segments(const vpto_grid* G, const float* o, const float* d, float* out, int max_segments) {
  NRay ir(v3(0, 0, 0), v3(1, 0, 0));
  if (!volume_intersect(G->g, v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]), ir)) return -1;
  RayMajorantIterator it(ir, &G->g);
  Segment s;
  int n = 0;
  while (it.next(s)) {
    if (n < max_segments) {
      out[n * 3 + 0] = s.t0;
      out[n * 3 + 1] = s.t1;
      out[n * 3 + 2] = s.d_maj;
    }
    ++n;
  }
  return n;
}

int vpto_render_jobs_mode(const vpt_configuration* cfg, const vpto_grid* density, const vpto_grid* temperature,
                          const float* bb_table, const float* cie, float y_integral, uint64_t jid_begin,
                          uint64_t jid_count, int rng_mode, float* film, float* records) {
  if (!cfg || !density || !film) return VPT_E_INVALID;
  std::vector<float> bb(501 * 3, 0.0f);
  if (bb_table) std::memcpy(bb.data(), bb_table, 500 * 3 * sizeof(float));
  Scene S = make_scene(cfg, &density->g, temperature ? &temperature->g : nullptr, bb.data(), cie, y_integral);
  for (uint64_t j = 0; j < jid_count; ++j)
    run_job(S, jid_begin + j, film, records, j, nullptr, nullptr, rng_mode == VPT_RNG_PIXEL);
  return VPT_OK;
}

int vpto_render_jobs_events(const vpt_configuration* cfg, const vpto_grid* density, const vpto_grid* temperature,
                            const float* bb_table, const float* cie, float y_integral, uint64_t jid_begin,
                            uint64_t jid_count, float* film, vpt_event* events, uint64_t capacity, uint64_t* count) {
  if (!cfg || !density || !film || !count) return VPT_E_INVALID;
  std::vector<float> bb(501 * 3, 0.0f);
  if (bb_table) std::memcpy(bb.data(), bb_table, 500 * 3 * sizeof(float));
  Scene S = make_scene(cfg, &density->g, temperature ? &temperature->g : nullptr, bb.data(), cie, y_integral);
  EventSink sink{events, events ? capacity : 0};
  for (uint64_t j = 0; j < jid_count; ++j) run_job(S, jid_begin + j, film, nullptr, j, nullptr, &sink);
  *count = sink.n;
  return VPT_OK;
}

// Volume::log_majorant_trace (volume.cpp:176-192): rows X0,Y0,Z0,X1,Y1,Z1,T0,T1,Majorant.
int vpto_majorant_trace(const vpto_grid* G, const float* o, const float* d, float* rows, int max_rows) {
  NRay ir(v3(0, 0, 0), v3(1, 0, 0));
  if (!volume_intersect(G->g, v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]), ir)) return 0;
  RayMajorantIterator it(ir, &G->g);
  Segment sg;
  int n = 0;
  while (it.next(sg)) {
    if (n < max_rows) {
      const float w0 = sg.t0 * it.scale, w1 = sg.t1 * it.scale;  // t * idx_to_world_scale()
      const V3 p0 = G->g.worldToIndexF(v3(o[0] + d[0] * w0, o[1] + d[1] * w0, o[2] + d[2] * w0));
      const V3 p1 = G->g.worldToIndexF(v3(o[0] + d[0] * w1, o[1] + d[1] * w1, o[2] + d[2] * w1));
      const float r[9] = {p0.x, p0.y, p0.z, p1.x, p1.y, p1.z, w0, w1, sg.d_maj};
      std::memcpy(rows + 9 * n, r, sizeof r);
    }
    ++n;
  }
  return n;
}

// Volume::log_dda_trace (volume.cpp:194-225): NanoVDB math::DDA<Ray<float>, Coord, 1> (HDDA.h,
// restated) over the index ray clipped to the bbox and widened by 16 at both ends.
int vpto_dda_trace(const vpto_grid* G, const float* o, const float* d, vpt_dda_row* rows, int max_rows) {
  const Grid& g = G->g;
  NRay w_ray(v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]));
  w_ray.t1 = 10000.0f;  // setMaxTime
  NRay ray = w_ray.worldToIndexF(g);
  if (!ray.clip(g.bbox_min, g.bbox_max)) return -1;
  ray.t0 = ray.t0 - 16.0f;  // setMinTime / setMaxTime
  ray.t1 = ray.t1 + 16.0f;
  // DDA::init
  float t0 = ray.t0;
  const V3 pos = ray.at(t0);
  const float P[3] = {pos.x, pos.y, pos.z}, D[3] = {ray.dir.x, ray.dir.y, ray.dir.z}, I[3] = {ray.inv.x, ray.inv.y, ray.inv.z};
  int32_t voxel[3], stp[3];
  float next[3], delta[3] = {0.0f, 0.0f, 0.0f};
  for (int a = 0; a < 3; ++a) {
    voxel[a] = nvdb_floor(P[a]);  // RoundDown<Coord>(pos) & ~(Dim - 1), Dim = 1
    if (D[a] == 0.0f) {
      next[a] = std::numeric_limits<float>::max();
      stp[a] = 0;
    } else if (I[a] > 0) {
      stp[a] = 1;
      next[a] = t0 + ((float)(voxel[a] + 1) - P[a]) * I[a];
      delta[a] = I[a];
    } else {
      stp[a] = -1;
      next[a] = t0 + ((float)voxel[a] - P[a]) * I[a];
      delta[a] = -I[a];
    }
  }
  int n = 0;
  do {
    if (n < max_rows) {
      vpt_dda_row& r = rows[n];
      const Grid::Hit h = g.query(voxel[0], voxel[1], voxel[2]);
      for (int a = 0; a < 3; ++a) r.ijk[a] = voxel[a];
      r.t = t0;
      r.value = h.value;                // getValue
      r.dim_getdim = h.dim;             // getDim(ijk, ray)
      g.node_info(voxel[0], voxel[1], voxel[2], r.dim_nodeinfo, r.maximum);
      r.active = h.active ? 1 : 0;      // isActive
    }
    ++n;
    // DDA::step
    const int axis = (next[0] < next[1] && next[0] < next[2]) ? 0 : (next[1] < next[2] ? 1 : 2);
    t0 = next[axis];
    next[axis] += delta[axis];
    voxel[axis] += stp[axis];
  } while (t0 <= ray.t1);
  return n;
}

int vpto_render_jobs(const vpt_configuration* cfg, const vpto_grid* density, const vpto_grid* temperature,
                     const float* bb_table, const float* cie, float y_integral, uint64_t jid_begin,
                     uint64_t jid_count, float* film, float* records, vpt_counters* counters) {
  if (!cfg || !density || !film) return VPT_E_INVALID;
  std::vector<float> bb(501 * 3, 0.0f);
  if (bb_table) std::memcpy(bb.data(), bb_table, 500 * 3 * sizeof(float));
  Scene S = make_scene(cfg, &density->g, temperature ? &temperature->g : nullptr, bb.data(), cie, y_integral);
  vpt_counters local{};
  for (uint64_t j = 0; j < jid_count; ++j)
    run_job(S, jid_begin + j, film, records, j, counters ? &local : nullptr);
  if (counters) add_counters(counters, local);
  return VPT_OK;
}

double vpto_render_pool(const vpt_configuration* cfg, const vpto_grid* density, const vpto_grid* temperature,
                        const float* bb_table, const float* cie, float y_integral, uint32_t num_waves,
                        int num_workers, float* film, vpt_counters* counters) {
  if (!cfg || !density || !film || num_workers <= 0) return -1.0;
  std::vector<float> bb(501 * 3, 0.0f);
  if (bb_table) std::memcpy(bb.data(), bb_table, 500 * 3 * sizeof(float));
  Scene S = make_scene(cfg, &density->g, temperature ? &temperature->g : nullptr, bb.data(), cie, y_integral);
  TileProvider tp(num_waves, (size_t)S.T);
  std::mutex cmtx;
  auto t0 = std::chrono::steady_clock::now();
  {
    std::vector<std::thread> threads;
    for (int w = 0; w < num_workers; ++w) {
      threads.emplace_back([&]() {  // main.cpp:63-68 -> vpt::run
        vpt_counters local{};
        unsigned tile, wave;
        size_t jid;
        while (tp.next(tile, wave, jid)) {
          run_job(S, jid, film, nullptr, 0, counters ? &local : nullptr);
          tp.release(tile, wave);
        }
        if (counters) {
          std::lock_guard<std::mutex> lk(cmtx);
          add_counters(counters, local);
        }
      });
    }
    for (auto& t : threads) t.join();
  }
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::milli>(t1 - t0).count();
}

vpt_grid_desc* vpto_synth_grid(int kind, int n) {
  if (n <= 0 || (n % 8) != 0 || kind < 0 || kind > 2) return nullptr;
  OwnedDesc* od = new OwnedDesc();
  const int nl = n / 8;
  std::vector<float> buf(512);
  int32_t bmin[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, bmax[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
  for (int li = 0; li < nl; ++li)
    for (int lj = 0; lj < nl; ++lj)
      for (int lk = 0; lk < nl; ++lk) {
        bool any = false;
        float mx = -std::numeric_limits<float>::infinity();
        uint64_t mask[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int a = 0; a < 8; ++a)
          for (int b = 0; b < 8; ++b)
            for (int c = 0; c < 8; ++c) {
              float v = (float)synth_value(kind, n, li * 8 + a, lj * 8 + b, lk * 8 + c);
              uint32_t off = (uint32_t)(a << 6 | b << 3 | c);
              buf[off] = v;
              if (v != 0.0f) {
                any = true;
                const int32_t c3[3] = {li * 8 + a, lj * 8 + b, lk * 8 + c};
                for (int e = 0; e < 3; ++e) {
                  bmin[e] = std::min(bmin[e], c3[e]);
                  bmax[e] = std::max(bmax[e], c3[e]);
                }
                mask[off >> 6] |= 1ULL << (off & 63);
                mx = std::max(mx, v);
              }
            }
        if (!any) continue;
        od->origin.push_back(li * 8);
        od->origin.push_back(lj * 8);
        od->origin.push_back(lk * 8);
        od->values.insert(od->values.end(), buf.begin(), buf.end());
        od->mask.insert(od->mask.end(), mask, mask + 8);
        od->maxv.push_back(mx);
      }
  vpt_grid_desc& d = od->d;
  std::memset(&d, 0, sizeof d);
  float half = (float)(n / 2);
  for (int a = 0; a < 9; ++a) d.map_mat[a] = d.map_inv_mat[a] = (a % 4 == 0) ? 1.0f : 0.0f;
  for (int a = 0; a < 3; ++a) {
    d.map_vec[a] = -half;
    d.index_bbox_min[a] = bmin[a];  // NanoVDB indexBBox = bbox of the active voxels
    d.index_bbox_max[a] = bmax[a];
  }
  d.background = 0.0f;
  d.leaf_count = od->maxv.size();
  d.leaf_origin = od->origin.data();
  d.leaf_values = od->values.data();
  d.leaf_value_mask = od->mask.data();
  d.leaf_max = od->maxv.data();
  return &od->d;
}

void vpto_synth_free(vpt_grid_desc* d) { delete reinterpret_cast<OwnedDesc*>(d); }

// film_to_image (main.cpp:12-24) with xyz_to_linsrgb / linsrgb_to_srgb (color.hpp:8-30).
void vpto_film_to_image(const float* film, int64_t w, int64_t h, uint8_t* out) {
  float m[9] = {(float)3.240479, (float)-1.537150, (float)-0.498535, (float)-0.969256, (float)1.875991,
                (float)0.041556, (float)0.055648, (float)-0.204043, (float)1.057311};
  auto srgb = [](float x) { return x <= 0.0031308f ? (12.92f * x) : (1.055f * std::pow(x, 1.0f / 2.4f) - 0.055f); };
  for (int64_t i = 0; i < w * h; ++i) {
    const float* p = film + i * 4;
    V3 xyz = v3(p[0] / p[3], p[1] / p[3], p[2] / p[3]);
    float lin[3];
    for (int r = 0; r < 3; ++r) lin[r] = m[r * 3] * xyz.x + (m[r * 3 + 1] * xyz.y + m[r * 3 + 2] * xyz.z);
    for (int c = 0; c < 3; ++c) {
      float v = std::min(std::max(srgb(lin[c]), 0.0f), 1.0f) * 255.0f;  // cwiseMax(0).cwiseMin(1) * 255
      out[i * 3 + c] = (v == v) ? (uint8_t)(int32_t)v : (uint8_t)0;  // cast<unsigned char>
    }
  }
}

}  // extern "C"
