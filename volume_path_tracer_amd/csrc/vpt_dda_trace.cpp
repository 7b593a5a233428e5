// vpt_dda_trace.cpp — Volume::log_dda_trace (src/volume.cpp:194-225) over a vpt_grid_desc.
//
// A debug aid, not part of the hot path: one world ray walked voxel by voxel with NanoVDB's
// math::DDA<Ray<float>, Coord, 1>, printing per voxel the ReadAccessor answers getValue, getDim,
// getNodeInfo (dim, maximum) and isActive.  It runs on the host over the grid description (the
// device tables carry neither voxel active masks nor internal-node statistics).
//
// NanoVDB semantics restated (the submodule is absent from the reference mount: parity unpinned):
// * Ray(eye, dir) has t0 = 1e-5 (Delta<float>), setMaxTime(10000); Ray::worldToIndexF,
//   Ray::clip(indexBBox) as in begin_ray (vpt_integrator.h); then t0 -= 16, t1 += 16.
// * DDA<Dim 1>::init/step: HDDA with dim 1 (voxel = floor(ray(t0)), next/delta per axis,
//   axis = MinIndex(next), time = next[axis], next[axis] += delta[axis]; continue while time <= t1).
// * getNodeInfo: the deepest node holding ijk -- leaf (dim 8, maximum = the leaf max after
//   fix_majorants_for_interpolation, which writes it into the grid at Volume construction), lower
//   node (dim 128), upper node (dim 4096), else the root (dim 4096, ChildT::dim()).  Internal node
//   and root maxima are NanoVDB's build statistics: the maximum over the stored maxima of child
//   nodes and the values of active tiles (0 for a node with no active value).
#include <algorithm>
#include <cmath>
#include <limits>
#include <unordered_map>
#include <vector>

#include "vpt_internal.h"

namespace vpt {
namespace {

struct K3 {
  int32_t i, j, k;
  bool operator==(const K3& o) const { return i == o.i && j == o.j && k == o.k; }
};
struct K3Hash {
  size_t operator()(const K3& a) const {
    return (size_t)(((uint64_t)(uint32_t)a.i * 0x9E3779B97F4A7C15ULL) ^ ((uint64_t)(uint32_t)a.j << 21) ^
                    ((uint64_t)(uint32_t)a.k << 42) ^ ((uint64_t)(uint32_t)a.k >> 22));
  }
};
struct Tile {
  float value;
  bool active;
};
// Running maximum of a node's active values / child maxima ("no value yet" until the first).
struct NodeMax {
  float v = 0.0f;
  bool any = false;
  void add(float x) {
    v = any ? std::max(v, x) : x;
    any = true;
  }
};

struct TraceGrid {
  const vpt_grid_desc& d;
  std::vector<float> leaf_max_fixed;
  std::unordered_map<K3, uint32_t, K3Hash> leaf;
  std::unordered_map<K3, Tile, K3Hash> t1, t2, t3;  // tiles of lower / upper nodes / root
  std::unordered_map<K3, NodeMax, K3Hash> lower, upper;
  NodeMax root;

  explicit TraceGrid(const vpt_grid_desc& desc) : d(desc) {}

  int build() {
    leaf_max_fixed.resize(d.leaf_count);
    if (d.leaf_count) {
      int rc = vpt_fix_majorants(&d, leaf_max_fixed.data(), 0);
      if (rc) return rc;
    }
    for (uint64_t n = 0; n < d.leaf_count; ++n) {
      const int32_t* o = d.leaf_origin + 3 * n;
      leaf[K3{o[0], o[1], o[2]}] = (uint32_t)n;
      lower[K3{o[0] & ~127, o[1] & ~127, o[2] & ~127}].add(d.leaf_max[n]);
    }
    for (uint64_t n = 0; n < d.lower_count; ++n) {
      const int32_t* o = d.lower_origin + 3 * n;
      lower[K3{o[0] & ~127, o[1] & ~127, o[2] & ~127}];
    }
    for (uint64_t n = 0; n < d.upper_count; ++n) {
      const int32_t* o = d.upper_origin + 3 * n;
      upper[K3{o[0] & ~4095, o[1] & ~4095, o[2] & ~4095}];
    }
    for (uint64_t n = 0; n < d.tile_count; ++n) {
      const int32_t* o = d.tile_origin + 3 * n;
      const Tile t{d.tile_value[n], d.tile_active[n] != 0};
      if (d.tile_level[n] == 1) {
        t1[K3{o[0] & ~7, o[1] & ~7, o[2] & ~7}] = t;
        NodeMax& m = lower[K3{o[0] & ~127, o[1] & ~127, o[2] & ~127}];
        if (t.active) m.add(t.value);
      } else if (d.tile_level[n] == 2) {
        t2[K3{o[0] & ~127, o[1] & ~127, o[2] & ~127}] = t;
        NodeMax& m = upper[K3{o[0] & ~4095, o[1] & ~4095, o[2] & ~4095}];
        if (t.active) m.add(t.value);
      } else if (d.tile_level[n] == 3) {
        t3[K3{o[0] & ~4095, o[1] & ~4095, o[2] & ~4095}] = t;
      } else {
        return set_error(VPT_E_INVALID, "grid: tile_level must be 1, 2 or 3");
      }
    }
    for (const auto& l : lower) {
      NodeMax& m = upper[K3{l.first.i & ~4095, l.first.j & ~4095, l.first.k & ~4095}];
      if (l.second.any) m.add(l.second.v);
    }
    for (const auto& u : upper) {
      t3.erase(u.first);  // a root slot holds a child or a value
      if (u.second.any) root.add(u.second.v);
    }
    for (const auto& t : t3)
      if (t.second.active) root.add(t.second.value);
    return VPT_OK;
  }

  void query(int32_t i, int32_t j, int32_t k, vpt_dda_row& r) const {
    r.ijk[0] = i;
    r.ijk[1] = j;
    r.ijk[2] = k;
    auto lf = leaf.find(K3{i & ~7, j & ~7, k & ~7});
    if (lf != leaf.end()) {
      const uint32_t n = ((uint32_t)(i & 7) << 6) | ((uint32_t)(j & 7) << 3) | (uint32_t)(k & 7);
      r.value = d.leaf_values[(uint64_t)lf->second * 512 + n];
      r.active = d.leaf_value_mask ? (int32_t)((d.leaf_value_mask[(uint64_t)lf->second * 8 + (n >> 6)] >> (n & 63)) & 1) : 1;
      r.dim_getdim = 1;
      r.dim_nodeinfo = 8;
      r.maximum = leaf_max_fixed[lf->second];
      return;
    }
    auto lo = lower.find(K3{i & ~127, j & ~127, k & ~127});
    if (lo != lower.end()) {
      auto t = t1.find(K3{i & ~7, j & ~7, k & ~7});
      r.value = t != t1.end() ? t->second.value : d.background;
      r.active = t != t1.end() && t->second.active;
      r.dim_getdim = 8;
      r.dim_nodeinfo = 128;
      r.maximum = lo->second.any ? lo->second.v : 0.0f;
      return;
    }
    auto up = upper.find(K3{i & ~4095, j & ~4095, k & ~4095});
    if (up != upper.end()) {
      auto t = t2.find(K3{i & ~127, j & ~127, k & ~127});
      r.value = t != t2.end() ? t->second.value : d.background;
      r.active = t != t2.end() && t->second.active;
      r.dim_getdim = 128;
      r.dim_nodeinfo = 4096;
      r.maximum = up->second.any ? up->second.v : 0.0f;
      return;
    }
    auto t = t3.find(K3{i & ~4095, j & ~4095, k & ~4095});
    r.value = t != t3.end() ? t->second.value : d.background;
    r.active = t != t3.end() && t->second.active;
    r.dim_getdim = 4096;
    r.dim_nodeinfo = 4096;
    r.maximum = root.any ? root.v : 0.0f;
  }
};

}  // namespace
}  // namespace vpt

extern "C" int vpt_dda_trace(const vpt_grid_desc* density, const float origin[3], const float direction[3],
                             vpt_dda_row* rows, int max_rows, int* n_rows) {
  using namespace vpt;
  if (!density || !origin || !direction || !n_rows || max_rows < 0 || (max_rows && !rows))
    return set_error(VPT_E_INVALID, "vpt_dda_trace: bad argument");
  TraceGrid g(*density);
  int rc = g.build();
  if (rc) return rc;
  DevGrid G{};
  std::copy(density->map_mat, density->map_mat + 9, G.mat);
  std::copy(density->map_inv_mat, density->map_inv_mat + 9, G.inv_mat);
  std::copy(density->map_vec, density->map_vec + 3, G.vec);
  // Ray(eye, dir) -> setMaxTime(10000) -> worldToIndexF (ray_dir_setup: the same float operations)
  const RayDir rd = ray_dir_setup(G, direction);
  float e[3];
  map_inv(G, origin[0], origin[1], origin[2], e[0], e[1], e[2]);
  float t0 = rd.len * 1e-5f, t1 = 10000.0f * rd.len;
  // Ray::clip(indexBBox): slab test against [min, max + 1]
  for (int a = 0; a < 3; ++a) {
    float lo = (float)density->index_bbox_min[a], hi = (float)(density->index_bbox_max[a] + 1);
    lo = (lo - e[a]) * rd.inv[a];
    hi = (hi - e[a]) * rd.inv[a];
    if (lo > hi) std::swap(lo, hi);
    if (lo > t0) t0 = lo;
    if (hi < t1) t1 = hi;
    if (t0 > t1) {
      *n_rows = -1;  // the reference returns before creating dda_trace.csv
      return VPT_OK;
    }
  }
  t0 = t0 - 16.0f;  // ray.setMinTime(ray.t0() - 16), setMaxTime(ray.t1() + 16)
  t1 = t1 + 16.0f;
  // DDA<Ray<float>, Coord, 1>::init
  float T = t0, next[3], delta[3] = {0, 0, 0};
  int32_t vox[3], step[3];
  const float P[3] = {e[0] + rd.d[0] * T, e[1] + rd.d[1] * T, e[2] + rd.d[2] * T};
  for (int a = 0; a < 3; ++a) {
    vox[a] = (int32_t)std::floor(P[a]);
    if (rd.d[a] == 0.0f) {
      next[a] = std::numeric_limits<float>::max();
      step[a] = 0;
    } else if (rd.inv[a] > 0) {
      step[a] = 1;
      next[a] = T + ((float)(vox[a] + 1) - P[a]) * rd.inv[a];
      delta[a] = rd.inv[a];
    } else {
      step[a] = -1;
      next[a] = T + ((float)vox[a] - P[a]) * rd.inv[a];
      delta[a] = -rd.inv[a];
    }
  }
  int n = 0;
  while (true) {
    if (n < max_rows) {
      g.query(vox[0], vox[1], vox[2], rows[n]);
      rows[n].t = T;
    }
    ++n;
    // DDA::step()
    const int axis = (next[0] < next[1] && next[0] < next[2]) ? 0 : (next[1] < next[2] ? 1 : 2);
    T = next[axis];
    next[axis] += delta[axis];
    vox[axis] += step[axis];
    if (!(T <= t1)) break;
  }
  *n_rows = n;
  return VPT_OK;
}
