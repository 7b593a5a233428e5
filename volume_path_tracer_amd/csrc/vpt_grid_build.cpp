// vpt_grid_build.cpp — flattens a NanoVDB-style float grid into the GPU layout.
//
// HBM layout (per grid):
//   cells8   int2[r8_n.x][r8_n.y][r8_n.z]  one entry per 8^3 voxel cell over every lower node
//            (x = leaf index or -(2*dim+active), y = leaf majorant or tile value bits)
//   cells128 int2[...]                     one entry per 128^3 cell over every upper node
//   root     RootTileDev[]                 value tiles at the root (outside every upper node)
//   walk8    uint32[w8_n.x][w8_n.y][w8_n.z] the HDDA fast path's word per cells8 entry: the majorant's
//                                          bits for an interior cell (for a +0 majorant: its zero-run
//                                          radius, see kZeroRunMax), the bits | kWalkEdge for another
//                                          dim-8 cell, kWalkSlow otherwise; padded by
//                                          kWalkPad cells of kWalkSlow on every side (w8_n = r8_n + 4)
//   bricks   float[leaf][8][8][9][4]       per voxel row (y, z) the 2x2 squares of x = 0..8; a voxel's
//                                          2x2x2 trilinear stencil is the squares of x and x + 1 (built
//                                          from 9^3 apron bricks: the leaf's voxels plus the +1
//                                          neighbours), NanoVDB SampleFromVoxels semantics
// One 8-byte cells8 load answers getDim, probeLeaf, probeValue and the majorant of
// RayMajorantIterator::update_current_majorant (volume.cpp:18-36) for any voxel of the cell.
//
// fix_majorants_for_interpolation (volume.cpp:104-160) is applied to the leaf maxima here.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <limits>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "vpt_internal.h"

namespace vpt {
namespace {

inline uint64_t pack(int32_t i, int32_t j, int32_t k) {
  return ((uint64_t)(uint32_t)i * 0x9E3779B97F4A7C15ULL) ^ ((uint64_t)(uint32_t)j << 21) ^ ((uint64_t)(uint32_t)k << 42) ^
         ((uint64_t)(uint32_t)k >> 22);
}
struct Key3 {
  int32_t i, j, k;
  bool operator==(const Key3& o) const { return i == o.i && j == o.j && k == o.k; }
};
struct Key3Hash {
  size_t operator()(const Key3& a) const { return (size_t)pack(a.i, a.j, a.k); }
};
struct TileVal {
  float value;
  int32_t active;
};

template <class F>
void parallel_for(int64_t n, int threads, F f) {
  if (threads <= 1 || n < 1024) {
    f(0, n);
    return;
  }
  std::vector<std::thread> ts;
  int64_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    int64_t b = t * chunk, e = std::min<int64_t>(n, b + chunk);
    if (b >= e) break;
    ts.emplace_back([=]() { f(b, e); });
  }
  for (auto& t : ts) t.join();
}

inline int2 enc(int32_t code, float v) {
  int32_t bits;
  std::memcpy(&bits, &v, 4);
  return int2{code, bits};
}

}  // namespace

float host_value_at(const HostGrid& g, int32_t i, int32_t j, int32_t k) { return value_at(g.dev, i, j, k); }

OwnedGrid* owned_grid_new() { return new OwnedGrid(); }

void OwnedGrid::finish() {
  vpt_grid_desc& g = d;
  g.leaf_count = leaf_max.size();
  g.leaf_origin = leaf_origin.data();
  g.leaf_values = leaf_values.data();
  g.leaf_value_mask = leaf_mask.data();
  g.leaf_max = leaf_max.data();
  g.tile_count = tile_value.size();
  g.tile_origin = tile_origin.data();
  g.tile_level = tile_level.data();
  g.tile_value = tile_value.data();
  g.tile_active = tile_active.data();
  g.lower_count = lower_origin.size() / 3;
  g.lower_origin = lower_origin.data();
  g.upper_count = upper_origin.size() / 3;
  g.upper_origin = upper_origin.data();
}


void compute_runs(HostGrid& h, int threads) {
  if (threads <= 0) threads = default_threads();
  const DevGrid& G = h.dev;
  const std::vector<int2>& cells8 = h.cells8;
  const int32_t nx = G.r8_n[0], ny = G.r8_n[1], nz = G.r8_n[2];
  const size_t n = cells8.size();
  h.runs8.assign(n, 0);
  h.run_fraction = 0.0;
  h.dev.runs8 = h.runs8.data();
  if (n == 0 || nx < 3 || ny < 3 || nz < 3) return;
  auto idx = [&](int64_t a, int32_t b, int32_t c) { return ((size_t)a * ny + b) * nz + c; };
  std::vector<int8_t> r(n);
  std::vector<uint32_t> lab(n);
  parallel_for(nx, threads, [&](int64_t b0, int64_t e0) {
    for (size_t q = idx(b0, 0, 0); q < idx(e0, 0, 0); ++q) {
      const int32_t x = cells8[q].x;
      const float m = majorant_of(Cell{cell8_code(x), math::as_f32((uint32_t)cells8[q].y)});
      r[q] = (cell8_interior(x) && m == m) ? 0 : -1;
      lab[q] = math::as_u32(m);
    }
  });
  // erosion pass k: a cell reaches radius k when its 3x3x3 block has radius >= k-1 and one label
  // (separable over z, y, x, as mark_interior)
  std::vector<uint8_t> ez(n), ey(n), grow(n);
  for (int32_t k = 1; k <= 15; ++k) {
    auto ok = [&](size_t q) { return r[q] >= k - 1; };
    parallel_for(nx, threads, [&](int64_t b0, int64_t e0) {
      for (int64_t a = b0; a < e0; ++a)
        for (int32_t b = 0; b < ny; ++b)
          for (int32_t c = 0; c < nz; ++c) {
            const size_t q = idx(a, b, c);
            ez[q] = c > 0 && c + 1 < nz && ok(q - 1) && ok(q) && ok(q + 1) && lab[q - 1] == lab[q] && lab[q + 1] == lab[q];
          }
    });
    parallel_for(nx, threads, [&](int64_t b0, int64_t e0) {
      for (int64_t a = b0; a < e0; ++a)
        for (int32_t b = 0; b < ny; ++b)
          for (int32_t c = 0; c < nz; ++c) {
            const size_t q = idx(a, b, c), s = (size_t)nz;
            ey[q] = b > 0 && b + 1 < ny && ez[q - s] && ez[q] && ez[q + s] && lab[q - s] == lab[q] && lab[q + s] == lab[q];
          }
    });
    std::vector<int64_t> grown_by(nx, 0);
    parallel_for(nx, threads, [&](int64_t b0, int64_t e0) {
      for (int64_t a = b0; a < e0; ++a)
        for (int32_t b = 0; b < ny; ++b)
          for (int32_t c = 0; c < nz; ++c) {
            const size_t q = idx(a, b, c), s = (size_t)ny * nz;
            const bool g = a > 0 && a + 1 < nx && ey[q - s] && ey[q] && ey[q + s] && lab[q - s] == lab[q] && lab[q + s] == lab[q];
            grow[q] = g;
            grown_by[a] += g;
          }
    });
    int64_t grown = 0;
    for (int64_t v : grown_by) grown += v;
    if (!grown) break;
    parallel_for(nx, threads, [&](int64_t b0, int64_t e0) {
      for (size_t q = idx(b0, 0, 0); q < idx(e0, 0, 0); ++q)
        if (grow[q]) r[q] = (int8_t)k;
    });
  }
  int64_t interior = 0, long_runs = 0;
  for (size_t q = 0; q < n; ++q) {
    if (r[q] > 0) h.runs8[q] = (uint8_t)r[q];
    interior += r[q] >= 0;
    long_runs += r[q] >= 2;
  }
  h.run_fraction = interior ? (double)long_runs / (double)interior : 0.0;
}

std::vector<uint8_t> zero_run_radii(const HostGrid& h, int threads) {
  if (threads <= 0) threads = default_threads();
  const DevGrid& G = h.dev;
  const int32_t nx = G.r8_n[0], ny = G.r8_n[1], nz = G.r8_n[2];
  const size_t n = h.cells8.size();
  std::vector<uint8_t> out(n, 0);
  if (n == 0) return out;
  auto idx = [&](int64_t a, int32_t b, int32_t c) { return ((size_t)a * ny + b) * nz + c; };
  // r = -1: not an interior +0 cell; else the radius reached so far
  std::vector<int16_t> r(n);
  parallel_for(nx, threads, [&](int64_t b0, int64_t e0) {
    for (size_t q = idx(b0, 0, 0); q < idx(e0, 0, 0); ++q) {
      const int32_t x = h.cells8[q].x;
      const float m = majorant_of(Cell{cell8_code(x), math::as_f32((uint32_t)h.cells8[q].y)});
      r[q] = (cell8_interior(x) && math::as_u32(m) == 0u) ? 0 : -1;
    }
  });
  // erosion pass k: a cell reaches radius k when its whole 3x3x3 block (inside the table) has
  // radius >= k - 1 (separable over z, y, x)
  std::vector<uint8_t> ez(n), ey(n), grow(n);
  for (int32_t k = 1; k <= (int32_t)kZeroRunMax; ++k) {
    auto ok = [&](size_t q) { return r[q] >= k - 1; };
    parallel_for(nx, threads, [&](int64_t b0, int64_t e0) {
      for (int64_t a = b0; a < e0; ++a)
        for (int32_t b = 0; b < ny; ++b)
          for (int32_t c = 0; c < nz; ++c) {
            const size_t q = idx(a, b, c);
            ez[q] = c > 0 && c + 1 < nz && ok(q - 1) && ok(q) && ok(q + 1);
          }
    });
    parallel_for(nx, threads, [&](int64_t b0, int64_t e0) {
      for (int64_t a = b0; a < e0; ++a)
        for (int32_t b = 0; b < ny; ++b)
          for (int32_t c = 0; c < nz; ++c) {
            const size_t q = idx(a, b, c), s = (size_t)nz;
            ey[q] = b > 0 && b + 1 < ny && ez[q - s] && ez[q] && ez[q + s];
          }
    });
    std::vector<int64_t> grown_by(nx, 0);
    parallel_for(nx, threads, [&](int64_t b0, int64_t e0) {
      for (int64_t a = b0; a < e0; ++a)
        for (int32_t b = 0; b < ny; ++b)
          for (int32_t c = 0; c < nz; ++c) {
            const size_t q = idx(a, b, c), s = (size_t)ny * nz;
            const bool g = a > 0 && a + 1 < nx && ey[q - s] && ey[q] && ey[q + s];
            grow[q] = g;
            grown_by[a] += g;
          }
    });
    int64_t grown = 0;
    for (int64_t v : grown_by) grown += v;
    if (!grown) break;
    parallel_for(nx, threads, [&](int64_t b0, int64_t e0) {
      for (size_t q = idx(b0, 0, 0); q < idx(e0, 0, 0); ++q)
        if (grow[q]) r[q] = (int16_t)k;
    });
  }
  for (size_t q = 0; q < n; ++q) out[q] = r[q] > 0 ? (uint8_t)r[q] : 0;
  return out;
}

void build_walk_table(HostGrid& h, int threads) {
  DevGrid& G = h.dev;
  const int32_t nx = G.r8_n[0], ny = G.r8_n[1], nz = G.r8_n[2];
  for (int a = 0; a < 3; ++a) {
    G.w8_org[a] = G.r8_org[a] - 8 * kWalkPad;
    G.w8_n[a] = G.r8_n[a] + 2 * kWalkPad;
  }
  const size_t n = (size_t)G.w8_n[0] * G.w8_n[1] * G.w8_n[2];
  G.w8_max = (uint32_t)(n - 1);
  h.walk8.assign(n, kWalkSlow);
  const std::vector<uint8_t> zr = VPT_ZERO_RUNS ? zero_run_radii(h, threads) : std::vector<uint8_t>(h.cells8.size(), 0);
  parallel_for((int64_t)nx, threads, [&](int64_t b0, int64_t e0) {
    for (int64_t a = b0; a < e0; ++a)
      for (int32_t b = 0; b < ny; ++b)
        for (int32_t c = 0; c < nz; ++c) {
          const size_t q = ((size_t)a * ny + b) * nz + c;
          const int32_t x = h.cells8[q].x;
          const int32_t code = cell8_code(x);
          if (!cell8_dim8(code)) continue;
          const uint32_t m = math::as_u32(majorant_of(Cell{code, math::as_f32((uint32_t)h.cells8[q].y)}));
          if (m & kWalkEdge) continue;  // a majorant with the sign bit set: general path (same result)
          uint32_t w = m | kWalkEdge;
          if (cell8_interior(x)) {
            if (VPT_ZERO_RUNS && m >= 1u && m <= kZeroRunMax) continue;  // bits that read as a zero run: general path
            w = (VPT_ZERO_RUNS && m == 0u) ? (uint32_t)zr[q] : m;        // +0: the zero-run radius (0 = none)
          }
          h.walk8[((size_t)(a + kWalkPad) * G.w8_n[1] + (b + kWalkPad)) * G.w8_n[2] + (c + kWalkPad)] = w;
        }
  });
  h.dev.walk8 = h.walk8.data();
}

namespace {
// Sets the interior bit (see cell8_interior) of every cells8 entry whose 3x3x3 neighbourhood lies
// in the table and holds only dim-8 cells (leaves: code >= 0; lower-node tiles: -16 / -17).
void mark_interior(const DevGrid& G, std::vector<int2>& cells8, int threads) {
  const int32_t nx = G.r8_n[0], ny = G.r8_n[1], nz = G.r8_n[2];
  if (cells8.empty() || nx < 3 || ny < 3 || nz < 3) return;
  auto at = [&](int32_t a, int32_t b, int32_t c) -> int32_t { return cells8[((size_t)a * ny + b) * nz + c].x; };
  auto dim8 = [](int32_t x) { return cell8_dim8(x); };
  // pass 1: per cell, are the 3 cells along z all dim 8; pass 2 over y, pass 3 over x
  std::vector<uint8_t> d((size_t)nx * ny * nz), ez(d.size()), ey(d.size());
  parallel_for(nx, threads, [&](int64_t b0, int64_t e0) {
    for (int64_t a = b0; a < e0; ++a)
      for (int32_t b = 0; b < ny; ++b)
        for (int32_t c = 0; c < nz; ++c) d[((size_t)a * ny + b) * nz + c] = dim8(at((int32_t)a, b, c));
  });
  auto idx = [&](int64_t a, int32_t b, int32_t c) { return ((size_t)a * ny + b) * nz + c; };
  parallel_for(nx, threads, [&](int64_t b0, int64_t e0) {
    for (int64_t a = b0; a < e0; ++a)
      for (int32_t b = 0; b < ny; ++b)
        for (int32_t c = 1; c + 1 < nz; ++c) ez[idx(a, b, c)] = d[idx(a, b, c - 1)] & d[idx(a, b, c)] & d[idx(a, b, c + 1)];
  });
  parallel_for(nx, threads, [&](int64_t b0, int64_t e0) {
    for (int64_t a = b0; a < e0; ++a)
      for (int32_t b = 1; b + 1 < ny; ++b)
        for (int32_t c = 0; c < nz; ++c) ey[idx(a, b, c)] = ez[idx(a, b - 1, c)] & ez[idx(a, b, c)] & ez[idx(a, b + 1, c)];
  });
  parallel_for(nx, threads, [&](int64_t b0, int64_t e0) {
    for (int64_t a = b0; a < e0; ++a) {
      if (a == 0 || a + 1 == nx) continue;
      for (int32_t b = 0; b < ny; ++b)
        for (int32_t c = 0; c < nz; ++c)
          if (ey[idx(a - 1, b, c)] & ey[idx(a, b, c)] & ey[idx(a + 1, b, c)]) cells8[idx(a, b, c)].x ^= kInteriorBit;
    }
  });
}
}  // namespace

int build_host_grid(const vpt_grid_desc& d, bool fix, int threads, HostGrid& out) {
  if (d.leaf_count && (!d.leaf_origin || !d.leaf_values || !d.leaf_max))
    return set_error(VPT_E_INVALID, "grid: leaf arrays missing");
  if (d.tile_count && (!d.tile_origin || !d.tile_level || !d.tile_value || !d.tile_active))
    return set_error(VPT_E_INVALID, "grid: tile arrays missing");
  if (d.leaf_count > (uint64_t)std::numeric_limits<int32_t>::max())
    return set_error(VPT_E_INVALID, "grid: too many leaves");
  if (threads <= 0) threads = default_threads();
  const uint64_t nleaf = d.leaf_count;

  DevGrid& G = out.dev;
  std::memset(&G, 0, sizeof G);
  std::memcpy(G.mat, d.map_mat, sizeof G.mat);
  std::memcpy(G.inv_mat, d.map_inv_mat, sizeof G.inv_mat);
  std::memcpy(G.vec, d.map_vec, sizeof G.vec);
  G.background = d.background;
  std::memcpy(G.bbox_min, d.index_bbox_min, sizeof G.bbox_min);
  std::memcpy(G.bbox_max, d.index_bbox_max, sizeof G.bbox_max);

  // --- node sets ------------------------------------------------------------------------------
  std::unordered_set<Key3, Key3Hash> lowers, uppers;
  std::unordered_map<Key3, TileVal, Key3Hash> t1, t2, t3;  // tiles by level, keyed by tile origin
  for (uint64_t n = 0; n < nleaf; ++n) {
    const int32_t* o = d.leaf_origin + 3 * n;
    if ((o[0] & 7) || (o[1] & 7) || (o[2] & 7)) return set_error(VPT_E_INVALID, "grid: leaf origin not 8-aligned");
    lowers.insert(Key3{o[0] & ~127, o[1] & ~127, o[2] & ~127});
  }
  for (uint64_t n = 0; n < d.lower_count; ++n) {
    const int32_t* o = d.lower_origin + 3 * n;
    lowers.insert(Key3{o[0] & ~127, o[1] & ~127, o[2] & ~127});
  }
  for (uint64_t n = 0; n < d.tile_count; ++n) {
    const int32_t* o = d.tile_origin + 3 * n;
    int lvl = d.tile_level[n];
    TileVal tv{d.tile_value[n], d.tile_active[n] ? 1 : 0};
    if (lvl == 1) {
      t1[Key3{o[0] & ~7, o[1] & ~7, o[2] & ~7}] = tv;
      lowers.insert(Key3{o[0] & ~127, o[1] & ~127, o[2] & ~127});
    } else if (lvl == 2) {
      t2[Key3{o[0] & ~127, o[1] & ~127, o[2] & ~127}] = tv;
      uppers.insert(Key3{o[0] & ~4095, o[1] & ~4095, o[2] & ~4095});
    } else if (lvl == 3) {
      t3[Key3{o[0] & ~4095, o[1] & ~4095, o[2] & ~4095}] = tv;
    } else {
      return set_error(VPT_E_INVALID, "grid: tile_level must be 1, 2 or 3");
    }
  }
  for (const Key3& l : lowers) uppers.insert(Key3{l.i & ~4095, l.j & ~4095, l.k & ~4095});
  for (uint64_t n = 0; n < d.upper_count; ++n) {
    const int32_t* o = d.upper_origin + 3 * n;
    uppers.insert(Key3{o[0] & ~4095, o[1] & ~4095, o[2] & ~4095});
  }
  for (const Key3& u : uppers) t3.erase(u);  // a root slot holds a child or a value, not both

  // Info for a voxel that is in no lower node: upper-node tile (dim 128) or root (dim 4096).
  auto upper_level = [&](int32_t i, int32_t j, int32_t k) -> int2 {
    Key3 uk{i & ~4095, j & ~4095, k & ~4095};
    if (uppers.count(uk)) {
      auto it = t2.find(Key3{i & ~127, j & ~127, k & ~127});
      if (it != t2.end()) return enc(-(2 * 128 + it->second.active), it->second.value);
      return enc(-(2 * 128), d.background);
    }
    auto it = t3.find(uk);
    if (it != t3.end()) return enc(-(2 * 4096 + it->second.active), it->second.value);
    return enc(-(2 * 4096), d.background);
  };

  // --- cells128 over all upper nodes -----------------------------------------------------------
  if (!uppers.empty()) {
    int32_t lo[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, hi[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
    for (const Key3& u : uppers) {
      const int32_t c[3] = {u.i, u.j, u.k};
      for (int a = 0; a < 3; ++a) {
        lo[a] = std::min(lo[a], c[a]);
        hi[a] = std::max(hi[a], c[a]);
      }
    }
    int64_t cnt = 1;
    for (int a = 0; a < 3; ++a) {
      G.r128_org[a] = lo[a];
      G.r128_n[a] = (int32_t)(((int64_t)hi[a] - lo[a]) / 128 + 32);
      cnt *= G.r128_n[a];
    }
    if (cnt > (int64_t)1 << 31) return set_error(VPT_E_NOMEM, "grid: upper-node table too large");
    out.cells128.resize((size_t)cnt);
    const int32_t ny = G.r128_n[1], nz = G.r128_n[2];
    parallel_for(G.r128_n[0], threads, [&](int64_t b, int64_t e) {
      for (int64_t a = b; a < e; ++a)
        for (int32_t bb = 0; bb < ny; ++bb)
          for (int32_t c = 0; c < nz; ++c)
            out.cells128[((size_t)a * ny + bb) * nz + c] =
                upper_level(G.r128_org[0] + (int32_t)a * 128, G.r128_org[1] + bb * 128, G.r128_org[2] + c * 128);
    });
  }

  // --- cells8 over all lower nodes -------------------------------------------------------------
  if (!lowers.empty()) {
    int32_t lo[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, hi[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
    for (const Key3& l : lowers) {
      const int32_t c[3] = {l.i, l.j, l.k};
      for (int a = 0; a < 3; ++a) {
        lo[a] = std::min(lo[a], c[a]);
        hi[a] = std::max(hi[a], c[a]);
      }
    }
    int64_t cnt = 1;
    int32_t nl[3];
    for (int a = 0; a < 3; ++a) {
      G.r8_org[a] = lo[a];
      nl[a] = (int32_t)(((int64_t)hi[a] - lo[a]) / 128 + 1);
      G.r8_n[a] = nl[a] * 16;
      cnt *= G.r8_n[a];
    }
    if (cnt > (int64_t)1 << 32) return set_error(VPT_E_NOMEM, "grid: leaf-slot table too large");
    // The device indexes the padded walk table and the run radii with 24-bit multiplies
    // ((a * ny + b) * nz + c, math::mul24): the x-y face must stay below 2^24 cells and the table
    // below 2^32 entries, or the device index would silently diverge from the host's.
    const int64_t wx = G.r8_n[0] + 2 * kWalkPad, wy = G.r8_n[1] + 2 * kWalkPad, wz = G.r8_n[2] + 2 * kWalkPad;
    if (wx * wy >= ((int64_t)1 << 24) || wx * wy * wz > ((int64_t)1 << 32))
      return set_error(VPT_E_INVALID, "grid: lower-node extent too large for the 24-bit walk-table index (x*y face >= 2^24 cells)");
    out.cells8.resize((size_t)cnt);
    std::vector<uint8_t> lower_present((size_t)nl[0] * nl[1] * nl[2], 0);
    for (const Key3& l : lowers)
      lower_present[((size_t)((l.i - lo[0]) / 128) * nl[1] + (l.j - lo[1]) / 128) * nl[2] + (l.k - lo[2]) / 128] = 1;
    const int32_t ny = G.r8_n[1], nz = G.r8_n[2];
    parallel_for(G.r8_n[0], threads, [&](int64_t b, int64_t e) {
      for (int64_t a = b; a < e; ++a)
        for (int32_t bb = 0; bb < ny; ++bb)
          for (int32_t c = 0; c < nz; ++c) {
            int32_t i = G.r8_org[0] + (int32_t)a * 8, j = G.r8_org[1] + bb * 8, k = G.r8_org[2] + c * 8;
            int2 v;
            if (lower_present[((size_t)(a >> 4) * nl[1] + (bb >> 4)) * nl[2] + (c >> 4)]) {
              auto it = t1.find(Key3{i, j, k});
              v = (it != t1.end()) ? enc(-(2 * 8 + it->second.active), it->second.value) : enc(-(2 * 8), d.background);
            } else {
              v = upper_level(i, j, k);
            }
            out.cells8[((size_t)a * ny + bb) * nz + c] = v;
          }
    });
    for (uint64_t n = 0; n < nleaf; ++n) {
      const int32_t* o = d.leaf_origin + 3 * n;
      size_t idx = ((size_t)((o[0] - lo[0]) >> 3) * ny + ((o[1] - lo[1]) >> 3)) * nz + ((o[2] - lo[2]) >> 3);
      out.cells8[idx] = enc((int32_t)n, d.leaf_max[n]);
    }
  }

  for (const auto& kv : t3) {
    RootTileDev r{};
    r.origin[0] = kv.first.i;
    r.origin[1] = kv.first.j;
    r.origin[2] = kv.first.k;
    r.value = kv.second.value;
    r.active = kv.second.active;
    out.root.push_back(r);
  }
  G.root_count = (int32_t)out.root.size();
  G.leaf_count = (int32_t)nleaf;
  G.cells8 = out.cells8.data();
  G.cells128 = out.cells128.data();
  G.root = out.root.data();

  // --- bricks: 8^3 leaf voxels + the +1 apron ------------------------------------------------
  // 9^3 apron bricks first (expanded into stencils below); every element is written below (interior, then apron)
  out.bricks.resize((size_t)nleaf * 729);
  G.bricks = out.bricks.data();
  // interior first (the apron reads neighbours' interiors through value_at)
  parallel_for((int64_t)nleaf, threads, [&](int64_t b, int64_t e) {
    for (int64_t n = b; n < e; ++n) {
      const float* src = d.leaf_values + (size_t)n * 512;
      float* dst = out.bricks.data() + (size_t)n * 729;
      for (int x = 0; x < 8; ++x)
        for (int y = 0; y < 8; ++y)
          for (int z = 0; z < 8; ++z) dst[x * 81 + y * 9 + z] = src[(x << 6) | (y << 3) | z];
    }
  });
  // getValue over the interiors written so far (apron layout)
  auto apron_value_at = [&](int32_t i, int32_t j, int32_t k) -> float {
    const Cell c = cell_at(G, i, j, k);
    if (c.code < 0) return c.value;
    return out.bricks[(size_t)c.code * 729 + (i & 7) * 81 + (j & 7) * 9 + (k & 7)];
  };
  parallel_for((int64_t)nleaf, threads, [&](int64_t b, int64_t e) {
    for (int64_t n = b; n < e; ++n) {
      const int32_t* o = d.leaf_origin + 3 * n;
      float* dst = out.bricks.data() + (size_t)n * 729;
      for (int x = 0; x < 9; ++x)
        for (int y = 0; y < 9; ++y)
          for (int z = 0; z < 9; ++z)
            if (x == 8 || y == 8 || z == 8) dst[x * 81 + y * 9 + z] = apron_value_at(o[0] + x, o[1] + y, o[2] + z);
    }
  });

  {
    // expand the apron bricks into square rows (per row (y, z) the 2x2 squares of x = 0..8)
    std::vector<float, NoInitAllocator<float>> apron;
    apron.swap(out.bricks);
    out.bricks.resize((size_t)nleaf * kBrickVox);  // (every square of every row is written below)
    parallel_for((int64_t)nleaf, threads, [&](int64_t b, int64_t e) {
      for (int64_t n = b; n < e; ++n) {
        const float* src = apron.data() + (size_t)n * 729;
        float* dst = out.bricks.data() + (size_t)n * kBrickVox;
        for (int x = 0; x < 9; ++x)
          for (int y = 0; y < 8; ++y)
            for (int z = 0; z < 8; ++z)
              for (int q = 0; q < 4; ++q)
                dst[((y * 8 + z) * 9 + x) * 4 + q] = src[x * 81 + (y + (q >> 1)) * 9 + z + (q & 1)];
      }
    });
    G.bricks = out.bricks.data();
  }
  // --- majorants -------------------------------------------------------------------------------
  out.leaf_max.assign(d.leaf_max, d.leaf_max + nleaf);
  if (fix) {
    parallel_for((int64_t)nleaf, threads, [&](int64_t b, int64_t e) {
      for (int64_t n = b; n < e; ++n) {
        const int32_t* o = d.leaf_origin + 3 * n;
        float m = d.leaf_max[n];
        // The 26 neighbour leaf boxes intersected with the leaf bbox expanded by 1 = the one-voxel
        // shell around the leaf; std::max keeps the first argument on ties/NaN like the reference.
        for (int32_t x = o[0] - 1; x <= o[0] + 8; ++x)
          for (int32_t y = o[1] - 1; y <= o[1] + 8; ++y)
            for (int32_t z = o[2] - 1; z <= o[2] + 8; ++z) {
              bool inside = x >= o[0] && x <= o[0] + 7 && y >= o[1] && y <= o[1] + 7 && z >= o[2] && z <= o[2] + 7;
              if (inside) continue;
              float v = value_at(G, x, y, z);
              m = std::max(m, v);
            }
        out.leaf_max[n] = m;
      }
    });
    for (uint64_t n = 0; n < nleaf; ++n) {
      const int32_t* o = d.leaf_origin + 3 * n;
      size_t idx = ((size_t)((o[0] - G.r8_org[0]) >> 3) * G.r8_n[1] + ((o[1] - G.r8_org[1]) >> 3)) * G.r8_n[2] +
                   ((o[2] - G.r8_org[2]) >> 3);
      out.cells8[idx] = enc((int32_t)n, out.leaf_max[n]);
    }
  }
  mark_interior(G, out.cells8, threads);
  build_walk_table(out, threads);
  return VPT_OK;
}

// The extremes of a grid's values, the leaf voxels scanned in parallel (blackbody_rows_suffice reads them: the
// temperature grid's 46 M voxels took ~30 ms on one thread inside the context's creation).
ValueRange value_range(const vpt_grid_desc& t, int threads) {
  if (threads <= 0) threads = default_threads();
  ValueRange r;
  r.lo = r.hi = t.background;
  r.finite = std::isfinite(t.background);
  auto take = [](ValueRange& q, float v) {
    q.lo = std::min(q.lo, v);
    q.hi = std::max(q.hi, v);
    q.finite = q.finite && std::isfinite(v);
  };
  for (uint64_t i = 0; i < t.tile_count; ++i) take(r, t.tile_value[i]);
  std::mutex m;
  parallel_for((int64_t)t.leaf_count, threads, [&](int64_t b, int64_t e) {
    ValueRange q = r;
    for (uint64_t i = (uint64_t)b * 512; i < (uint64_t)e * 512; ++i) take(q, t.leaf_values[i]);
    std::lock_guard<std::mutex> lk(m);
    r.lo = std::min(r.lo, q.lo);
    r.hi = std::max(r.hi, q.hi);
    r.finite = r.finite && q.finite;
  });
  return r;
}

// ------------------------------------------------------------------------------------------------
// Synthetic stand-in volumes: the real wdas_cloud.nvdb / fire.nvdb are not available.
// ------------------------------------------------------------------------------------------------
namespace {

double synth_voxel(int kind, int n, int i, int j, int k) {
  if (kind == 0) return 1.0;
  const double half = n / 2.0;
  const double px = (i + 0.5) / half - 1.0, py = (j + 0.5) / half - 1.0, pz = (k + 0.5) / half - 1.0;
  const double r = std::sqrt(px * px + py * py + pz * pz);
  const double base = std::min(1.0, std::max(0.0, (0.85 - r) / 0.35));
  if (kind == 2) return 40.0 * base;
  return base * (0.5 + 0.5 * std::sin(11.0 * px + 2.0) * std::sin(13.0 * py + 1.0) * std::sin(17.0 * pz + 3.0));
}
}  // namespace

}  // namespace vpt

extern "C" int vpt_fix_majorants(const vpt_grid_desc* grid, float* out_leaf_max, int num_threads) {
  if (!grid || !out_leaf_max) return vpt::set_error(VPT_E_INVALID, "vpt_fix_majorants: null argument");
  vpt::HostGrid hg;
  int rc = vpt::build_host_grid(*grid, true, num_threads, hg);
  if (rc) return rc;
  std::copy(hg.leaf_max.begin(), hg.leaf_max.end(), out_leaf_max);
  return VPT_OK;
}

// kind 0: constant 1.0 over [0,n)^3 (C2); kind 1: procedural cloud density (C3);
// kind 2: temperature 40*base on the same lattice (C4).  world = index - n/2, voxel size 1.
// Leaves with no non-zero voxel are omitted; non-zero voxels are active; indexBBox = active bbox;
// leaf max = max over active voxels (NanoVDB's stored statistic).
extern "C" vpt_grid_desc* vpt_synth_grid(int kind, int n) {
  if (n <= 0 || (n % 8) != 0 || kind < 0 || kind > 2) {
    vpt::set_error(VPT_E_INVALID, "vpt_synth_grid: kind in {0,1,2}, n a positive multiple of 8");
    return nullptr;
  }
  auto* s = vpt::owned_grid_new();
  const int nl = n / 8;
  const int T = vpt::default_threads();
  struct Part {
    std::vector<int32_t> origin;
    std::vector<float> values, maxv;
    std::vector<uint64_t> mask;
    int32_t lo[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, hi[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
  };
  std::vector<Part> parts(nl);
  vpt::parallel_for(nl, T, [&](int64_t b, int64_t e) {
    std::vector<float> buf(512);
    for (int64_t li = b; li < e; ++li) {
      Part& P = parts[li];
      for (int lj = 0; lj < nl; ++lj)
        for (int lk = 0; lk < nl; ++lk) {
          bool any = false;
          float mx = -std::numeric_limits<float>::infinity();
          uint64_t mask[8] = {0, 0, 0, 0, 0, 0, 0, 0};
          for (int a = 0; a < 8; ++a)
            for (int bb = 0; bb < 8; ++bb)
              for (int c = 0; c < 8; ++c) {
                const int i = (int)li * 8 + a, j = lj * 8 + bb, k = lk * 8 + c;
                float v = (float)vpt::synth_voxel(kind, n, i, j, k);
                int off = (a << 6) | (bb << 3) | c;
                buf[off] = v;
                if (v != 0.0f) {
                  any = true;
                  mask[off >> 6] |= 1ULL << (off & 63);
                  mx = std::max(mx, v);
                  const int32_t cc[3] = {i, j, k};
                  for (int q = 0; q < 3; ++q) {
                    P.lo[q] = std::min(P.lo[q], cc[q]);
                    P.hi[q] = std::max(P.hi[q], cc[q]);
                  }
                }
              }
          if (!any) continue;
          P.origin.insert(P.origin.end(), {(int32_t)li * 8, lj * 8, lk * 8});
          P.values.insert(P.values.end(), buf.begin(), buf.end());
          P.mask.insert(P.mask.end(), mask, mask + 8);
          P.maxv.push_back(mx);
        }
    }
  });
  int32_t lo[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, hi[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
  for (auto& P : parts) {
    s->leaf_origin.insert(s->leaf_origin.end(), P.origin.begin(), P.origin.end());
    s->leaf_values.insert(s->leaf_values.end(), P.values.begin(), P.values.end());
    s->leaf_mask.insert(s->leaf_mask.end(), P.mask.begin(), P.mask.end());
    s->leaf_max.insert(s->leaf_max.end(), P.maxv.begin(), P.maxv.end());
    for (int q = 0; q < 3; ++q) {
      lo[q] = std::min(lo[q], P.lo[q]);
      hi[q] = std::max(hi[q], P.hi[q]);
    }
  }
  vpt_grid_desc& d = s->d;
  const float half = (float)(n / 2);
  for (int a = 0; a < 9; ++a) d.map_mat[a] = d.map_inv_mat[a] = (a % 4 == 0) ? 1.0f : 0.0f;
  for (int q = 0; q < 3; ++q) {
    d.map_vec[q] = -half;
    d.index_bbox_min[q] = lo[q];
    d.index_bbox_max[q] = hi[q];
  }
  d.background = 0.0f;
  s->finish();
  return &s->d;
}

extern "C" void vpt_synth_free(vpt_grid_desc* d) { delete reinterpret_cast<vpt::OwnedGrid*>(d); }
