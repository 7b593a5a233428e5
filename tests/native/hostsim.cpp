// hostsim.cpp — TEST HARNESS: runs the device integrator state machine (vpt_integrator.h)
// serially on the CPU so that its control flow and float semantics can be checked bit-for-bit
// against the oracle without a GPU.  Not part of the product library; the product path is the
// HIP kernel in volume_path_tracer_amd/csrc/vpt_gpu.hip.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../volume_path_tracer_amd/csrc/vpt_internal.h"

namespace vpt {
static thread_local std::string g_err;
int set_error(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
}  // namespace vpt

namespace {
// Runs variant (run skipping) of the density-only path: -1 = the GPU's rule (run_fraction >= 1/4,
// vpt_gpu.hip), 0 / 1 = forced (vpths_set_runs).
int g_runs = -1;
// Throughput mode's pixels per work item (vpt_gpu_set_pixel_chunk; vpths_set_pixel_chunk).
uint32_t g_pixel_chunk = 1;
struct HostEnv {
  uint64_t jid_begin, jid_count, next = 0;
  float* film;
  float* records;
  int32_t tile_area;
  uint32_t pixel_chunk = 1;
  const uint32_t* order = nullptr;  // job order (see vpt_integrator.h ST_FETCH)
  const uint32_t* perm = nullptr;   // explicit job order (vpt_gpu_set_job_permutation)
  uint32_t order_tail_k0 = 0;
  uint32_t order_tail_n = 0;
  uint32_t order_group = vpt::kOrderGroup;
  const HostEnv* args() const { return this; }  // (the kernel reads its launch arguments through args())
  int32_t count(bool pred) { return pred ? 1 : 0; }  // one lane
  vpt::LaneCold cold_{};
  vpt::LaneCold& cold() { return cold_; }
  uint64_t cnt[vpt::CNT_COUNT] = {};
  void tally(int32_t k, int32_t w) { cnt[k] += (uint64_t)w; }
  void prof(int32_t) {}
  void prof_add(int32_t, int32_t) {}
  void tick(int32_t) {}
  void event(vpt::Lane&, uint32_t, const float*, const float*, float) {}
  bool fetch_urgent(bool) const { return false; }  // (no feeds on the host)
  bool fetch_job(uint64_t& j, int32_t /*wave_lanes: the GPU's job spreading*/) {
    if (next >= jid_count) return false;
    j = next++;
    return true;
  }
  void job_end(const vpt::DevScene&, const vpt::LaneCold&) {}  // (staged feeds' per-tile job counts: GPU only)
  void job_start(const vpt::DevScene&, vpt::LaneCold&, uint64_t) {}  // (feeds' ordered frames: GPU only)
  const double (*logf_table() const)[2] { return vpt::math::kLogfTab; }
  void blackbody(const vpt::DevScene& S, float t, float& X, float& Y, float& Z) const {
    if (S.bb_lds_ok) {  // the kernel's LDS path: only the first kBbLdsRows rows (NaN beyond, so a
                        // lookup past them would show in the parity tests)
      std::vector<float> rows(501 * 3, __builtin_nanf(""));
      std::copy(S.bb, S.bb + vpt::kBbLdsRows * 3, rows.begin());
      vpt::blackbody_xyz(S, rows.data(), t, X, Y, Z);
    } else {
      vpt::blackbody_xyz(S, S.bb, t, X, Y, Z);
    }
  }
  void film_commit(const vpt::DevScene&, bool) {}  // (one lane: film_add adds directly)
  void film_add(const vpt::DevScene& S, const vpt::Lane& ln, int32_t px, int32_t py, int32_t rw) {
    float* f = film + ((int64_t)py * S.W + px) * 4;
    f[3] += 1.0f;
    const vpt::LaneCold& lc = cold_;
    f[0] += S.imaging_ratio * lc.L[0];
    f[1] += S.imaging_ratio * lc.L[1];
    f[2] += S.imaging_ratio * lc.L[2];
    if (records) {
      int32_t xl = px - lc.x0, yl = py - lc.y0;
      float* r = records + (ln.jid_local * (uint64_t)tile_area + (uint64_t)(yl * rw + xl)) * 3;
      r[0] = lc.L[0];
      r[1] = lc.L[1];
      r[2] = lc.L[2];
    }
  }
};
}  // namespace

// order != nullptr: [jid_begin, jid_begin + jid_count) is whole waves and items are taken in the
// kernel's cost order (order = tile ranks; the last tail_waves waves tile-major, see ordered_job; tail_waves < 0:
// the same-tile order).
extern "C" int vpths_render_jobs_order(const vpt_configuration* cfg, const vpt_grid_desc* density,
                                       const vpt_grid_desc* temperature, const float* bb500, uint64_t jid_begin,
                                       uint64_t jid_count, float* film, float* records, vpt_counters* counters,
                                       int rng_mode, const uint32_t* order, int tail_waves) {
  vpt::DevScene S{};
  int rc = vpt::build_scene(*cfg, S);
  if (rc) return rc;
  vpt::HostGrid hd, ht;
  if ((rc = vpt::build_host_grid(*density, true, 0, hd))) return rc;
  vpt::compute_runs(hd, 0);
  const bool runs = g_runs < 0 ? hd.run_fraction >= 0.25 : g_runs != 0;
  S.density = hd.dev;
  vpt::scene_finalize(S);
  if (temperature) {
    if ((rc = vpt::build_host_grid(*temperature, false, 0, ht))) return rc;
    S.temperature = ht.dev;
    S.has_temperature = 1;
    S.bb_lds_ok = vpt::blackbody_rows_suffice(vpt::value_range(*temperature, 0), cfg->volume_parameters.temperature_scale,
                                              cfg->volume_parameters.temperature_offset, vpt::kBbLdsRows);
  }
  std::vector<float> bb(501 * 3, 0.0f);
  if (bb500)
    std::memcpy(bb.data(), bb500, 500 * 3 * sizeof(float));
  else
    vpt::blackbody_table(bb.data());
  S.bb = bb.data();
  S.cie = vpt::cie_table();
  S.gate_min = 1;
  S.gate_idle = 1;
  S.gate_eval = 1;
  S.gate_walk = 1;  // exercise the inner walk loop
  S.pixel_mode = rng_mode == VPT_RNG_PIXEL ? 1 : 0;
  S.tile_area = (uint32_t)(S.tw * S.th);
  if (S.pixel_mode && S.tile_area % g_pixel_chunk != 0) return VPT_E_INVALID;
  HostEnv env{jid_begin, S.pixel_mode ? jid_count * S.tile_area / g_pixel_chunk : jid_count, 0, film, records, S.tw * S.th,
              S.pixel_mode ? g_pixel_chunk : 1u};
  if (order) {
    env.order = order;
    if (tail_waves < 0) {  // VPT_ORDER_COST_SAME_TILE: every wave tile-major, one tile per group
      tail_waves = (int)(jid_count / S.T);
      env.order_group = 1;
    }
    env.order_tail_n = (uint32_t)tail_waves;
    env.order_tail_k0 = (uint32_t)(jid_count - (uint64_t)tail_waves * S.T);
  }
  vpt::Lane ln;
  std::memset(&ln, 0, sizeof ln);
  vpt::lane_init(ln);
  vpt::cold_init(env.cold());
  if (temperature)
    while (ln.state != vpt::ST_DONE) vpt::lane_iteration<true, true, false>(&S, ln, env);
  else
    while (ln.state != vpt::ST_DONE) {
      if (runs)
        vpt::lane_iteration<false, true, true>(&S, ln, env);
      else
        vpt::lane_iteration<false, true, false>(&S, ln, env);
    }
  env.cnt[vpt::CNT_DDA_STEPS] += ln.n_dda;
  if (counters) {
    uint64_t* o = reinterpret_cast<uint64_t*>(counters);
    for (int k = 0; k < vpt::CNT_COUNT; ++k) o[k] += env.cnt[k];
  }
  return 0;
}

extern "C" int vpths_render_jobs_mode(const vpt_configuration* cfg, const vpt_grid_desc* density,
                                      const vpt_grid_desc* temperature, const float* bb500, uint64_t jid_begin,
                                      uint64_t jid_count, float* film, float* records, vpt_counters* counters,
                                      int rng_mode) {
  return vpths_render_jobs_order(cfg, density, temperature, bb500, jid_begin, jid_count, film, records, counters,
                                 rng_mode, nullptr, 0);
}

extern "C" int vpths_render_jobs(const vpt_configuration* cfg, const vpt_grid_desc* density,
                                 const vpt_grid_desc* temperature, const float* bb500, uint64_t jid_begin,
                                 uint64_t jid_count, float* film, float* records, vpt_counters* counters) {
  return vpths_render_jobs_mode(cfg, density, temperature, bb500, jid_begin, jid_count, film, records, counters,
                                VPT_RNG_REFERENCE);
}

// Leaf majorants after fix_majorants (product builder), for comparison with the oracle.
extern "C" int vpths_fixed_leaf_max(const vpt_grid_desc* d, float* out) {
  vpt::HostGrid h;
  int rc = vpt::build_host_grid(*d, true, 0, h);
  if (rc) return rc;
  std::memcpy(out, h.leaf_max.data(), h.leaf_max.size() * sizeof(float));
  return 0;
}

// getValue / max(8,getDim) / majorant through the product's flattened tables.
extern "C" int vpths_probe(const vpt_grid_desc* d, const int32_t* ijk, int n, float* value, int32_t* dim, float* maj) {
  vpt::HostGrid h;
  int rc = vpt::build_host_grid(*d, true, 0, h);
  if (rc) return rc;
  for (int q = 0; q < n; ++q) {
    vpt::Cell c = vpt::cell_at(h.dev, ijk[3 * q], ijk[3 * q + 1], ijk[3 * q + 2]);
    value[q] = vpt::value_at(h.dev, ijk[3 * q], ijk[3 * q + 1], ijk[3 * q + 2]);
    dim[q] = vpt::hdda_dim_of(c);
    maj[q] = vpt::majorant_of(c);
  }
  return 0;
}

// The HDDA walk table (build_walk_table) checked by brute force through cell_at: an interior word
// (sign bit clear) needs all 27 cells of its neighbourhood at HDDA dim 8 and holds the cell's
// majorant bits; an edge word (kWalkEdge set) needs the cell itself at dim 8 and holds its majorant
// bits | kWalkEdge; every dim-8 cell of the r8 table whose majorant has the sign bit clear is one of
// the two (but interior cells whose majorant bits are 1..kZeroRunMax, which are slow); the padding is
// kWalkSlow.  A +0 interior cell holds its zero-run radius r: r = 0 is checked as an interior +0 cell,
// r >= 1 by induction -- each of its 26 neighbours holds a zero-run word of radius >= r - 1 (the ball
// of radius r is the union of the neighbours' balls of radius r - 1).
// counts = {interior, edge, slow, padding, zero-run words with r >= 1}; returns violations.
extern "C" int64_t vpths_check_walk(const vpt_grid_desc* d, int64_t* counts) {
  vpt::HostGrid h;
  if (vpt::build_host_grid(*d, true, 0, h)) return -1;
  const vpt::DevGrid& G = h.dev;
  auto bits = [](float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; };
  auto word = [&](int32_t a, int32_t b, int32_t c) { return h.walk8[((size_t)a * G.w8_n[1] + b) * G.w8_n[2] + c]; };
  int64_t bad = 0;
  for (int k = 0; k < 5; ++k) counts[k] = 0;
  for (int32_t a = 0; a < G.w8_n[0]; ++a)
    for (int32_t b = 0; b < G.w8_n[1]; ++b)
      for (int32_t c = 0; c < G.w8_n[2]; ++c) {
        const uint32_t w = word(a, b, c);
        const int32_t o[3] = {G.w8_org[0] + 8 * a, G.w8_org[1] + 8 * b, G.w8_org[2] + 8 * c};
        const bool in_r8 = a >= vpt::kWalkPad && a < vpt::kWalkPad + G.r8_n[0] && b >= vpt::kWalkPad &&
                           b < vpt::kWalkPad + G.r8_n[1] && c >= vpt::kWalkPad && c < vpt::kWalkPad + G.r8_n[2];
        if (!in_r8) {
          ++counts[3];
          bad += w != vpt::kWalkSlow;
          continue;
        }
        const vpt::Cell C = vpt::cell_at(G, o[0], o[1], o[2]);
        const uint32_t m = bits(vpt::majorant_of(C));
        const bool dim8 = vpt::hdda_dim_of(C) == 8;
        bool all8 = true;
        for (int da = -1; da <= 1; ++da)
          for (int db = -1; db <= 1; ++db)
            for (int dc = -1; dc <= 1; ++dc)
              all8 = all8 && vpt::hdda_dim_of(vpt::cell_at(G, o[0] + 8 * da, o[1] + 8 * db, o[2] + 8 * dc)) == 8;
        if (w == vpt::kWalkSlow) {
          ++counts[2];
          const bool tiny = all8 && m >= 1u && m <= vpt::kZeroRunMax;
          bad += dim8 && !(m & vpt::kWalkEdge) && m != vpt::kWalkSlow && !tiny;  // a fast cell left slow
          continue;
        }
        if (w & vpt::kWalkEdge) {
          ++counts[1];
          bad += !dim8 || (m & vpt::kWalkEdge) || (w & ~vpt::kWalkEdge) != m;
          continue;
        }
        ++counts[0];
        if (w > vpt::kZeroRunMax) {
          bad += !all8 || w != m;
          continue;
        }
        bad += !all8 || m != 0u;  // a zero-run word: an interior +0 cell
        if (w == 0) continue;
        ++counts[4];
        for (int da = -1; da <= 1; ++da)
          for (int db = -1; db <= 1; ++db)
            for (int dc = -1; dc <= 1; ++dc) {
              const uint32_t nw = word(a + da, b + db, c + dc);  // in the padded table: all8 above
              bad += !(nw <= vpt::kZeroRunMax && nw + 1u >= w);
            }
      }
  return bad;
}

extern "C" void vpths_set_runs(int on) { g_runs = on; }
extern "C" void vpths_set_pixel_chunk(int chunk) { g_pixel_chunk = (uint32_t)chunk; }

// Walk-word loads issued and walk words synthesised from zero runs since the last reset.
extern "C" void vpths_walk_loads(uint64_t* loads, uint64_t* synth, int reset) {
  *loads = vpt::g_walk_loads;
  *synth = vpt::g_walk_synth;
  if (reset) vpt::g_walk_loads = vpt::g_walk_synth = 0;
}

// Run radii (vpt::compute_runs) checked by brute force: every cell within Chebyshev distance r of a
// cell with radius r is in the table, interior, and has the same majorant bits.  hist[r] = cells
// with radius r (r = 0..15); *fraction = HostGrid::run_fraction; returns the violations.
extern "C" int64_t vpths_check_runs(const vpt_grid_desc* d, int64_t* hist, double* fraction) {
  vpt::HostGrid h;
  if (vpt::build_host_grid(*d, true, 0, h)) return -1;
  vpt::compute_runs(h, 0);
  *fraction = h.run_fraction;
  const vpt::DevGrid& G = h.dev;
  const int64_t nx = G.r8_n[0], ny = G.r8_n[1], nz = G.r8_n[2];
  auto at = [&](int64_t a, int64_t b, int64_t c) { return ((size_t)a * ny + b) * nz + c; };
  auto maj_bits = [&](size_t q) {
    float v;
    std::memcpy(&v, &h.cells8[q].y, 4);
    const float m = vpt::majorant_of(vpt::Cell{vpt::cell8_code(h.cells8[q].x), v});
    uint32_t u;
    std::memcpy(&u, &m, 4);
    return u;
  };
  int64_t bad = 0;
  for (int r = 0; r <= 15; ++r) hist[r] = 0;
  if (h.runs8.size() != h.cells8.size()) return -2;
  for (int64_t a = 0; a < nx; ++a)
    for (int64_t b = 0; b < ny; ++b)
      for (int64_t c = 0; c < nz; ++c) {
        const size_t q = at(a, b, c);
        const int r = h.runs8[q];
        if (r > 15) return -3;
        ++hist[r];
        for (int64_t x = a - r; x <= a + r && r > 0; ++x)
          for (int64_t y = b - r; y <= b + r; ++y)
            for (int64_t z = c - r; z <= c + r; ++z) {
              if (x < 0 || y < 0 || z < 0 || x >= nx || y >= ny || z >= nz) {
                ++bad;
                continue;
              }
              const size_t f = at(x, y, z);
              if (!vpt::cell8_interior(h.cells8[f].x) || maj_bits(f) != maj_bits(q)) ++bad;
            }
      }
  return bad;
}

// The math clones vs glibc, over every input the integrator can produce.
#include <cmath>
extern "C" int64_t vpths_math_mismatches(int which) {
  int64_t bad = 0;
  for (uint32_t b = 0;; ++b) {
    float fr;
    std::memcpy(&fr, &b, 4);
    if (fr > 4294967296.0f) break;
    if (fr != std::floor(fr)) continue;
    float u = fr * 0x1p-32f;
    if (!(u < 0x1.fffffep-1f)) u = 0x1.fffffep-1f;
    if (which == 0) {
      float x = 1.0f - u;
      if (vpt::math::as_u32(vpt::math::logf_glibc(x)) != vpt::math::as_u32(std::log(x))) ++bad;
      if (vpt::math::as_u32(vpt::math::logf_glibc_unit(x)) != vpt::math::as_u32(std::log(x))) ++bad;
    } else {
      float phi = 2.0f * 3.14159274f * u;
      if (which == 1 && vpt::math::as_u32(vpt::math::sinf_glibc(phi)) != vpt::math::as_u32(std::sin(phi))) ++bad;
      if (which == 2 && vpt::math::as_u32(vpt::math::cosf_glibc(phi)) != vpt::math::as_u32(std::cos(phi))) ++bad;
      if (which == 3) {  // the fused clone the HG sampler calls
        float sn, cs;
        vpt::math::sincosf_glibc(phi, sn, cs);
        if (vpt::math::as_u32(sn) != vpt::math::as_u32(std::sin(phi))) ++bad;
        if (vpt::math::as_u32(cs) != vpt::math::as_u32(std::cos(phi))) ++bad;
      }
    }
  }
  return bad;
}

// powf(x, 2.0f) == x * x for every finite float (the device squares instead of calling pow).
extern "C" int64_t vpths_pow2_mismatches(void) {
  int64_t bad = 0;
  for (uint64_t b = 0; b < (1ULL << 32); b += 1) {
    uint32_t u = (uint32_t)b;
    float x;
    std::memcpy(&x, &u, 4);
    if (!std::isfinite(x)) continue;
    float p = std::pow(x, 2.0f), q = x * x;
    if (vpt::math::as_u32(p) != vpt::math::as_u32(q)) ++bad;
  }
  return bad;
}

// Walk-table lookups outside the padded table since the last reset (vpt_integrator.h walk_index):
// the padding argument of hdda_pre_advance says there are none.
extern "C" uint64_t vpths_walk_outside(int reset) {
  const uint64_t n = vpt::g_walk_outside;
  if (reset) vpt::g_walk_outside = 0;
  return n;
}
