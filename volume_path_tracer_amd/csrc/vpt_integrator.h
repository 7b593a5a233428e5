// vpt_integrator.h — the per-lane volumetric path-tracing state machine (device code).
//
// One lane owns one (tile, wave) job at a time and traces the tile's pixels serially in the job's
// pcg32_fast stream, exactly as vpt::run does on one CPU thread (src/worker.cpp:104-207): the RNG
// stream order forbids tracing a tile's pixels concurrently.  The nested loops of the reference
//   run -> per pixel -> per bounce -> MajorantTransmittanceSampler::next -> RayMajorantIterator::next
// (worker.cpp:130-195, majorant_transmittance_sampler.cpp:21-81, volume.cpp:38-76)
// are flattened into one state machine whose unit of work is ONE HDDA step or ONE free-flight draw,
// so the 64 lanes of a wavefront advance together no matter how different their paths are, and a
// lane whose job ends picks the next job (persistent kernel, lane refill).
//
// Every floating-point operation is the reference's, in the reference's order (built with
// -ffp-contract=off): Eigen 3-vector reductions as x0 + (x1 + x2), NanoVDB Map products with fmaf,
// NanoVDB Vec3::length as (x*x + y*y) + z*z, glibc logf/sinf/cosf via vpt_math.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vpt_math.h"

namespace vpt {

// ------------------------------------------------------------------------------------------------
// HBM layout of one grid (built by vpt_grid_build.cpp)
// ------------------------------------------------------------------------------------------------
// Cell code: >= 0 -> leaf index (value = leaf majorant after fix_majorants_for_interpolation);
//            <  0 -> no leaf: -(2*dim + active), dim = ReadAccessor::getDim (8 lower tile,
//                    128 upper tile, 4096 root tile / background), value = tile value.
struct RootTileDev {
  int32_t origin[3];
  float value;
  int32_t active;
  int32_t pad[3];
};

struct DevGrid {
  float mat[9], inv_mat[9], vec[3];  // nanovdb::Map float members
  float background;
  int32_t bbox_min[3], bbox_max[3];  // indexBBox (inclusive)
  int32_t r8_org[3], r8_n[3];        // dense 8^3-cell table over all lower nodes
  int32_t w8_org[3], w8_n[3];        // walk8: the r8 table padded by kWalkPad cells on every side
  uint32_t w8_max;                   // last walk8 index
  int32_t r128_org[3], r128_n[3];    // dense 128^3-cell table over all upper nodes
  int32_t root_count, leaf_count;
  const int2* cells8;
  const uint8_t* runs8;  // per cells8 entry: run radius (see mark_runs), for the Runs kernel variant
  const uint32_t* walk8; // per (padded) cells8 entry: the majorant's bits if the cell is interior, else kWalkSlow
  const int2* cells128;
  const RootTileDev* root;
  const float* bricks;  // [leaf][y 8][z 8][x 9][4]: per voxel row the 2x2 squares of its stencils (see brick_index)
};

// Stencil pool of square rows: per leaf and voxel row (y, z) in 0..7, the 2x2 (dy, dz) squares of
// x = 0..8 (x = 8 crossing into the +x neighbour, y + 1 / z + 1 into the +y / +z ones), 4 floats =
// 16 B each, corner order dy<<1 | dz.  The stencil of voxel (x, y, z) is the squares of x and x + 1:
// 32 contiguous bytes, corner q = dx<<2 | dy<<1 | dz, two 16-byte loads from one 128-B line, or from
// two when the pair straddles a line boundary (1 pair in 8).  The pool is 4.5x the 8^3 voxels (9 KiB
// per leaf: 0.84 GB for the 512^3 stand-in).  History: r01's 9^3 apron bricks spread a stencil over up
// to 4 lines; r02's stencil-major pool (8 floats per voxel, 8x the voxels, 1.49 GB) kept it in one
// line; the square rows (r03) keep 7 of 8 stencils in one line, store each line's x-neighbours twice as
// densely and cut the pool by 44 %: C3 359.5 -> 352.6 ms, C4 102.6 -> 99.7 ms (two rounds, one box).
constexpr int kBrickVox = 576 * 4;
__host__ __device__ __forceinline__ int64_t brick_index(int32_t code, int32_t i, int32_t j, int32_t k) {
  return ((int64_t)code * 576 + ((j & 7) * 8 + (k & 7)) * 9 + (i & 7)) * 4;
}

struct Cell {
  int32_t code;
  float value;
};

// A constant materialised where it is used.  Literal operands a VOP3 or LDS instruction cannot
// encode are otherwise hoisted out of the state-machine loop into a VGPR held for the whole kernel
// (r02: four such VGPRs in the 72-VGPR production kernel).
// The v_mov is part of the volatile asm, so the compiler can neither hoist nor share it.
__host__ __device__ __forceinline__ int32_t local_const(int32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  int32_t r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "i"(c));
  return r;
#else
  return c;
#endif
}
__host__ __device__ __forceinline__ float local_const(float c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bit_cast(float, local_const(__builtin_bit_cast(int32_t, c)));
#else
  return c;
#endif
}
// A value the compiler must treat as computed here (keeps loop-invariant work of a rare block in it).
__host__ __device__ __forceinline__ float local_value(float v) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(v));
#endif
  return v;
}

// cells8 entries carry one more bit: "interior" = this 8^3 cell and its 26 neighbours all have
// HDDA dim 8 (leaf or lower-node tile) and lie inside the table.  It is stored as bit 30 differing
// from the sign bit (codes are leaf indices < 2^30 or small negatives, where bit 30 == bit 31).
constexpr int32_t kInteriorBit = 1 << 30;
// walk8 entry of a cell the HDDA fast path cannot take (not interior; or an interior cell whose
// majorant has exactly these NaN bits, which then takes the general path -- same result).
constexpr uint32_t kWalkSlow = 0xFFFFFFFFu;
// walk8 flag of a dim-8 cell that is not interior (an "edge" cell: some cell of its 3x3x3
// neighbourhood is not dim 8).  Its low bits are the cell's majorant; the fast path holds for a step
// whose lookahead point lies in the cell itself.  Majorants with the sign bit set are stored as
// kWalkSlow.
constexpr uint32_t kWalkEdge = 0x80000000u;
// Zero runs (empty-space skipping without changing a step): an interior cell with majorant +0 stores
// its zero-run radius r (the bits 0..kZeroRunMax) -- every cell within Chebyshev distance r is interior
// with majorant +0 as well.  The HDDA's next cell is face-adjacent, so its word is known to be a zero
// run of radius >= r - 1: hdda_pre_advance writes r - 1 instead of loading it, and a ray crossing empty
// space loads one walk word per ~r cells.  Every step still runs (same times, same float operations);
// only its load goes.  Interior majorants whose bits are 1..kZeroRunMax (tiny denormals) are stored
// as kWalkSlow.
constexpr uint32_t kZeroRunMax = 63;
#ifndef VPT_ZERO_RUNS
#define VPT_ZERO_RUNS 1
#endif
#if !defined(__HIP_DEVICE_COMPILE__)
// Host builds only (the CPU simulator): walk-word loads issued and walk words synthesised from a zero run.
inline uint64_t g_walk_loads = 0, g_walk_synth = 0;
#endif
// Cells of kWalkSlow padding around the walk table.  The HDDA prefetches the walk word of the cell
// it is about to enter whenever it walks at dim 8; that cell is at most 2 cells outside the r8 table
// (see hdda_pre_advance), so the prefetch needs no bounds test.
constexpr int32_t kWalkPad = 2;
// r03 step trim: the fast path's pre-advance without the dim test, s_t1 by one min, the free-flight
// draw's 1 - u by one fma and a max (rng_one_minus_uniform).  0 = the r03v code (A/B builds).
#ifndef VPT_STEP_TRIM
#define VPT_STEP_TRIM 1
#endif
// A cells8 code whose cell has HDDA dim 8: a leaf (code >= 0) or a lower-node tile (-16 / -17).
__host__ __device__ __forceinline__ bool cell8_dim8(int32_t code) { return code >= 0 || code == -16 || code == -17; }
__host__ __device__ __forceinline__ int32_t cell8_code(int32_t x) {
  return (x & ~kInteriorBit) | ((x >> 1) & kInteriorBit);
}
__host__ __device__ __forceinline__ bool cell8_interior(int32_t x) { return ((x ^ (x << 1)) & (1 << 31)) != 0; }

// Row-major index (a * n1 + b) * n2 + c of a table cell (a, b, c inside the table): two full-rate
// v_mad_u32_u24, whose operands are below 2^24 for tables of up to 4096 cells a side; the compiler otherwise
// emits v_mad_u64_u32 for these (r06zb, with walk_index's: C3 335.6 / 336.4 vs 336.6 / 337.3 ms, C4 flat).
#ifndef VPT_WALK_MAD24_ASM
#define VPT_WALK_MAD24_ASM 1
#endif
__host__ __device__ __forceinline__ uint32_t mad_index(int32_t a, int32_t b, int32_t c, const int32_t n[3]) {
#if defined(__HIP_DEVICE_COMPILE__) && VPT_WALK_MAD24_ASM
  uint32_t ab, idx;
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(ab) : "v"(a), "s"(n[1]), "v"(b));
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(idx) : "v"(ab), "s"(n[2]), "v"(c));
  return idx;
#else
  return ((uint32_t)a * (uint32_t)n[1] + (uint32_t)b) * (uint32_t)n[2] + (uint32_t)c;
#endif
}

__host__ __device__ __forceinline__ Cell cell_at(const DevGrid& g, int32_t i, int32_t j, int32_t k) {
  int32_t a = (i - g.r8_org[0]) >> 3, b = (j - g.r8_org[1]) >> 3, c = (k - g.r8_org[2]) >> 3;
  if ((uint32_t)a < (uint32_t)g.r8_n[0] && (uint32_t)b < (uint32_t)g.r8_n[1] && (uint32_t)c < (uint32_t)g.r8_n[2]) {
    int2 e = g.cells8[mad_index(a, b, c, g.r8_n)];
    return Cell{cell8_code(e.x), math::as_f32((uint32_t)e.y)};
  }
  a = (i - g.r128_org[0]) >> 7;
  b = (j - g.r128_org[1]) >> 7;
  c = (k - g.r128_org[2]) >> 7;
  if ((uint32_t)a < (uint32_t)g.r128_n[0] && (uint32_t)b < (uint32_t)g.r128_n[1] && (uint32_t)c < (uint32_t)g.r128_n[2]) {
    int2 e = g.cells128[mad_index(a, b, c, g.r128_n)];
    return Cell{e.x, math::as_f32((uint32_t)e.y)};
  }
  for (int32_t r = 0; r < g.root_count; ++r) {
    const RootTileDev& t = g.root[r];
    if ((i & ~4095) == t.origin[0] && (j & ~4095) == t.origin[1] && (k & ~4095) == t.origin[2])
      return Cell{-(2 * 4096 + t.active), t.value};
  }
  return Cell{local_const(-(2 * 4096)), g.background};
}

// max(8, ReadAccessor::getDim(ijk)) (volume.cpp:11-14): a leaf's getDim is 1.
__host__ __device__ __forceinline__ int32_t hdda_dim_of(Cell c) { return c.code >= 0 ? 8 : ((-c.code) >> 1); }
// update_current_majorant (volume.cpp:18-36): leaf max, else active tile value, else 0.
__host__ __device__ __forceinline__ float majorant_of(Cell c) {
  if (c.code >= 0) return c.value;
  return ((-c.code) & 1) ? c.value : 0.0f;
}
// ReadAccessor::getValue(ijk)
__host__ __device__ __forceinline__ float value_at(const DevGrid& g, int32_t i, int32_t j, int32_t k) {
  Cell c = cell_at(g, i, j, k);
  if (c.code < 0) return c.value;
  return g.bricks[brick_index(c.code, i, j, k)];
}

// nanovdb::math::SampleFromVoxels<Acc,1,true> caches the 2x2x2 stencil of the last cell; the cache
// never changes a value, and on the cloud it hits < 2% of evaluations, so the device re-reads the
// stencil every time and only remembers the last cell to count refreshes (algorithmic bytes).
struct StencilCell {
  int32_t i, j, k;
  int32_t code;  // cell code of the last stencil's corner cell (reused while in the same 8^3 cell)
};

__host__ __device__ __forceinline__ void fetch_stencil(const DevGrid& g, Cell c, int32_t i, int32_t j, int32_t k,
                                                       float v[8]) {
  if (c.code >= 0) {
    // Corner cell inside a leaf: its stencil is one 32-byte piece of the pool.
    const float4* p = reinterpret_cast<const float4*>(g.bricks + brick_index(c.code, i, j, k));
    const float4 lo = p[0], hi = p[1];
    v[0] = lo.x;
    v[1] = lo.y;
    v[2] = lo.z;
    v[3] = lo.w;
    v[4] = hi.x;
    v[5] = hi.y;
    v[6] = hi.z;
    v[7] = hi.w;
  } else {
    // Corner cell without a leaf (tile / background cell, rare): eight getValue calls, one at a
    // time — a compact loop whose lookups are not all in flight at once (register pressure), the
    // result selected into statically indexed registers.
#pragma unroll 1
    for (int q = 0; q < 8; ++q) {
      const float val = value_at(g, i + (q >> 2), j + ((q >> 1) & 1), k + (q & 1));
      v[0] = q == 0 ? val : v[0];
      v[1] = q == 1 ? val : v[1];
      v[2] = q == 2 ? val : v[2];
      v[3] = q == 3 ? val : v[3];
      v[4] = q == 4 ? val : v[4];
      v[5] = q == 5 ? val : v[5];
      v[6] = q == 6 ? val : v[6];
      v[7] = q == 7 ? val : v[7];
    }
  }
}

// TrilinearSampler::sample: lerp(a, b, w) = a + w * (b - a), z then y then x.
__host__ __device__ __forceinline__ float lerpf(float a, float b, float w) { return a + w * (b - a); }
// Returns true when the cell differs from the previous evaluation (a NanoVDB stencil refresh).
// The leaf-slot lookup is skipped while the corner cell stays in the previous one's 8^3 cell.
__host__ __device__ __forceinline__ bool trilinear(const DevGrid& g, StencilCell& last, float x, float y, float z,
                                                   float& out) {
  float fi = floorf(x), fj = floorf(y), fk = floorf(z);
  float u = x - fi, v = y - fj, w = z - fk;
  int32_t i = (int32_t)fi, j = (int32_t)fj, k = (int32_t)fk;
  bool refresh = i != last.i || j != last.j || k != last.k;
  const int32_t dx = (i ^ last.i) | (j ^ last.j) | (k ^ last.k);
  const bool same_leaf = last.code >= 0 && dx >= 0 && dx < 8;  // same 8^3 cell as a leaf-backed stencil
  Cell c;
  if (same_leaf) {
    c.code = last.code;
    c.value = 0.0f;  // only read for non-leaf cells, which are never reused (code < 0 -> value_at)
  } else {
    c = cell_at(g, i, j, k);
  }
  last.i = i;
  last.j = j;
  last.k = k;
  last.code = c.code;
  float s[8];
  fetch_stencil(g, c, i, j, k, s);
  out = lerpf(lerpf(lerpf(s[0], s[1], w), lerpf(s[2], s[3], w), v), lerpf(lerpf(s[4], s[5], w), lerpf(s[6], s[7], w), v), u);
  return refresh;
}
constexpr int32_t kNoCell = (int32_t)0x80000000;  // "no previous cell" (reset per sampler instance)

// nanovdb Map: matMult with fmaf.
__host__ __device__ __forceinline__ void map_inv(const DevGrid& g, float x, float y, float z, float& ox, float& oy, float& oz) {
  const float* m = g.inv_mat;
  float a = x - g.vec[0], b = y - g.vec[1], c = z - g.vec[2];
  ox = __builtin_fmaf(a, m[0], __builtin_fmaf(b, m[1], c * m[2]));
  oy = __builtin_fmaf(a, m[3], __builtin_fmaf(b, m[4], c * m[5]));
  oz = __builtin_fmaf(a, m[6], __builtin_fmaf(b, m[7], c * m[8]));
}
__host__ __device__ __forceinline__ void jac_inv(const DevGrid& g, float x, float y, float z, float& ox, float& oy, float& oz) {
  const float* m = g.inv_mat;
  ox = __builtin_fmaf(x, m[0], __builtin_fmaf(y, m[1], z * m[2]));
  oy = __builtin_fmaf(x, m[3], __builtin_fmaf(y, m[4], z * m[5]));
  oz = __builtin_fmaf(x, m[6], __builtin_fmaf(y, m[7], z * m[8]));
}
__host__ __device__ __forceinline__ void map_fwd(const DevGrid& g, float x, float y, float z, float& ox, float& oy, float& oz) {
  const float* m = g.mat;
  ox = __builtin_fmaf(x, m[0], __builtin_fmaf(y, m[1], __builtin_fmaf(z, m[2], g.vec[0])));
  oy = __builtin_fmaf(x, m[3], __builtin_fmaf(y, m[4], __builtin_fmaf(z, m[5], g.vec[1])));
  oz = __builtin_fmaf(x, m[6], __builtin_fmaf(y, m[7], __builtin_fmaf(z, m[8], g.vec[2])));
}

// ------------------------------------------------------------------------------------------------
// Scene constants (host-computed once with the reference's formulas)
// ------------------------------------------------------------------------------------------------
struct DevScene {
  DevGrid density;
  DevGrid temperature;
  int32_t has_temperature;
  uint32_t seed;
  int32_t W, H, tw, th;
  uint32_t ntx;
  uint32_t max_depth;
  uint64_t T;  // jobs per wave
  int32_t single_pixel_enabled;
  int32_t sp_x, sp_y;
  float jitter_scale;   // use_jitter ? 0.5 : 0.0 (worker.cpp:122)
  float cam_L[9];       // Camera::raster_to_world_dir linear (row-major)
  float cam_t[3];       // and translation
  float cam_pos[3];
  float imaging_ratio;
  float le_inf[3];      // infinite_light.xyz * multiplier (worker.cpp:199)
  float Li[3];          // distant_light.xyz * multiplier (worker.cpp:55)
  int32_t li_zero;      // Li == 0 -> sample_Ld returns before any draw (worker.cpp:57-58)
  float wi[3];          // distant_light.inv_direction.normalized() (worker.cpp:54)
  // Shadow rays all have direction wi: their index-space direction, its reciprocal, the length
  // factor and the iterator scale are scene constants (scene_finalize; same float operations).
  float sh_d[3], sh_inv[3], sh_len, sh_scale, sh_rscale;
  // Henyey-Greenstein terms that depend on g only (random.hpp:56-84, utils.hpp:61-66): the same
  // float values the reference recomputes at every call.
  float hg_g2, hg_1pg2, hg_1mg2, hg_1pg, hg_2g, hg_inv2g, hg_num;
  float sigma_a, sigma_s, sigma_t, g_hg, le_scale, temp_scale, temp_offset;
  float sigt_c;  // RN(sigma_t * kOvershootC): the free-flight overshoot pre-test's constant factor (SM_DRAW)
  // Wave gating of the rare states: a rare block runs when at least gate_min lanes of the wavefront
  // wait for it, or when fewer than gate_idle lanes are sampling (1/64 = always run).
  int32_t gate_min, gate_idle;
  int32_t gate_eval;  // the density evaluation (trilinear + event) runs for >= gate_eval waiting lanes
  int32_t gate_walk;  // keep stepping in an inner loop while >= gate_walk lanes walk (0: one step)
  // Throughput mode (VPT_RNG_PIXEL): the work item is one pixel of a job, its stream
  // is hash(seed, jid * tile_area + pixel).  0 = the reference's per-job stream.
  int32_t pixel_mode;
  uint32_t tile_area;
  int32_t wave_lanes;   // lanes of each wavefront that take jobs (64; latency-bound launches: 0 = auto)
  const float* bb;      // blackbody table [501][3] (row 500 = 0)
  int32_t bb_lds_ok;    // every reachable lookup reads rows < kBbLdsRows: the kernel's LDS copy serves it
  const float* cie;     // [471][3] for T >= 49900 K
  float y_integral;
};

// The scene as the kernel reads it: a pointer into the constant address space (scalar loads).
// opaque() hides the pointer's value from the optimiser, so loads through it are not hoisted out
// of the state-machine loop (they would pin ~100 SGPRs for the whole kernel and spill to VGPR
// lanes); each block re-reads the few constants it uses with s_load instead.
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) DevScene* ScenePtr;
#else
typedef const DevScene* ScenePtr;
#endif
__host__ __device__ __forceinline__ ScenePtr opaque(ScenePtr p) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+s"(p));
#endif
  return p;
}

// ------------------------------------------------------------------------------------------------
// RNG: hash(seed, jid) + pcg32_fast + uniform<float> (hash.hpp:20-67, random.hpp:86-115)
// ------------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t job_seed(uint64_t seed, uint64_t k) {
  const uint64_t m = 0xc6a4a7935bd1e995ULL;
  uint64_t h = seed ^ (8ULL * m);
  k *= m;
  k ^= k >> 47;
  k *= m;
  h ^= k;
  h *= m;
  h ^= h >> 47;
  h *= m;
  h ^= h >> 47;
  return h | 3ULL;  // pcg32_fast::seed: state = s | 3
}
// Lane::pix flags of a throughput-mode work item: trace only the pixel it names (kOnePixel), which
// has been started (kPixelTaken); kPixelMask extracts the pixel counter.
constexpr int32_t kOnePixel = 1 << 30;
constexpr int32_t kPixelTaken = 1 << 29;
constexpr int32_t kPixelMask = kPixelTaken - 1;

// pcg32_fast's output (pcg_random.hpp xsh_rs): (uint32)((old ^ (old >> 22)) >> (22 + (old >> 61))).  On
// the device the shifts by 22..29 take the low word of a 64-bit pair with v_alignbit_b32 (32-bit
// funnel shifts) instead of two 64-bit shifts.
__host__ __device__ __forceinline__ uint32_t pcg32_output(uint64_t old) {
#if defined(__HIP_DEVICE_COMPILE__) && VPT_STEP_TRIM
  const uint32_t lo = (uint32_t)old, hi = (uint32_t)(old >> 32);
  const uint32_t xlo = lo ^ __builtin_amdgcn_alignbit(hi, lo, 22u), xhi = hi ^ (hi >> 22);
  return __builtin_amdgcn_alignbit(xhi, xlo, 22u + (hi >> 29));
#else
  const uint32_t rshift = (uint32_t)(old >> 61);
  old ^= old >> 22;
  return (uint32_t)(old >> (22 + rshift));
#endif
}
__host__ __device__ __forceinline__ float rng_uniform(uint64_t& state) {
  const uint32_t r = pcg32_output(state);
  state = state * 6364136223846793005ULL;
  float v = (float)r * 0x1p-32f;
  const float one_minus_eps = 0x1.fffffep-1f;
  return (v < one_minus_eps) ? v : one_minus_eps;  // std::min<float>(1-eps, v)
}
// 1 - rng_uniform(state), as the free-flight draw uses it (random.hpp:20-22: -log(1 - u)).  With
// v = r * 2^-32 (exact), RN(1 - min(v, 1 - 2^-24)) == max(RN(1 - v), 2^-24): below 1 - 2^-24 the min is
// v and 1 - v > 2^-24, so its rounding is >= 2^-24; at or above it both sides are 2^-24 (v may round
// up to 1).  RN(1 - v) is one fma of the exact product.
__host__ __device__ __forceinline__ float rng_one_minus_uniform(uint64_t& state) {
  const uint32_t r = pcg32_output(state);
  state = state * 6364136223846793005ULL;
  return fmaxf(__builtin_fmaf(-(float)r, 0x1p-32f, 1.0f), 0x1p-24f);
}

// ------------------------------------------------------------------------------------------------
// Blackbody lookup (precompute_blackbody.cpp:25-52)
// ------------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ float bb_idx_to_temp(int idx) { return (idx - 1) * 100.0f; }
__host__ __device__ inline float planck_dev(float lambda_m, float t) {
  if (t <= 0.0f) return 0.0f;
  const float c = 299792458.f, h = 6.62606957e-34f, kb = 1.3806488e-23f;
  const float num = 2 * h * c * c;
  float l2 = lambda_m * lambda_m;
  float lambda5 = (float)((double)l2 * (double)l2 * (double)lambda_m);  // pow(double(l),5) (not bit-exact)
  float e = expf((h * c) / (lambda_m * kb * t));
  return num / (lambda5 * (e - 1));
}
// Rows of the blackbody table the temperature kernel copies into LDS (T < 6 300 K): a grid whose
// temperatures stay below that (host check, vpt_gpu_create: the trilinear value is a convex combination
// of voxel / tile / background values, so max(v) * scale + offset bounds it) looks every row up there;
// others read the whole table from memory.  64 rows = 768 B per block instead of 6 KB.
constexpr int kBbLdsRows = 64;
// bb: the blackbody table [501][3] (S.bb, or the kernel's LDS copy of its first kBbLdsRows rows).
__host__ __device__ inline void blackbody_xyz(const DevScene& S, const float* bb, float t, float& X, float& Y, float& Z) {
  if (!(t - t == 0.0f)) {  // !isfinite
    X = Y = Z = __builtin_nanf("");
    return;
  }
  if (t <= 0.0f) {
    X = Y = Z = 0.0f;
    return;
  }
  if (t >= 49900.0f) {
    // Direct spectral integration (spectral.hpp:62-75).  Rare path: std::pow/std::exp are glibc's
    // on the host, so this branch is not bit-exact (documented in DESIGN.md).
    float acc[3] = {0.0f, 0.0f, 0.0f};
    for (int c = 0; c < 3; ++c) {
      float integ = 0.0f;
      for (int i = 0; i < 471; ++i) integ += S.cie[i * 3 + c] * planck_dev((float)(360 + i) * 1e-9f, t);
      acc[c] = integ;
    }
    X = acc[0] / S.y_integral;
    Y = acc[1] / S.y_integral;
    Z = acc[2] / S.y_integral;
    return;
  }
  int dn = (int)math::div_by_recip(t, 100.0f, 0.01f);  // t / 100 (0.01f == RN(1/100))
  while (t <= bb_idx_to_temp(dn - 1)) --dn;
  while (t >= bb_idx_to_temp(dn + 1)) ++dn;
  const float* a = bb + dn * 3;
  if (t == bb_idx_to_temp(dn)) {
    X = a[0];
    Y = a[1];
    Z = a[2];
    return;
  }
  float w = math::div_by_recip(t - bb_idx_to_temp(dn), 100.0f, 0.01f);
  const float* b = a + 3;
  X = a[0] + (b[0] - a[0]) * w;  // vpt::lerp: a + (b - a) * t (utils.hpp:26-29)
  Y = a[1] + (b[1] - a[1]) * w;
  Z = a[2] + (b[2] - a[2]) * w;
}

// q / rw for a pixel counter q >= 0 and a row width rw >= 1.  Below 2^20 the quotient comes from the
// hardware reciprocal: (q + 0.5) / rw lies >= 0.5 / rw from every integer and the estimate's error
// is < 2^-22 relative (v_rcp_f32 within 1 ulp, one rounded product), i.e. < 0.25 / rw.
__host__ __device__ __forceinline__ int32_t div_pix(int32_t q, int32_t rw) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (q < (1 << 20)) return (int32_t)(((float)q + 0.5f) * __builtin_amdgcn_rcpf((float)rw));
#endif
  return q / rw;
}

// ------------------------------------------------------------------------------------------------
// Lane state
// ------------------------------------------------------------------------------------------------
enum : int32_t {
  ST_FETCH = 0,   // take the next job
  ST_PIXEL = 1,   // start the next pixel of the tile
  ST_RAY = 2,     // Volume::intersect + iterator setup: primary ray (top of the depth loop) or shadow ray
  ST_SAMPLE = 3,  // inside MajorantTransmittanceSampler::next (primary or shadow ray)
  ST_NEE_DONE = 4,
  ST_FINISH = 5,  // pixel done: environment light, film
  ST_DONE = 6,
  ST_SHADOW = 7,  // sample_Ld's Volume::intersect + iterator setup (direction wi: constants)
  ST_FINISH_T = 8 // pixel done after absorption / scatter past max_depth ("terminated": no env light)
};
// SM_EVAL: density at s_t0 pending.  SM_NONE: the lane is not sampling (state != ST_SAMPLE); every
// transition out of ST_SAMPLE sets it, so the walk loop's blocks test sm alone.
enum : int32_t { SM_NEED_SEG = 0, SM_STEP = 1, SM_DRAW = 2, SM_EVAL = 3, SM_NONE = 4 };
// Block ids for the optional SIMT-utilisation profile (env.prof; a no-op unless VPT_PROFILE).
enum : int32_t {
  PB_ITER = 0, PB_FETCH, PB_PIXEL, PB_RAY, PB_SAMPLE, PB_NEED_SEG, PB_STEP, PB_DRAW, PB_TRILINEAR,
  PB_EVENT, PB_SHADOW_HIT, PB_NONE, PB_NEE_DONE, PB_FINISH,
  // census of the wavefront at every walk-loop iteration (lanes per state)
  PB_W_WALK, PB_W_EVAL, PB_W_NEE, PB_W_FIN, PB_W_RAY, PB_W_PIX, PB_W_DONE, PB_COUNT
};
// Section ids for the wave-time profile (env.tick: shader cycles since the previous tick, per
// wavefront; gating ballots are charged to the section that follows them).
enum : int32_t { PT_FETCH = 0, PT_PIXEL, PT_RAY, PT_WALK, PT_EVAL, PT_NEE, PT_FINISH, PT_SEG, PT_STEP, PT_DRAW, PT_COUNT };

// Event counters, in vpt_counters order.  They are tallied per wavefront (env.tally) rather than
// held per lane.  The production kernel counts the four that price algorithmic bytes;
// the debug kernel (per-sample records) counts all of them for parity checks.
enum : int32_t {
  CNT_SAMPLES = 0, CNT_DDA_STEPS, CNT_SEGMENTS, CNT_DRAWS, CNT_STENCILS, CNT_DENSITY_EVALS, CNT_TEMP_STENCILS,
  CNT_SCATTERS, CNT_SHADOW_RAYS, CNT_RNG_DRAWS, CNT_EXCHANGED, CNT_COUNT
};

// The lane's cold state: touched only by the per-pixel, per-bounce and film blocks, never by the
// walk.  The kernel keeps it in LDS (Env::cold(), one 15-word slot per lane: an odd stride, so a
// wavefront's accesses hit distinct banks) instead of VGPRs, which leaves the walk its registers.
struct LaneCold {
  int32_t x0, y0, pix;
  uint32_t depth;
  float L[3];
  float ro[3], rd[3];  // current primary world ray; ro is also the scatter point during NEE
  StencilCell dens_cell;  // the density sampler's last stencil cell (collision evaluation only)
  float Tr;               // shadow-ray transmittance (< 0: sample_Ld returns zero)
  float y_draw;           // 1 - u of a free-flight draw whose exact distance is pending (SM_EVAL)
  uint32_t item_lo, item_hi;  // throughput mode: jid * tile_area of the lane's job (its pixels' streams);
                              // reference mode: item_lo = the job's index in the launch (the ordered film);
                              // feeds: the reserved item while the lane waits for it
#ifdef VPT_JOB_LOG
  uint32_t t_start;       // diagnostic build: s_memrealtime at the job's fetch
  uint32_t job;           // and the job's index in the launch
#endif
};

struct Lane {
  int32_t state, sm, shadow;
  uint64_t rng;
  uint64_t jid_local;  // job index relative to jid_begin (records / events only)
  uint32_t n_events;   // events logged so far in this job (event traces only)
  // RayMajorantIterator: index-space ray, scale, majorant, HDDA (NanoVDB math::HDDA state)
  float e[3], d[3];  // (invDir = rcp_rn(d) is recomputed where HDDA::update needs it)
  float scale, rscale;  // m_scale and recip_for_div(m_scale)
  float maj;
  int32_t dim;
  float Tn, T1;     // Tn: HDDA time of the pending cell (the one the HDDA has been advanced into)
  uint32_t pw;      // walk word of the pending cell (prefetched; kWalkSlow when not at dim 8)
  float nxt[3];
  int32_t vox[3];   // HDDA voxel in 8^3-cell units relative to the walk table's origin: (voxel - w8_org) / 8
  float finc[3];    // HDDA: dim * delta[axis] (the float product NanoVDB adds at every step)
  int32_t vinc[3];  // HDDA: dim * step[axis] / 8 (cell units; every HDDA dim is a multiple of 8)
  // current majorant segment
  float s_t0, s_t1, s_dmaj;
  StencilCell temp_cell;
  uint32_t n_dda;  // hot counter, per lane (flushed by the kernel at exit)
};

// HDDA step direction and per-cell increment from the (normalised, index-space) direction:
// step = 0 if dir == 0, +1 if invDir > 0, else -1; delta = |invDir| (NanoVDB HDDA::init).
__host__ __device__ __forceinline__ int32_t hdda_stp(float d, float inv) { return d == 0.0f ? 0 : (inv > 0 ? 1 : -1); }

// The direction-only part of Ray::worldToIndexF + RayMajorantIterator's scale: index-space unit
// direction d, invDir = 1/d, |worldToIndexDirF(dir)| (scales t0) and m_scale.
struct RayDir {
  float d[3], inv[3], len, scale, rscale;
};
__host__ __device__ __forceinline__ RayDir ray_dir_setup(const DevGrid& g, const float dir[3]) {
  RayDir r;
  float dx, dy, dz;
  jac_inv(g, dir[0], dir[1], dir[2], dx, dy, dz);
  // Correctly rounded sqrt / reciprocal through the short exact sequences of vpt_math.h.
  float len = math::sqrt_rn(dx * dx + dy * dy + dz * dz);
  float inv_len = math::rcp_rn(len);
  r.d[0] = dx * inv_len;
  r.d[1] = dy * inv_len;
  r.d[2] = dz * inv_len;
  r.len = len;
  r.inv[0] = math::rcp_rn(r.d[0]);
  r.inv[1] = math::rcp_rn(r.d[1]);
  r.inv[2] = math::rcp_rn(r.d[2]);
  // m_scale = 1 / |worldToIndexDirF(index dir)|
  float jx, jy, jz;
  jac_inv(g, r.d[0], r.d[1], r.d[2], jx, jy, jz);
  r.scale = math::rcp_rn(math::sqrt_rn(jx * jx + jy * jy + jz * jz));
  r.rscale = math::recip_for_div(r.scale);
  return r;
}

// HDDA::step() without the time test: axis = MinIndex(next), mNext[axis] += mDim * mDelta[axis],
// mVoxel[axis] += mDim * mStep[axis]; returns the new time.  Written as selects
// over all three axes: branches (or an axis index) make the compiler move the HDDA state into an
// indexed scratch array.
__host__ __device__ __forceinline__ float hdda_advance(Lane& ln) {
  const float n0 = ln.nxt[0], n1 = ln.nxt[1], n2 = ln.nxt[2];
  const bool c12 = n1 < n2;
  const bool a0 = n0 < n1 && n0 < n2;
  const bool a1 = !a0 && c12;
  const bool a2 = !(a0 || a1);
  const float tn = a0 ? n0 : (c12 ? n1 : n2);
  ln.nxt[0] = a0 ? tn + ln.finc[0] : n0;
  ln.nxt[1] = a1 ? tn + ln.finc[1] : n1;
  ln.nxt[2] = a2 ? tn + ln.finc[2] : n2;
  ln.vox[0] += a0 ? ln.vinc[0] : 0;
  ln.vox[1] += a1 ? ln.vinc[1] : 0;
  ln.vox[2] += a2 ? ln.vinc[2] : 0;
  return tn;
}

#if !defined(__HIP_DEVICE_COMPILE__)
// Host builds only (the CPU simulator, tests/native/hostsim.cpp): walk-table lookups of a cell outside
// the padded table, which the padding argument of hdda_pre_advance rules out.  Tests read it as 0.
inline uint64_t g_walk_outside = 0;
#endif

// Walk-table index of the 8^3 cell v, in cell units relative to the table's origin (Lane::vox).
// The min() only guarantees a memory-safe address; hdda_pre_advance never asks for a cell beyond the
// padding.  The padding is in index space, and so is the HDDA's lookahead (1.0001 along the index-space
// ray, whose direction Ray::worldToIndexF normalises): the argument holds for every voxel size and any
// affine map.
__host__ __device__ __forceinline__ uint32_t walk_index(const DevGrid& g, const int32_t v[3]) {
  const uint32_t a = (uint32_t)v[0], b = (uint32_t)v[1], c = (uint32_t)v[2];
#if defined(__HIP_DEVICE_COMPILE__) && VPT_WALK_MAD24_ASM
  // Two full-rate v_mad_u32_u24 (the compiler otherwise folds the first mul24 + add into a v_mad_u64_u32).  The instruction masks its operands to 24 bits as mul24 does: the same value.
  uint32_t ab, idx;
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(ab) : "v"(a), "s"((uint32_t)g.w8_n[1]), "v"(b));
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(idx) : "v"(ab), "s"((uint32_t)g.w8_n[2]), "v"(c));
#else
  const uint32_t idx = math::mul24(math::mul24(a, (uint32_t)g.w8_n[1]) + b, (uint32_t)g.w8_n[2]) + c;
#endif
  return idx < g.w8_max ? idx : g.w8_max;
}

// Host builds: count a walk-word load of the cell holding v (and whether it lies outside the table).
__host__ __device__ __forceinline__ void note_walk_load(const DevGrid& g, const int32_t v[3]) {
#if !defined(__HIP_DEVICE_COMPILE__)
  const uint32_t a = (uint32_t)v[0], b = (uint32_t)v[1], c = (uint32_t)v[2];
  if (a >= (uint32_t)g.w8_n[0] || b >= (uint32_t)g.w8_n[1] || c >= (uint32_t)g.w8_n[2]) ++g_walk_outside;
  ++g_walk_loads;
#else
  (void)g;
  (void)v;
#endif
}
__host__ __device__ __forceinline__ uint32_t load_walk_word(const DevGrid& g, uint32_t idx) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(g.walk8) + idx * 4u);
}

// The HDDA runs one step ahead of the segment logic: after a step has examined its cell (or at
// begin_ray) the HDDA advances into the next cell (Tn = its entry time) and issues the load of that
// cell's walk word, which the next step consumes -- the load is in flight while the lane draws
// and the wavefront runs its other blocks.  The advance is the one the next step would make: the
// HDDA state only changes in the step's slow path, which runs before the pre-advance.
// Padding argument (kWalkPad = 2): at dim 8 the current cell is within one cell of the r8 table (it
// was reached from an interior cell, or its lookahead cell -- within ~1 voxel -- has dim 8 and so
// lies in the table), and the next cell is adjacent to it.
// synth: the step took the fast path on a zero-run word r >= 1 (still in ln.pw): the next cell's word
// is r - 1, without a load (kZeroRunMax).  The word is decremented in place by a select before the
// (masked) load, so the load writes the register the next step reads and no VALU write follows it
// (either would make the wavefront wait for the load here instead of at the next step).
__host__ __device__ __forceinline__ void hdda_pre_advance(const DevGrid& g, Lane& ln, bool synth = false) {
  ln.Tn = hdda_advance(ln);
  synth = VPT_ZERO_RUNS && synth;
  ln.pw = synth ? ln.pw - 1u : kWalkSlow;
  if (!synth && ln.dim == 8) {
    ln.pw = load_walk_word(g, walk_index(g, ln.vox));
    note_walk_load(g, ln.vox);
  }
#if !defined(__HIP_DEVICE_COMPILE__)
  if (synth) ++g_walk_synth;
#endif
}

// Volume::intersect (volume.cpp:78-88) + RayMajorantIterator ctor (volume.cpp:90-98).
__host__ __device__ __forceinline__ bool begin_ray(const DevGrid& g, Lane& ln, const float o[3], const RayDir& rd) {
  // nanovdb::math::Ray<float>(eye, dir) with t0 = 1e-5 (Delta<float>), t1 = FLT_MAX; worldToIndexF.
  float ex, ey, ez;
  map_inv(g, o[0], o[1], o[2], ex, ey, ez);
  const float dx = rd.d[0], dy = rd.d[1], dz = rd.d[2];
  float t0 = rd.len * 1e-5f;
  float t1 = 3.40282347e+38f;
  const float ix = rd.inv[0], iy = rd.inv[1], iz = rd.inv[2];
  // Ray::clip(indexBBox): slab test against [min, max + 1].
  const float E[3] = {ex, ey, ez}, I[3] = {ix, iy, iz};
  for (int a = 0; a < 3; ++a) {
    float lo = (float)g.bbox_min[a], hi = (float)(g.bbox_max[a] + 1);
    lo = (lo - E[a]) * I[a];
    hi = (hi - E[a]) * I[a];
    if (lo > hi) {
      float tmp = lo;
      lo = hi;
      hi = tmp;
    }
    if (lo > t0) t0 = lo;
    if (hi < t1) t1 = hi;
  }
  // One test after the three slabs: t0 never decreases and t1 never increases (and neither becomes
  // NaN), so an empty interval after any axis stays empty -- the same answer as Ray::clip's early exit.
  if (t0 > t1) return false;
  ln.e[0] = ex;
  ln.e[1] = ey;
  ln.e[2] = ez;
  ln.d[0] = dx;
  ln.d[1] = dy;
  ln.d[2] = dz;
  ln.scale = rd.scale;
  ln.rscale = rd.rscale;
  // HDDA(ray, max(8, getDim(floor(ray.start())))) -> init(ray, t0, t1, dim)
  float px = ex + dx * t0, py = ey + dy * t0, pz = ez + dz * t0;
  const Cell c0 = cell_at(g, (int32_t)floorf(px), (int32_t)floorf(py), (int32_t)floorf(pz));
  int32_t dim = hdda_dim_of(c0);
  // update_current_majorant at the start voxel (floor(start) & ~(dim-1)): the cell of a dim-d
  // voxel answers every query of its d^3 block alike, so c0 gives the first segment's majorant.
  ln.maj = majorant_of(c0);
  ln.dim = dim;
  ln.T1 = t1;
  ln.s_t1 = t0;  // the sampler's position: NEED_SEG starts the first segment here
  const float P[3] = {px, py, pz}, D[3] = {dx, dy, dz};
  for (int a = 0; a < 3; ++a) {
    int32_t v = ((int32_t)floorf(P[a])) & (~(dim - 1));
    // cell units relative to the table (v and w8_org are multiples of 8): the walk index needs no
    // subtraction or shift per step
    ln.vox[a] = (v - g.w8_org[a]) >> 3;
    ln.finc[a] = (float)dim * fabsf(I[a]);
    ln.vinc[a] = (dim >> 3) * hdda_stp(D[a], I[a]);
    // HDDA::init: the next boundary at v + dim (I > 0) or v; none for D == 0 (selects, not branches)
    const float n = t0 + ((float)(I[a] > 0 ? v + dim : v) - P[a]) * I[a];
    ln.nxt[a] = D[a] == 0.0f ? 3.40282347e+38f : n;
  }
  hdda_pre_advance(g, ln);
  ln.sm = SM_NEED_SEG;
  return true;
}

// The general HDDA step (volume.cpp:63-70) on the pending cell at time tk, whose walk word w is not an
// interior one: new_dim = max(8, getDim(floor(ray(time + 1.0001f)))), HDDA::update, and the majorant.
__host__ __device__ __forceinline__ bool hdda_general(const DevGrid& g, Lane& ln, uint32_t w, float tk,
                                                      const int32_t vc[3]) {
  float tl = tk + 1.0001f;
  const int32_t lx = (int32_t)floorf(ln.e[0] + ln.d[0] * tl), ly = (int32_t)floorf(ln.e[1] + ln.d[1] * tl),
                lz = (int32_t)floorf(ln.e[2] + ln.d[2] * tl);
  // the pending cell's voxel, absolute (vc in cell units relative to the walk table)
  const int32_t vx = (vc[0] << 3) + g.w8_org[0], vy = (vc[1] << 3) + g.w8_org[1], vz = (vc[2] << 3) + g.w8_org[2];
  const int32_t dl = (vx ^ lx) | (vy ^ ly) | (vz ^ lz);
  if (w != kWalkSlow && dl >= 0 && dl < 8) {
    // An edge cell (dim 8, not interior) whose lookahead point lies in the cell itself: getDim
    // answers the cell's dim, 8 == dim, and update_current_majorant the cell's majorant.
    ln.maj = math::as_f32(w & ~kWalkEdge);
    return false;
  }
  Cell la = cell_at(g, lx, ly, lz);
  int32_t nd = hdda_dim_of(la);
  int32_t ax = vx, ay = vy, az = vz;
  const bool changed = nd != ln.dim;
  // HDDA::update(ray, dim): recomputes the voxel and the boundaries from the ray at tk
  if (changed) {
    ln.dim = nd;
    const float P[3] = {ln.e[0] + ln.d[0] * tk, ln.e[1] + ln.d[1] * tk, ln.e[2] + ln.d[2] * tk};
    int32_t V[3];
    for (int b = 0; b < 3; ++b) {
      V[b] = ((int32_t)floorf(P[b])) & (~(nd - 1));
      ln.vox[b] = (V[b] - g.w8_org[b]) >> 3;
    }
    ax = V[0];
    ay = V[1];
    az = V[2];
    for (int b = 0; b < 3; ++b) {
      // local_value: the direction is loop-invariant in the walk, and the compiler would compute
      // invDir and the step signs before the loop and hold them in registers for this rare block.
      const float db = local_value(ln.d[b]);
      const float inv = math::rcp_rn(db);  // == the ray's invDir (begin_ray / scene_finalize)
      const int32_t st = hdda_stp(db, inv);
      ln.finc[b] = (float)nd * fabsf(inv);
      ln.vinc[b] = (nd >> 3) * st;
      if (st == 0) continue;
      float n = tk + ((float)V[b] - P[b]) * inv;
      if (st > 0) n += (float)nd * inv;
      ln.nxt[b] = n;
    }
  }
  // update_current_majorant at the (new) voxel: the lookahead cell answers it when both points lie
  // in the same nd^3 block, saving a dependent load.  nd = 8: every query is a function of the
  // 8^3 cell; nd = 128 / 4096: the lookahead's cell is an upper-node tile / root tile /
  // background, which covers its whole nd^3 block.  (Here ln.dim == nd.)
  const int32_t dx = (ax ^ lx) | (ay ^ ly) | (az ^ lz);
  ln.maj = majorant_of((dx & ~(nd - 1)) == 0 ? la : cell_at(g, ax, ay, az));
  return changed;
}

// RayMajorantIterator::next's prologue for a segment that starts at the previous one's end (or the
// clip entry): d_maj = maj (volume.cpp:54) once per segment -- the steps compare their cells against it,
// and only set maj.
__host__ __device__ __forceinline__ void begin_segment(Lane& ln) {
  ln.s_t0 = ln.s_t1;
  ln.s_dmaj = ln.maj;
}

// One iteration of the do-while in RayMajorantIterator::next (volume.cpp:53-71), on the pending
// cell (the HDDA was advanced into it by the previous step or by begin_ray, see hdda_pre_advance).
// Returns true when the segment [s_t0, s_t1) with majorant s_dmaj is complete.
// Fast path: at dim 8 in an interior cell the lookahead point (within ~1 voxel of the cell) lies in a
// dim-8 cell, so getDim answers 8 == dim and HDDA::update is a no-op; the prefetched walk word answers
// both "interior?" and the majorant.
// Runs: the grid's run radii (runs8) let an interior step that keeps the majorant take the next r
// HDDA steps without loading their cells (grids with large equal-majorant regions, e.g. C2).
template <bool Runs = false>
__host__ __device__ __forceinline__ bool hdda_step(const DevGrid& g, Lane& ln) {
  const float tk = ln.Tn;  // the step's time (HDDA::step's mT0)
#if VPT_STEP_TRIM
  // The segment's end if this step ends it (tk), or T1 when the HDDA has left [t0, t1]: one select
  // instead of a copy on each path.  Nothing reads s_t1 while a segment grows (NEED_SEG has taken it).
  const bool in = tk <= ln.T1;
  ln.s_t1 = in ? tk : ln.T1;
  if (!in) return true;
#else
  if (!(tk <= ln.T1)) {
    ln.s_t1 = ln.T1;
    return true;
  }
  // The segment's end if this step ends it: nothing reads s_t1 while a segment grows (NEED_SEG has
  // taken it), and tk's register is free for the pre-advance's Tn.
  ln.s_t1 = tk;
#endif
  const uint32_t w = ln.pw;
  bool synth = false;  // a zero run r >= 1: the pre-advance derives the next word (kZeroRunMax)
  if ((int32_t)w >= 0) {
    const float m = (VPT_ZERO_RUNS && w <= kZeroRunMax) ? 0.0f : math::as_f32(w);
    ln.maj = m;
    synth = w - 1u < kZeroRunMax;
    if (Runs && m == ln.s_dmaj) {
      // an interior cell lies in the r8 table: its run radius from the unpadded index
      // r8_org = w8_org + 8 kWalkPad
      const uint32_t a = (uint32_t)(ln.vox[0] - kWalkPad), b = (uint32_t)(ln.vox[1] - kWalkPad),
                     c = (uint32_t)(ln.vox[2] - kWalkPad);
      for (int32_t r = (int32_t)g.runs8[math::mul24(math::mul24(a, (uint32_t)g.r8_n[1]) + b, (uint32_t)g.r8_n[2]) + c];
           r > 0; --r) {
        synth = false;  // the HDDA has left the cell w describes
        ++ln.n_dda;
        const float t = hdda_advance(ln);
        if (!(t <= ln.T1)) {
          ln.Tn = t;
          ln.s_t1 = ln.T1;
          return true;
        }
      }
    }
  } else {
    hdda_general(g, ln, w, tk, ln.vox);
  }
  // the next step's advance, and its cell's walk word in flight
  hdda_pre_advance(g, ln, synth);
  return ln.maj != ln.s_dmaj;  // (a NaN majorant ends its segment, as the reference's ==)
}

// Walk-loop iterations between two checks of its exit condition (the ballots).  The extra
// iterations only delay the loop's exit, never a lane's own order of operations.  C3 at 7 waves:
// 433.5 ms (1) / 427.2 (2) / 423.2 (3) / 424.1 (4); C4 139.8 / 136.5 / 137.3 / 136.5.
// Re-measured on the r02g kernel (profiles/archive/r02g_exp_walk_unroll.txt): C3 366.8-367.3 (2) / 365.2-365.8 (3)
// / 365.3-365.5 (4) ms, C4 103.1 / 102.4 / 106.3 (the temperature kernel spills at 4).
#ifndef VPT_WALK_UNROLL
#define VPT_WALK_UNROLL 3
#endif

// Wave issue priority (s_setprio) while a wavefront walks (3) and while it evaluates densities (2,
// not in the temperature kernel): the walk's loads and the evaluation's gathers issue ahead of the
// other blocks' instructions of the SIMD's other waves.  r02: C3 363.7 -> 358.3 ms (walk alone
// 361.0), C4 103.2 -> 102.3 with the walk's priority only (with the evaluation's as well: 105.6).
constexpr int kPrioWalk = 3, kPrioEval = 2;
__host__ __device__ __forceinline__ void wave_priority(int p) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (p == 0) __builtin_amdgcn_s_setprio(0);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else __builtin_amdgcn_s_setprio(3);
#else
  (void)p;
#endif
}

// Free-flight overshoot pre-test margin (SM_DRAW): RN(log2(e) * (1 + 2^-16)).
constexpr float kOvershootC = 0x1.7155e8p+0f;

// ------------------------------------------------------------------------------------------------
// Phase function helpers (random.hpp:56-84, utils.hpp:39-66)
// ------------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ void sample_hg(const DevScene& S, const float w[3], float u0, float u1, float out[3]) {
  const float g = S.g_hg;
  float cos_theta;
  if (fabsf(g) < 1e-3f) {
    cos_theta = 1 - 2 * u0;
  } else {
    // 1/(2g) * (1 + g2 - pow((1 - g2)/(1 + g - 2g u), 2)); pow(x, 2) is the correctly rounded square
    float q = S.hg_1mg2 / (S.hg_1pg - S.hg_2g * u0);
    cos_theta = S.hg_inv2g * (S.hg_1pg2 - q * q);
  }
  float sin_theta = sqrtf(fmaxf(0.0f, 1.0f - cos_theta * cos_theta));
  float phi = 2.0f * 3.14159274f * u1;
  float sc = sin_theta < -1.0f ? -1.0f : (sin_theta > 1.0f ? 1.0f : sin_theta);
  float cc = cos_theta < -1.0f ? -1.0f : (cos_theta > 1.0f ? 1.0f : cos_theta);
#ifdef VPT_SEPARATE_SINCOS
  float lx = sc * math::cosf_glibc(phi), ly = sc * math::sinf_glibc(phi), lz = cc;
#else
  float sphi, cphi;
  math::sincosf_glibc(phi, sphi, cphi);
  float lx = sc * cphi, ly = sc * sphi, lz = cc;
#endif
  float n2 = lx * lx + (ly * ly + lz * lz);  // local.normalize()
  if (n2 > 0.0f) {
    // three correctly rounded divisions by s through one reciprocal (vpt_math.h div_by_recip)
    const float s = sqrtf(n2), rs = math::recip_for_div(s);
    lx = math::div_by_recip(lx, s, rs);
    ly = math::div_by_recip(ly, s, rs);
    lz = math::div_by_recip(lz, s, rs);
  }  // coordinate_system(w, x, y)
  float sign = copysignf(1.0f, w[2]);
  float a = -1.0f / (sign + w[2]);
  float b = w[0] * w[1] * a;
  float X0 = 1.0f + sign * a * (w[0] * w[0]), X1 = sign * b, X2 = -sign * w[0];
  float Y0 = b, Y1 = sign + a * (w[1] * w[1]), Y2 = -w[1];
  out[0] = (lx * X0 + ly * Y0) + lz * w[0];
  out[1] = (lx * X1 + ly * Y1) + lz * w[1];
  out[2] = (lx * X2 + ly * Y2) + lz * w[2];
}

// henyey_greenstein(cos, g) = inv_4_pi * (1 - g*g) / (den * sqrt(max(0, den))), den = 1 + g*g + 2g cos
__host__ __device__ __forceinline__ float hg_eval(const DevScene& S, float cos_theta) {
  float den = S.hg_1pg2 + S.hg_2g * cos_theta;
  return S.hg_num / (den * sqrtf(fmaxf(0.0f, den)));
}

// Scene constants that depend on the density grid's map or on g (called once on the host).
__host__ __device__ inline void scene_finalize(DevScene& S) {
  RayDir r = ray_dir_setup(S.density, S.wi);
  for (int i = 0; i < 3; ++i) {
    S.sh_d[i] = r.d[i];
    S.sh_inv[i] = r.inv[i];
  }
  S.sh_len = r.len;
  S.sh_scale = r.scale;
  S.sh_rscale = r.rscale;
  const float g = S.g_hg;
  S.hg_g2 = g * g;
  S.hg_1pg2 = 1.0f + S.hg_g2;
  S.hg_1mg2 = 1.0f - S.hg_g2;
  S.hg_1pg = 1.0f + g;
  S.hg_2g = 2.0f * g;
  S.hg_inv2g = 1.0f / (2.0f * g);
  const float inv_4_pi = (float)(0.318309886183790671537767526745028724 / 4.0);  // float(inv_pi / 4.0)
  S.hg_num = inv_4_pi * (1.0f - g * g);
  S.sigt_c = S.sigma_t * kOvershootC;
}

// A primary ray's real-or-null collision (worker.cpp:148-188) at the index point pi with density
// dens: emission (HasTemp), then sample_discrete({Null, Absorption, Scatter}, u) with
// p_a = sigma_a*dens/sigma_maj, p_s = sigma_s*dens/sigma_maj.  u < 0: draw the event's uniform here
// (after the emission, as the reference); else u is that draw, taken by the caller.  The emission re-reads the
// scene through sp at its own point: the temperature grid's fields and the blackbody constants, loaded from the
// evaluation's copy S, were scheduled at the evaluation's start and held across the density lookup -- ~17 SGPRs
// spilled to VGPR lanes and read back (a v_writelane / v_readlane pair each) on every evaluation.
// (r04's temperature-corner prefetch, measured 2.5 % slower on C4: tools/experiments/r04_temp_prefetch.patch.)
template <bool HasTemp, bool Debug, class Env>
__host__ __device__ __forceinline__ void primary_event(ScenePtr sp, const DevScene& S, const DevGrid& G, Lane& ln, LaneCold& lc, Env& env,
                                                       float pi_x, float pi_y, float pi_z, float dens, float p_a,
                                                       float p_s, float u) {
  env.prof(PB_EVENT);
  float cp[3];
  map_fwd(G, pi_x, pi_y, pi_z, cp[0], cp[1], cp[2]);
  if (Debug) env.event(ln, VPT_EV_SAMPLED_POINT, cp, nullptr, dens);
  const float p_n = fmaxf(1.0f - p_a - p_s, 0.0f);
  if (HasTemp) {
    const DevScene St = *opaque(sp);
    float tx, ty, tz, tadim, X, Y, Z;
    map_inv(St.temperature, cp[0], cp[1], cp[2], tx, ty, tz);
#ifdef VPT_EXP_TEMP_NOCACHE
    StencilCell tc{kNoCell, 0, 0, -1};
    env.tally(CNT_TEMP_STENCILS, trilinear(St.temperature, tc, tx, ty, tz, tadim) ? 1 : 0);
#else
    env.tally(CNT_TEMP_STENCILS, trilinear(St.temperature, ln.temp_cell, tx, ty, tz, tadim) ? 1 : 0);
#endif
    float tK = tadim * St.temp_scale + St.temp_offset;
    env.blackbody(St, tK, X, Y, Z);
    float sc = p_a * St.le_scale;
    lc.L[0] = lc.L[0] + sc * X;
    lc.L[1] = lc.L[1] + sc * Y;
    lc.L[2] = lc.L[2] + sc * Z;
  }
  if (u < 0.0f) {
    u = rng_uniform(ln.rng);
    if (Debug) env.tally(CNT_RNG_DRAWS, 1);
  }
  // sample_discrete({Null p_n, Absorption p_a, Scatter p_s}, u) (random.hpp:30-47)
  float total = ((0.0f + p_n) + p_a) + p_s;
  float uu = u * total;
  int ev;
  uu -= p_n;
  if (uu <= 0) {
    ev = 0;
  } else {
    uu -= p_a;
    ev = (uu <= 0) ? 1 : 2;
  }
  if (ev == 1) {
    if (Debug) env.event(ln, VPT_EV_ABSORBED, nullptr, nullptr, 0.0f);
    ln.state = ST_FINISH_T;
  } else if (ev == 2) {
    if (lc.depth++ >= S.max_depth) {
      if (Debug) env.event(ln, VPT_EV_SCATTER_TERMINATED, nullptr, nullptr, 0.0f);
      ln.state = ST_FINISH_T;
    } else {
      if (Debug) env.tally(CNT_SCATTERS, 1);
      // The next primary ray starts at the scatter point (worker.cpp:179): keep it in ro.
      for (int i = 0; i < 3; ++i) lc.ro[i] = cp[i];
      // sample_Ld (worker.cpp:52-90)
      if (S.li_zero) {
        lc.Tr = -1.0f;  // returns Li == 0 without draws
        ln.state = ST_NEE_DONE;
      } else {
        lc.Tr = local_const(1.0f);
        ln.shadow = 1;
        ln.state = ST_SHADOW;
      }
    }
  }
  // ev == 0 (Null): keep drawing in the same segment.
  if (Debug && ev == 0) env.event(ln, VPT_EV_NULL, nullptr, nullptr, 0.0f);
  if (ev != 0) ln.sm = SM_NONE;
}

// A tentative collision at s_t0 (SM_EVAL): density, then the primary path's event
// (worker.cpp:145-188) or the shadow ray's ratio-tracking update (worker.cpp:66-85).
template <bool HasTemp, bool Debug, class Env>
__host__ __device__ __forceinline__ void eval_collision(ScenePtr sp, const DevScene& S, const DevGrid& G, Lane& ln, Env& env) {
  LaneCold& lc = env.cold();
  const float sigma_maj = ln.s_dmaj * S.sigma_t;
  {
    // The draw's exact free-flight distance, deferred from SM_DRAW (majorant_transmittance_sampler.cpp:44-45):
    // dt = -log(1 - u) / sigma_maj (random.hpp:20-22), t = t0 + dt / m_scale.
    const float dt_m = -math::logf_glibc_unit(lc.y_draw, env.logf_table()) / sigma_maj;
    const float tc = ln.s_t0 + math::div_by_recip(dt_m, ln.scale, ln.rscale);  // == dt_m / m_scale
    if (!(tc < ln.s_t1)) {  // overshoot after all: drop the segment
      ln.sm = SM_NEED_SEG;
      return;
    }
    ln.s_t0 = tc;  // the tentative collision
  }
  env.prof(PB_TRILINEAR);
  const float t = ln.s_t0;
  float pi_x = ln.e[0] + ln.d[0] * t, pi_y = ln.e[1] + ln.d[1] * t, pi_z = ln.e[2] + ln.d[2] * t;
  float dens;
  if (Debug) env.tally(CNT_DENSITY_EVALS, 1);
  env.tally(CNT_STENCILS, trilinear(G, lc.dens_cell, pi_x, pi_y, pi_z, dens) ? 1 : 0);
  ln.sm = SM_DRAW;  // density <= 0, a null event or an unkilled shadow ray: keep drawing
  if (dens > 0.0f) {
    if (!HasTemp) {
      // Primary rays (worker.cpp:145-188) and shadow rays (worker.cpp:66-85) share the division by
      // sigma_maj and the one uniform draw, so a wavefront holding both kinds runs one division
      // and one RNG sequence instead of two: q1 is p_a for a primary ray and sigma_n / sigma_maj
      // for a shadow ray; the draw is the event's (primary) or the Russian roulette's (shadow,
      // only when T_ray <= 0.05).  Each lane's operations and draws are the reference's, in order.
      // (Measured: C3 +1 %; the temperature kernel keeps the two branches, where it cost 1.6 %.)
      const bool sh = ln.shadow != 0;
      const float sigma_n = fmaxf(0.0f, sigma_maj - S.sigma_t * dens);
      const float q1 = (sh ? sigma_n : S.sigma_a * dens) / sigma_maj;
      const float tr = lc.Tr * q1;  // shadow: T_ray *= sigma_n / sigma_maj
      const bool draw = !sh || tr <= 0.05f;
      float u = 0.0f;
      if (draw) {
        u = rng_uniform(ln.rng);
        if (Debug) env.tally(CNT_RNG_DRAWS, 1);
      }
      if (!sh) {
        primary_event<HasTemp, Debug>(sp, S, G, ln, lc, env, pi_x, pi_y, pi_z, dens, q1, (S.sigma_s * dens) / sigma_maj, u);
      } else {
        env.prof(PB_SHADOW_HIT);
        float T = tr;  // Russian roulette, q = 0.75
        if (draw) T = (u < 0.75f) ? 0.0f : T / (1 - 0.75f);
        lc.Tr = T;
        if (T <= 0.0f) {
          lc.Tr = -1.0f;  // returns Zero()
          ln.state = ST_NEE_DONE;
          ln.sm = SM_NONE;
        }
      }
    } else if (!ln.shadow) {
      // worker.cpp:148-188
      const float p_a = (S.sigma_a * dens) / sigma_maj;
      const float p_s = (S.sigma_s * dens) / sigma_maj;
      primary_event<HasTemp, Debug>(sp, S, G, ln, lc, env, pi_x, pi_y, pi_z, dens, p_a, p_s, -1.0f);
    } else {
      env.prof(PB_SHADOW_HIT);
      // Ratio tracking with Russian roulette (worker.cpp:68-85)
      float sigma_n = fmaxf(0.0f, sigma_maj - S.sigma_t * dens);
      lc.Tr *= sigma_n / sigma_maj;
      if (lc.Tr <= 0.05f) {
        float q = 0.75f;
        if (Debug) env.tally(CNT_RNG_DRAWS, 1);
        if (rng_uniform(ln.rng) < q)
          lc.Tr = 0.0f;
        else
          lc.Tr /= 1 - q;
      }
      if (lc.Tr <= 0.0f) {
        lc.Tr = -1.0f;  // returns Zero()
        ln.state = ST_NEE_DONE;
        ln.sm = SM_NONE;
      }
    }
  }
}

// Scheduling order over a whole-wave range (never changes a job's samples, which its jid keys):
// item k -> job (wave w, tile order[i]) with `order` = tiles by descending estimated cost.
// Items before tail_k0 (= whole waves x T) run wave by wave, each wave costliest tile first.  The
// last tail_n waves run as one costliest-first list, so the launch drains on cheap (sky) jobs: the
// rank list is cut into groups of `group` tiles and a group's tail_n waves are consecutive items, wave
// by wave.  group 64 (VPT_ORDER_COST_TAIL / _TILE_MAJOR): the 64 lanes of a wavefront trace 64 different
// tiles (one tile per lane would put the wavefront's film atomics on the same 64 addresses).  group 1
// (VPT_ORDER_COST_SAME_TILE, tail_n = every wave, ordered-film launches only): one tile's waves
// consecutively -- a wavefront's lanes trace the same 64 pixels, and their rays walk the same cells.
constexpr uint32_t kOrderGroup = 64;
__host__ __device__ __forceinline__ uint64_t ordered_job(uint32_t k, uint32_t T, const uint32_t* order, uint32_t tail_k0,
                                                         uint32_t tail_n, uint32_t group) {
  if (k < tail_k0) {
    const uint32_t w = k / T;
    return (uint64_t)w * T + order[k - w * T];
  }
  k -= tail_k0;
  const uint32_t full = T / group, span = group * tail_n;
  uint32_t w, i;
  if (k < full * span) {
    const uint32_t g = k / span, r = k - g * span;
    w = r / group;
    i = g * group + (r - w * group);
  } else {  // (never with group 1: full * span covers the tail)
    const uint32_t R = T - full * group, r = k - full * span;
    w = r / R;
    i = full * group + (r - w * R);
  }
  return (uint64_t)(tail_k0 / T + w) * T + order[i];
}

// ------------------------------------------------------------------------------------------------
// One iteration of the lane loop.  Env supplies fetch_job(uint64_t& item, wave_lanes) -> bool, jid_begin, the
// job order (order == nullptr: item k is job jid_begin + k; else ordered_job()),
// film_add(S, lane, px, py, rw).  HasTemp: the scene has a temperature grid (fire).
// Debug: keep every counter and the job index (per-sample records).
// ------------------------------------------------------------------------------------------------

template <bool HasTemp, bool Debug, bool Runs, class Env>
__host__ __device__ __forceinline__ void lane_iteration(ScenePtr sp, Lane& ln, Env& env) {
  env.prof(PB_ITER);
  LaneCold& lc = env.cold();
  // Every block reads the scene constants it needs afresh (scalar loads behind opaque(), see
  // ScenePtr): nothing stays live in SGPRs across the whole loop, so the walk keeps its own.
  int32_t gate_min;
  bool starving;
  {
    const DevScene S = *opaque(sp);
    gate_min = S.gate_min;
    // Lanes of the wavefront sampling right now; rare states run when enough lanes wait for them
    // or the wavefront is short of sampling work (never changes a lane's own operation order).
    const int32_t n_walking = env.count(ln.state == ST_SAMPLE && ln.sm != SM_EVAL);
    starving = n_walking < S.gate_idle;
  }
  auto go = [&](int32_t st) -> bool {
    const int32_t n = env.count(ln.state == st);
    return n > 0 && (starving || n >= gate_min) && ln.state == st;
  };
  auto go2 = [&](int32_t st_a, int32_t st_b) -> bool {
    const bool mine = ln.state == st_a || ln.state == st_b;
    const int32_t n = env.count(mine);
    return n > 0 && (starving || n >= gate_min) && mine;
  };
  // Block order follows the state flow so a lane moves on within one pass where it can:
  // NEE completion / film write -> next job / pixel -> ray setup -> walk -> density evaluation.

  {
    const DevScene S = *opaque(sp);
    const DevGrid& G = S.density;
    (void)G;
    if (go(ST_NEE_DONE)) {
      env.prof(PB_NEE_DONE);
      if (lc.Tr >= 0.0f) {
        // p * T_ray * Li with p = HG(w . wi)
        float c = lc.rd[0] * S.wi[0] + (lc.rd[1] * S.wi[1] + lc.rd[2] * S.wi[2]);
        float p = hg_eval(S, c);
        float pt = p * lc.Tr;
        lc.L[0] = lc.L[0] + pt * S.Li[0];
        lc.L[1] = lc.L[1] + pt * S.Li[1];
        lc.L[2] = lc.L[2] + pt * S.Li[2];
      } else {
        // L + 0.0f (sample_Ld returned zero): the same value as L for every L but -0.0, which it
        // turns into +0.0 -- written as a select, so no register holds a constant for it.
        lc.L[0] = lc.L[0] == 0.0f ? 0.0f : lc.L[0];
        lc.L[1] = lc.L[1] == 0.0f ? 0.0f : lc.L[1];
        lc.L[2] = lc.L[2] == 0.0f ? 0.0f : lc.L[2];
      }
      float u0 = rng_uniform(ln.rng);
      float u1 = rng_uniform(ln.rng);
      if (Debug) env.tally(CNT_RNG_DRAWS, 2);
      float nd[3];
      sample_hg(S, lc.rd, u0, u1, nd);
      for (int i = 0; i < 3; ++i) lc.rd[i] = nd[i];
      if (Debug) env.event(ln, VPT_EV_SCATTER, lc.ro, lc.rd, 0.0f);
      ++lc.depth;  // the for-loop increment (worker.cpp:130)
      ln.shadow = 0;
      ln.state = ST_RAY;
    }
  }
  env.tick(PT_NEE);
  {
    const DevScene S = *opaque(sp);
    const DevGrid& G = S.density;
    (void)G;
    const bool fin = go2(ST_FINISH, ST_FINISH_T);
    if (fin) {
      env.prof(PB_FINISH);
      if (ln.state == ST_FINISH) {  // not terminated (worker.cpp:198-200)
        lc.L[0] = lc.L[0] + S.le_inf[0];
        lc.L[1] = lc.L[1] + S.le_inf[1];
        lc.L[2] = lc.L[2] + S.le_inf[2];
      }
      // the pixel just traced is pix - 1 of the tile
      const int32_t rw = min(S.W - lc.x0, S.tw);
      const int32_t q = (lc.pix & kPixelMask) - 1, y = div_pix(q, rw);
      env.film_add(S, ln, lc.x0 + (q - y * rw), lc.y0 + y, rw);
      env.tally(CNT_SAMPLES, 1);
      ln.state = ST_PIXEL;
    }
    env.film_commit(S, fin);  // (the converged wavefront: see KernelEnvT::film_add)
  }
  env.tick(PT_FINISH);
  {
    const DevScene S = *opaque(sp);
    const DevGrid& G = S.density;
    (void)G;
    // (a feed lane holding an unread item runs the block at once: its ring slot is pinned until it reads it)
    const int32_t n_fetch = env.count(ln.state == ST_FETCH);
    if (n_fetch > 0 && (starving || n_fetch >= gate_min || env.fetch_urgent(ln.state == ST_FETCH)) &&
        ln.state == ST_FETCH) {
      env.prof(PB_FETCH);
      uint64_t j;
      // 1: job j (an item index, or a job id in the feed mode); 0: no more work; < 0 (feed mode): the lane
      // holds an item the host has not published yet -- it stays in ST_FETCH and asks again
      const int got = (int)env.fetch_job(j, S.wave_lanes);
      if (got <= 0) {
        if (got == 0) ln.state = ST_DONE;
        return;
      }
      uint32_t p = 0;
      if (S.pixel_mode) {  // throughput mode: item = job * tile_area + pixel, taken pixel_chunk at a time
        j *= env.args()->pixel_chunk;
        p = (uint32_t)(j % S.tile_area);
        j /= S.tile_area;
      }
      if (const uint32_t* const perm = env.args()->perm)
        j = perm[j];
      else if (const uint32_t* const order = env.args()->order)
        j = ordered_job((uint32_t)j, (uint32_t)S.T, order, env.args()->order_tail_k0, env.args()->order_tail_n,
                        env.args()->order_group);
      if (Debug) {
        ln.jid_local = j;
        ln.n_events = 0;
      }
#ifdef VPT_JOB_LOG
      lc.job = (uint32_t)j;
      lc.t_start = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
      uint64_t jid = env.args()->jid_begin + j;
      if (S.pixel_mode) {  // each pixel's stream is seeded when the pixel starts (ST_PIXEL)
        const uint64_t base = jid * S.tile_area;
        lc.item_lo = (uint32_t)base;
        lc.item_hi = (uint32_t)(base >> 32);
      } else {
        ln.rng = job_seed(S.seed, jid);
        lc.item_lo = (uint32_t)j;  // the job's index in the launch: its slot in the ordered film's samples
        env.job_start(S, lc, jid);  // (a feed launch with an ordered frame: the job's slot there)
      }
      uint64_t tile = jid % S.T;
      lc.x0 = (int32_t)(tile % S.ntx) * S.tw;  // TileProvider::compute_tile_rect
      lc.y0 = (int32_t)(tile / S.ntx) * S.th;
      lc.pix = S.pixel_mode ? (int32_t)p | kOnePixel : 0;
      if (HasTemp) {
        ln.temp_cell.i = kNoCell;
        ln.temp_cell.code = -1;
      }
      ln.state = ST_PIXEL;
    }
  }
  env.tick(PT_FETCH);
  {
    const DevScene S = *opaque(sp);
    const DevGrid& G = S.density;
    (void)G;
    if (go(ST_PIXEL)) {
      env.prof(PB_PIXEL);
      // Clipped tile extent (tile_provider.cpp:102): recomputed, not stored.
      const int32_t rw = min(S.W - lc.x0, S.tw);
      const int32_t rh = min(S.H - lc.y0, S.th);
      // Skip pixels filtered by single_pixel mode without any draw (worker.cpp:113-116).
      int32_t px, py;
      const int32_t one = lc.pix & kOnePixel;
      int32_t q = lc.pix & kPixelMask;
      // Throughput mode: the lane's chunk of pixel_chunk pixels (a power of two dividing the tile area; chunk
      // starts are multiples of it) ends at the next multiple once a pixel of it has been taken.
      const int32_t K = (int32_t)env.args()->pixel_chunk;
      const int32_t end = one ? (((lc.pix & kPixelTaken) && (q & (K - 1)) == 0) ? 0 : min((q & ~(K - 1)) + K, rw * rh))
                              : rw * rh;
      while (true) {
        if (q >= end) {
#ifdef VPT_JOB_LOG
          env.job_done(lc.job, (uint32_t)((lc.x0 / S.tw) + (lc.y0 / S.th) * S.ntx), lc.t_start);
#endif
          env.job_end(S, lc);
          ln.state = ST_FETCH;
          return;
        }
        int32_t y = div_pix(q, rw);
        px = lc.x0 + (q - y * rw);
        py = lc.y0 + y;
        ++q;
        lc.pix = q | (one ? (kOnePixel | kPixelTaken) : 0);
        if (!S.single_pixel_enabled || (px == S.sp_x && py == S.sp_y)) break;
      }
      if (one)  // throughput mode: the pixel's own stream, hash(seed, jid * tile_area + pixel)
        ln.rng = job_seed(S.seed, (((uint64_t)lc.item_hi << 32) | lc.item_lo) + (uint64_t)(q - 1));
      float jx = rng_uniform(ln.rng);
      float jy = rng_uniform(ln.rng);
      if (Debug) env.tally(CNT_RNG_DRAWS, 2);
      jx *= S.jitter_scale;
      jy *= S.jitter_scale;
      // Camera::generate_ray (camera.hpp:14-23)
      float rx = ((float)px + 0.5f) + jx, ry = ((float)py + 0.5f) + jy;
      float dv[3];
      for (int i = 0; i < 3; ++i) dv[i] = S.cam_t[i] + (S.cam_L[i * 3] * rx + (S.cam_L[i * 3 + 1] * ry + S.cam_L[i * 3 + 2] * 0.0f));
      float n2 = dv[0] * dv[0] + (dv[1] * dv[1] + dv[2] * dv[2]);
      if (n2 > 0.0f) {
        const float s = math::sqrt_rn(n2), rs = math::recip_for_div(s);
        dv[0] = math::div_by_recip(dv[0], s, rs);
        dv[1] = math::div_by_recip(dv[1], s, rs);
        dv[2] = math::div_by_recip(dv[2], s, rs);
      }
      for (int i = 0; i < 3; ++i) {
        lc.ro[i] = S.cam_pos[i];
        lc.rd[i] = dv[i];
        lc.L[i] = 0.0f;
      }
      lc.depth = 0;
      ln.shadow = 0;
      ln.state = ST_RAY;
      if (Debug) env.event(ln, VPT_EV_NEW_RAY, lc.ro, lc.rd, 0.0f);
    }
  }
  env.tick(PT_PIXEL);
  {
    const DevScene S = *opaque(sp);
    const DevGrid& G = S.density;
    (void)G;
    // Volume::intersect + iterator setup for primary rays (top of the depth loop, worker.cpp:122-126)
    // and sample_Ld's shadow rays (worker.cpp:64-65, direction wi: scene constants) in one block.
    if (go2(ST_RAY, ST_SHADOW)) {
      env.prof(PB_RAY);
      const bool primary = ln.state == ST_RAY;
      if (primary && !(lc.depth < S.max_depth)) {
        ln.state = ST_FINISH;  // for (depth < max_depth) exhausted
      } else {
        RayDir rd;
        if (primary) {
          rd = ray_dir_setup(G, lc.rd);
        } else {
          for (int i = 0; i < 3; ++i) {
            rd.d[i] = S.sh_d[i];
            rd.inv[i] = S.sh_inv[i];
          }
          rd.len = S.sh_len;
          rd.scale = S.sh_scale;
          rd.rscale = S.sh_rscale;
        }
        lc.dens_cell.i = kNoCell;  // a new sampler (and its stencil cache) per ray
        lc.dens_cell.code = -1;
        if (begin_ray(G, ln, lc.ro, rd)) {
          if (Debug && !primary) env.tally(CNT_SHADOW_RAYS, 1);
          ln.state = ST_SAMPLE;
        } else {
          // a primary miss ends the path; a shadow miss keeps T_ray = 1
          ln.state = primary ? ST_FINISH : ST_NEE_DONE;
        }
      }
    }
  }
  env.tick(PT_RAY);
  {
    const DevScene S = *opaque(sp);
    const DevGrid& G = S.density;
    (void)G;
#ifdef VPT_PROFILE
    const int32_t c_nee = env.count(ln.state == ST_NEE_DONE), c_fin = env.count(ln.state == ST_FINISH || ln.state == ST_FINISH_T),
                  c_ray = env.count(ln.state == ST_RAY || ln.state == ST_SHADOW),
                  c_pix = env.count(ln.state == ST_PIXEL || ln.state == ST_FETCH), c_done = 64 - env.count(true);
#endif
    if (ln.state == ST_SAMPLE) {
      env.prof(PB_SAMPLE);
      // The walk (segment fetch, HDDA step, free-flight draw) loops here while enough lanes of the
      // wavefront are walking and too few wait on a density evaluation; the other states wait
      // (their gating counts them next outer iteration).  Each lane's own op order is unchanged.
      wave_priority(kPrioWalk);
      do {
#if VPT_WALK_UNROLL > 1
#pragma unroll
      for (int rep = 0; rep < VPT_WALK_UNROLL; ++rep) {
#endif
#ifdef VPT_PROFILE
      env.prof_add(PB_W_WALK, env.count(ln.state == ST_SAMPLE && ln.sm != SM_EVAL));
      env.prof_add(PB_W_EVAL, env.count(ln.state == ST_SAMPLE && ln.sm == SM_EVAL));
      env.prof_add(PB_W_NEE, c_nee);
      env.prof_add(PB_W_FIN, c_fin);
      env.prof_add(PB_W_RAY, c_ray);
      env.prof_add(PB_W_PIX, c_pix);
      env.prof_add(PB_W_DONE, c_done);
#endif
      if (ln.sm == SM_NEED_SEG) {
        env.prof(PB_NEED_SEG);
        // RayMajorantIterator::next prologue (volume.cpp:40-51)
        // the sampler's position is the previous segment's end (or the clip entry, begin_ray)
        if (ln.s_t1 >= ln.T1) {
          // the sampler ran dry: a shadow ray keeps T_ray; a primary ray did not scatter (break)
          ln.state = ln.shadow ? ST_NEE_DONE : ST_FINISH;
          ln.sm = SM_NONE;
          env.prof(PB_NONE);
        } else {
          begin_segment(ln);
          ln.sm = SM_STEP;
        }
      }
      env.tick(PT_SEG);
      if (ln.sm == SM_STEP) {
        env.prof(PB_STEP);
        ++ln.n_dda;
        if (hdda_step<Runs>(G, ln)) {
          if (Debug) env.tally(CNT_SEGMENTS, 1);
          ln.sm = (ln.s_dmaj <= 0.0f) ? SM_NEED_SEG : SM_DRAW;  // empty segment: no draw (:32-35)
        }
      }
      env.tick(PT_STEP);
      if (ln.sm == SM_DRAW) {
        env.prof(PB_DRAW);
        // MajorantTransmittanceSampler::next body (majorant_transmittance_sampler.cpp:39-79).  Most draws
        // overshoot the segment (C3: 45 of 57 per sample) and their distance is never used, so the
        // draw only proves the overshoot with the hardware log2: a = -v_log_f32(1 - u) satisfies
        // a*ln2 <= X*(1 + 2.71*2^-24) for X = -logf(1 - u) as the exact path computes it, over every
        // 1 - u (tools/proofs/log2_bound.hip).  With kOvershootC = log2(e)*(1 + 2^-16) rounded, a >
        // thr = (s_t1 - s_t0)*sigma_maj*m_scale*kOvershootC then implies RN(s_t0 + RN(RN(X/sigma_maj)
        // /m_scale)) >= s_t1 (every rounding is covered by the 2^-16 margin, whatever the order of the
        // four products: thr is computed as ((s_t1 - s_t0)*RN(d_maj*RN(sigma_t*kOvershootC)))*m_scale, three
        // roundings of 2^-24 each against 2^-16; the guards keep the intermediate results normal:
        // m_scale in [2^-26, 2^26) via rscale, s_t1 - s_t0 >= 2^-96).
        // Anything else parks in SM_EVAL, which computes the exact distance first (eval_collision).
#if VPT_STEP_TRIM
        const float y = rng_one_minus_uniform(ln.rng);
#else
        const float y = 1 - rng_uniform(ln.rng);
#endif
        if (Debug) {
          env.tally(CNT_DRAWS, 1);
          env.tally(CNT_RNG_DRAWS, 1);
        }
        const float D = ln.s_t1 - ln.s_t0;
        const float thr = (D * (ln.s_dmaj * S.sigt_c)) * ln.scale;
        if (math::neg_log2_hw(y) > thr && D >= 0x1p-96f && ln.rscale == ln.rscale) {
          ln.sm = SM_NEED_SEG;
        } else {
          lc.y_draw = y;
          ln.sm = SM_EVAL;
        }
      }
      env.tick(PT_DRAW);
#if VPT_WALK_UNROLL > 1
      }
#endif
      } while (S.gate_walk > 0 && env.count(ln.state == ST_SAMPLE && ln.sm != SM_EVAL) >= S.gate_walk &&
               env.count(ln.state == ST_SAMPLE && ln.sm == SM_EVAL) < S.gate_eval);
      wave_priority(0);
    }
  }
  env.tick(PT_WALK);
  {
    const DevScene S = *opaque(sp);
    const DevGrid& G = S.density;
    (void)G;
    // Tentative collisions wait until gate_eval lanes of the wavefront have one (or the walk runs
    // short of lanes), so the stencil gathers and the event logic run on a fuller wavefront.
    const int32_t n_eval = env.count(ln.state == ST_SAMPLE && ln.sm == SM_EVAL);
    const bool run_eval = n_eval > 0 && (n_eval >= S.gate_eval || env.count(ln.state == ST_SAMPLE && ln.sm != SM_EVAL) < S.gate_idle);
    if (!HasTemp && run_eval) wave_priority(kPrioEval);
    if (run_eval && ln.state == ST_SAMPLE && ln.sm == SM_EVAL) eval_collision<HasTemp, Debug>(sp, S, G, ln, env);
    if (!HasTemp) wave_priority(0);
  }
  env.tick(PT_EVAL);
}

__host__ __device__ __forceinline__ void lane_init(Lane& ln) {
  ln.state = ST_FETCH;
  ln.sm = SM_NONE;
  ln.shadow = 0;
  ln.temp_cell.i = kNoCell;
  ln.temp_cell.code = -1;
  ln.n_dda = 0;
}
__host__ __device__ __forceinline__ void cold_init(LaneCold& lc) {
  lc.dens_cell.i = kNoCell;
  lc.dens_cell.code = -1;
  lc.pix = 0;  // (a feed-mode launch reads it before the first fetch)
}

}  // namespace vpt
