// vpt_math.h — float transcendentals that reproduce glibc bit for bit on the integrator's inputs.
//
// The reference calls std::log / std::sin / std::cos on floats (random.hpp:21, :71-72), i.e.
// glibc logf/sinf/cosf (glibc >= 2.28: the ARM optimized-routines algorithms; x86-64 selects the
// -mfma build of the same C source at run time).  On the GPU, ocml's versions differ from glibc in
// 1-4% of the integrator's inputs, and one flipped bit in a free-flight distance decorrelates
// the whole path.  These are the same algorithms (same tables, same double-precision operation
// sequence with fused multiply-adds), so the GPU's IEEE double arithmetic gives glibc's results.
// tests/test_math_clone.py checks them against the host's glibc over EVERY input the integrator
// can produce (1 - u and 2*pi*u for all 2^24+ values of uniform<float>()).
//
// Used by device code (the integrator kernel) and, through the same header, by a host test.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vpt {
namespace math {

__host__ __device__ __forceinline__ uint32_t as_u32(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return u;
}
__host__ __device__ __forceinline__ float as_f32(uint32_t u) {
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}
// a * b for a, b < 2^24 (v_mul_u32_u24: full rate, where a 32-bit multiply is quarter rate)
__host__ __device__ __forceinline__ uint32_t mul24(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul24(a, b);
#else
  return a * b;
#endif
}

// The double coefficients below, on the device, are read at each use from constant memory through an
// opaque pointer (scalar loads into SGPR pairs).  As literals the compiler hoists them out of the
// integrator's state-machine loop into VGPR pairs held for the whole kernel (r02: 4 VGPRs plus an
// 8-byte spill in the 72-VGPR production kernel).
enum : int { MK_LN2, MK_A0, MK_A1, MK_A2, MK_HPI_INV, MK_HPI, MK_C1, MK_C2, MK_C3, MK_C4, MK_S1, MK_S2, MK_S3, MK_COUNT };
#if defined(__HIP_DEVICE_COMPILE__)
static __constant__ double kMathK[MK_COUNT] = {
    0x1.62e42fefa39efp-1,                                                        // Ln2
    -0x1.00ea348b88334p-2, 0x1.5575b0be00b6ap-2, -0x1.ffffef20a4123p-2,            // logf A0..A2
    0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,                                  // 1/(pi/2) scaled, pi/2
    -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16,  // cos c1..c4
    -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13};         // sin s1..s3
__device__ __forceinline__ double mk(int i) {
  const __attribute__((address_space(4))) double* p = (const __attribute__((address_space(4))) double*)(const double*)kMathK;
  asm volatile("" : "+s"(p));
  return p[i];
}
#define VPT_MK(i, v) ::vpt::math::mk(i)
#else
#define VPT_MK(i, v) (v)
#endif

// logf: LOGF_TABLE_BITS = 4, polynomial order 4 (glibc sysdeps/ieee754/flt-32/e_logf.c).
// Table entries: 1/c and log(c) for the 16 sub-intervals of [0x3f330000, 2*0x3f330000).
// A memory-resident constexpr table (emitted as device constant data): a per-lane indexed load
// instead of a 16-way select chain that would hold all 32 doubles in registers.
static constexpr double kLogfTab[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010b0p+0, -0x1.01eae7f513a67p-2}, {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8ea0p+0, -0x1.1aa2bc79c8100p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aa0p-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d224770p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};

// glibc logf for x > 0 finite (the integrator only takes log(1 - u), u in [0, 1 - 2^-24]).
__host__ __device__ __forceinline__ float logf_glibc(float x) {
  const double Ln2 = 0x1.62e42fefa39efp-1;
  const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
  uint32_t ix = as_u32(x);
  if (ix == 0x3f800000u) return 0.0f;
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
    // zero / subnormal / inf / nan / negative
    if (ix * 2 == 0) return -__builtin_inff();
    if (ix == 0x7f800000u) return x;
    if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return __builtin_nanf("");
    ix = as_u32(x * 0x1p23f);
    ix -= 23u << 23;
  }
  uint32_t tmp = ix - 0x3f330000u;
  int i = (int)((tmp >> (23 - 4)) % 16u);
  int k = (int32_t)tmp >> 23;
  uint32_t iz = ix - (tmp & (0x1ffu << 23));
  const double invc = kLogfTab[i][0], logc = kLogfTab[i][1];
  double z = (double)as_f32(iz);
  double r = __builtin_fma(z, invc, -1.0);
  double y0 = __builtin_fma((double)k, Ln2, logc);
  double r2 = r * r;
  double y = __builtin_fma(A1, r, A2);
  y = __builtin_fma(A0, r2, y);
  y = __builtin_fma(y, r2, y0 + r);
  return (float)y;
}

// The integrator only takes log(1 - u), u = uniform<float>() in [0, 1 - 2^-24], so x is a normal
// float in [2^-24, 1]: glibc's special-case branches (zero, subnormal, inf, nan, x == 1 rounding-mode
// sign) never fire and are omitted (x == 1 gives +0 on the main path too).  Checked against glibc
// over every such x by tests/test_math_clone.py.
// tab: the kLogfTab values (the kernel passes its LDS copy: an LDS read instead of a vector-memory
// load, which would count in vmcnt with the walk's loads).
__host__ __device__ __forceinline__ float logf_glibc_unit(float x, const double (*tab)[2] = kLogfTab) {
  const double Ln2 = VPT_MK(MK_LN2, 0x1.62e42fefa39efp-1);
  const double A0 = VPT_MK(MK_A0, -0x1.00ea348b88334p-2), A1 = VPT_MK(MK_A1, 0x1.5575b0be00b6ap-2),
               A2 = VPT_MK(MK_A2, -0x1.ffffef20a4123p-2);
  const uint32_t ix = as_u32(x);
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> (23 - 4)) % 16u);
  const int k = (int32_t)tmp >> 23;
  const uint32_t iz = ix - (tmp & (0x1ffu << 23));
  const double invc = tab[i][0], logc = tab[i][1];
  const double z = (double)as_f32(iz);
  const double r = __builtin_fma(z, invc, -1.0);
  const double y0 = __builtin_fma((double)k, Ln2, logc);
  const double r2 = r * r;
  double y = __builtin_fma(A1, r, A2);
  y = __builtin_fma(A0, r2, y);
  y = __builtin_fma(y, r2, y0 + r);
  return (float)y;
}

// sinf / cosf (glibc sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h), for |x| < 120.
// glibc's __sincosf_table[1] is table[0] with the cosine coefficients negated; since
// fma(a, -b, -c) == -fma(a, b, c) exactly, using table[0] and negating the cosine result when
// (n & 2) gives bit-identical values without selecting between two coefficient sets.
namespace sc {
constexpr double hpi_inv = 0x1.45f306dc9c883p+23, hpi = 0x1.921fb54442d18p+0;
constexpr double c0 = 0x1p0, c1 = -0x1.ffffffd0c621cp-2, c2 = 0x1.55553e1068f19p-5, c3 = -0x1.6c087e89a359dp-10,
                 c4 = 0x1.99343027bf8c3p-16;
constexpr double s1 = -0x1.555545995a603p-3, s2 = 0x1.1107605230bc4p-7, s3 = -0x1.994eb3774cf24p-13;
}  // namespace sc
__host__ __device__ __forceinline__ uint32_t abstop12(float x) { return (as_u32(x) >> 20) & 0x7ff; }
// sinf_poly(x, x2, table[neg], n): n even -> sine polynomial, odd -> cosine polynomial.
__host__ __device__ __forceinline__ float sinf_poly(double x, double x2, bool neg_cos, int n) {
  if ((n & 1) == 0) {
    double x3 = x * x2;
    double s1 = __builtin_fma(x2, VPT_MK(MK_S3, sc::s3), VPT_MK(MK_S2, sc::s2));
    double x7 = x3 * x2;
    double s = __builtin_fma(x3, VPT_MK(MK_S1, sc::s1), x);
    return (float)__builtin_fma(x7, s1, s);
  }
  double x4 = x2 * x2;
  double c2 = __builtin_fma(x2, VPT_MK(MK_C4, sc::c4), VPT_MK(MK_C3, sc::c3));
  double c1 = __builtin_fma(x2, VPT_MK(MK_C1, sc::c1), sc::c0);
  double x6 = x4 * x2;
  double c = __builtin_fma(x4, VPT_MK(MK_C2, sc::c2), c1);
  double r = __builtin_fma(x6, c2, c);
  return (float)(neg_cos ? -r : r);
}
__host__ __device__ __forceinline__ double reduce_fast(double x, int* np) {
  double r = x * VPT_MK(MK_HPI_INV, sc::hpi_inv);
  int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return __builtin_fma(-(double)n, VPT_MK(MK_HPI, sc::hpi), x);
}
// sign[4] = {1, -1, -1, 1}
__host__ __device__ __forceinline__ double quadrant_sign(int n) { return ((n + 1) & 2) ? -1.0 : 1.0; }
// Valid for finite |y| < 120 (the integrator calls it with phi = 2*pi*u in [0, 2*pi)).
__host__ __device__ __forceinline__ float sinf_glibc(float y) {
  double x = y;
  if (abstop12(y) < 0x3f4u) {  // abstop12(pi/4)
    double s = x * x;
    if (abstop12(y) < 0x398u) return y;  // abstop12(0x1p-12f)
    return sinf_poly(x, s, false, 0);
  }
  int n;
  x = reduce_fast(x, &n);
  double s = quadrant_sign(n);
  return sinf_poly(x * s, x * x, (n & 2) != 0, n);
}
__host__ __device__ __forceinline__ float cosf_glibc(float y) {
  double x = y;
  if (abstop12(y) < 0x3f4u) {
    double x2 = x * x;
    if (abstop12(y) < 0x398u) return 1.0f;
    return sinf_poly(x, x2, false, 1);
  }
  int n;
  x = reduce_fast(x, &n);
  double s = quadrant_sign(n);
  return sinf_poly(x * s, x * x, (n & 2) != 0, n ^ 1);
}
// sinf and cosf of one argument with one range reduction and each polynomial evaluated once:
// sinf uses the sine polynomial for even quadrants and the cosine one for odd, cosf the reverse,
// on the same reduced argument, so selecting between the two gives both functions' exact values.
__host__ __device__ __forceinline__ void sincosf_glibc(float y, float& sn, float& cs) {
  double x = y, xs = y;
  int n = 0;
  if (abstop12(y) >= 0x3f4u) {
    x = reduce_fast(x, &n);
    xs = x * quadrant_sign(n);
  }
  const double x2 = x * x;
  const float ps = sinf_poly(xs, x2, false, 0);
  const float pc = sinf_poly(xs, x2, (n & 2) != 0, 1);
  sn = (n & 1) ? pc : ps;
  cs = (n & 1) ? ps : pc;
  if (abstop12(y) < 0x398u) {
    sn = y;
    cs = 1.0f;
  }
}

// ---- exact short sequences for 1/x, sqrt(x) and a/b ------------------------------------------
// The IEEE-correct f32 division and square root macros cost ~19 and ~22 v_add_f32 issue slots on
// gfx950 (tools/ubench).  These produce the same bits with a few instructions inside the guarded
// ranges, and fall back to the correct operation outside them:
// * rcp_rn:  y0 = v_rcp_f32(x); RN(1/x) = fma(fma(-x, y0, 1), y0, y0) for every x with exponent
//            field in [1, 252] (|x| in [2^-126, 2^126));
// * sqrt_rn: y = v_rsq_f32(x); s = x*y; RN(sqrt x) = fma(fma(-s, s, x), 0.5*y, s) for every
//            finite x >= 2^-101;
//   both checked on MI355X over all 2^32 inputs (tools/proofs/rcp_sqrt.hip: 0 mismatches there);
// * div_by_recip: Markstein's correction  q = RN(a*y); RN(a/b) = RN(q + fma(-q, b, a)*y)  with
//   y = RN(1/b), exact for every pair of normal a, b with normal quotient -- checked over all 2^46
//   significand pairs (tools/proofs/recip_div.hip).  Guard: b in [2^-26, 2^26) (via recip_for_div)
//   and |q| in [2^-100, 2^100) keep a, y, q normal; otherwise the division runs.
// Host builds use the plain operations (which these equal).
__host__ __device__ __forceinline__ float rcp_rn(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (((as_u32(x) >> 23) & 0xffu) - 1u < 252u) {
    const float y0 = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(__builtin_fmaf(-x, y0, 1.0f), y0, y0);
  }
#endif
  return 1.0f / x;
}
__host__ __device__ __forceinline__ float sqrt_rn(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (as_u32(x) - 0x0d000000u < 0x7f800000u - 0x0d000000u) {  // finite, positive, >= 2^-101
    const float y = __builtin_amdgcn_rsqf(x);
    const float s = x * y;
    return __builtin_fmaf(__builtin_fmaf(-s, s, x), 0.5f * y, s);
  }
#endif
  return sqrtf(x);
}
__host__ __device__ __forceinline__ bool recip_div_ok(float q) {
  return (as_u32(q) & 0x7fffffffu) - 0x0d800000u < 0x64000000u;  // |q| in [2^-100, 2^100)
}
// RN(a / b), given y = recip_for_div(b).
__host__ __device__ __forceinline__ float div_by_recip(float a, float b, float y) {
  const float q = a * y;
  if (recip_div_ok(q)) return __builtin_fmaf(__builtin_fmaf(-q, b, a), y, q);
  return a / b;
}
// y = RN(1/b) when |b| is in [2^-26, 2^26) (div_by_recip's domain), else NaN (then every
// div_by_recip(a, b, y) takes the division).
__host__ __device__ __forceinline__ float recip_for_div(float b) {
  const uint32_t e = (as_u32(b) >> 23) & 0xffu;
  return (e - (127u - 26u) < 52u) ? rcp_rn(b) : __builtin_nanf("");
}
// RN(a / b) for any a, b.
// -log2(x) by the hardware (v_log_f32), for the free-flight overshoot pre-test only; its error bound
// over the integrator's inputs is measured by tools/proofs/log2_bound.hip.  Host builds return 0,
// which never passes the pre-test (every draw takes the exact path).
__host__ __device__ __forceinline__ float neg_log2_hw(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return -__builtin_amdgcn_logf(x);
#else
  (void)x;
  return 0.0f;
#endif
}
__host__ __device__ __forceinline__ float div_rn(float a, float b) { return div_by_recip(a, b, recip_for_div(b)); }
}  // namespace math
}  // namespace vpt
