// Exhaustive check (tools only) over all 2^32 float bit patterns x of two short sequences that the
// integrator uses instead of the IEEE-correct division / square root macros:
//   rcp:  y0 = v_rcp_f32(x); y = fma(fma(-x, y0, 1), y0, y0)              == RN(1/x) ?
//   sqrt: s0 = v_sqrt_f32(x); r = fma(-s0, s0, x); s = fma(r, 0.5/s0 ...)  (see below) == RN(sqrt x) ?
// Mismatches are tallied per exponent of x, so the caller can guard the exponent range where the
// short sequence is exact.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>

__device__ __forceinline__ float rcp_short(float x) {
  const float y0 = __builtin_amdgcn_rcpf(x);
  return __builtin_fmaf(__builtin_fmaf(-x, y0, 1.0f), y0, y0);
}
__device__ __forceinline__ float sqrt_short(float x) {
  // y ~ 1/sqrt(x) (v_rsq_f32); s = x*y; h = 0.5*y; r = x - s*s (fma); s' = s + r*h (fma)
  const float y = __builtin_amdgcn_rsqf(x);
  const float s = x * y, h = 0.5f * y;
  const float r = __builtin_fmaf(-s, s, x);
  return __builtin_fmaf(r, h, s);
}

__global__ void check(uint32_t hi, unsigned long long* bad_rcp, unsigned long long* bad_sqrt) {
  const uint32_t x_bits = (hi << 24) | (blockIdx.x * blockDim.x + threadIdx.x);
  const float x = __uint_as_float(x_bits);
  const uint32_t e = (x_bits >> 23) & 0xff;
  const float r_ref = 1.0f / x, r = rcp_short(x);
  if (__float_as_uint(r_ref) != __float_as_uint(r) && !(r_ref != r_ref && r != r)) atomicAdd(bad_rcp + e, 1ULL);
  if (!(x_bits >> 31)) {
    const float s_ref = sqrtf(x), s = sqrt_short(x);
    if (__float_as_uint(s_ref) != __float_as_uint(s) && !(s_ref != s_ref && s != s)) atomicAdd(bad_sqrt + e, 1ULL);
  }
}

int main() {
  unsigned long long *br, *bs;
  hipMalloc(&br, 256 * 8);
  hipMalloc(&bs, 256 * 8);
  hipMemset(br, 0, 256 * 8);
  hipMemset(bs, 0, 256 * 8);
  for (uint32_t hi = 0; hi < 256; ++hi) hipLaunchKernelGGL(check, dim3(1 << 16), dim3(256), 0, 0, hi, br, bs);
  hipDeviceSynchronize();
  unsigned long long r[256], s[256];
  hipMemcpy(r, br, sizeof r, hipMemcpyDeviceToHost);
  hipMemcpy(s, bs, sizeof s, hipMemcpyDeviceToHost);
  unsigned long long tr = 0, ts = 0;
  for (int e = 0; e < 256; ++e) {
    tr += r[e];
    ts += s[e];
    if (r[e] || s[e]) printf("exponent field %3d (2^%4d): rcp mismatches %llu, sqrt mismatches %llu\n", e, e - 127, r[e], s[e]);
  }
  printf("total: rcp %llu, sqrt %llu mismatches over all 2^32 inputs\n", tr, ts);
  return 0;
}
