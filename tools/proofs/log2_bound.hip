// Exhaustive bound (tools only) of the hardware log2 (v_log_f32) over every float y in
// [2^-25, 1] -- a superset of the 1 - u values of uniform<float>() that the free-flight draw takes
// the logarithm of.  Reports max and min of (a - t) / t with a = -v_log_f32(y), t = -log2(y) in
// double (t > 0), and the y where they occur: the draw's overshoot pre-test uses the max as its
// relative margin (vpt_integrator.h, SM_DRAW).  Also max of a*ln2 / X with X = -logf(y) as the
// integrator computes it (math::logf_glibc_unit, == glibc): the pre-test's bound is stated on it.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <cstring>

#include "../../volume_path_tracer_amd/csrc/vpt_math.h"

__device__ __forceinline__ unsigned long long ord(double d) {  // order-preserving map of doubles to u64
  const unsigned long long b = (unsigned long long)__double_as_longlong(d);
  return (b >> 63) ? ~b : (b | (1ULL << 63));
}
__host__ double unord(unsigned long long o) {
  unsigned long long b = (o >> 63) ? (o & ~(1ULL << 63)) : ~o;
  double d;
  std::memcpy(&d, &b, 8);
  return d;
}

__global__ void check(uint32_t lo, uint32_t hi, unsigned long long* out) {
  const uint32_t bits = lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (bits > hi) return;
  const float y = __uint_as_float(bits);
  const float a = -__builtin_amdgcn_logf(y);
  const double t = -log2((double)y);
  const float X = -vpt::math::logf_glibc_unit(y);
  if (t == 0.0 || X == 0.0f) {
    if (a != 0.0f || X != 0.0f || t != 0.0) atomicAdd(out + 4, 1ULL);
    return;
  }
  atomicMax(out + 5, ord((double)a * 0x1.62e42fefa39efp-1 / (double)X - 1.0));
  const double rel = ((double)a - t) / t;
  const unsigned long long o = ord(rel);
  const unsigned long long prev_max = atomicMax(out + 0, o);
  if (o > prev_max) atomicMax(out + 1, ((unsigned long long)o & ~0xffffffffULL) | bits);  // arg (approx)
  const unsigned long long prev_min = atomicMin(out + 2, o);
  if (o < prev_min) atomicMin(out + 3, ((unsigned long long)o & ~0xffffffffULL) | bits);
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 6 * 8);
  unsigned long long init[6] = {0, 0, ~0ULL, ~0ULL, 0, 0};
  hipMemcpy(d, init, sizeof init, hipMemcpyHostToDevice);
  float f0 = 0x1p-25f, f1 = 1.0f;
  uint32_t lo, hi;
  std::memcpy(&lo, &f0, 4);
  std::memcpy(&hi, &f1, 4);
  const uint32_t n = hi - lo + 1;
  hipLaunchKernelGGL(check, dim3((n + 255) / 256), dim3(256), 0, 0, lo, hi, d);
  hipDeviceSynchronize();
  unsigned long long r[6];
  hipMemcpy(r, d, sizeof r, hipMemcpyDeviceToHost);
  float ymax, ymin;
  uint32_t bmax = (uint32_t)r[1], bmin = (uint32_t)r[3];
  std::memcpy(&ymax, &bmax, 4);
  std::memcpy(&ymin, &bmin, 4);
  printf("inputs %u (y in [2^-25, 1])\n", n);
  printf("max rel (a - t)/t = %.6e (= %.3f x 2^-24) near y = %a\n", unord(r[0]), unord(r[0]) * 16777216.0, ymax);
  printf("min rel (a - t)/t = %.6e (= %.3f x 2^-24) near y = %a\n", unord(r[2]), unord(r[2]) * 16777216.0, ymin);
  printf("max a*ln2/X - 1 = %.6e (= %.3f x 2^-24), X = -logf_glibc(y)\n", unord(r[5]), unord(r[5]) * 16777216.0);
  printf("zero-result disagreements (a, X, t not all 0 together): %llu\n", r[4]);
  return 0;
}
