// Exhaustive check (tools only): for every pair of float significands a, b in [1, 2),
//   y = RN(1/b);  q = RN(a*y);  r = fma(-q, b, a);  q' = fma(r, y, q)
// equals the correctly rounded quotient RN(a/b).  Exponent scaling is exact for normal operands
// and results, so this covers every a/b whose operands and quotient are normal and finite.
// The integrator uses this to divide by per-ray / per-cell constants with a stored reciprocal.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__global__ __launch_bounds__(256) void check(uint32_t b_first, uint32_t b_count, unsigned long long* bad,
                                             uint32_t* first_bad) {
  for (uint32_t bi = blockIdx.x; bi < b_count; bi += gridDim.x) {
    const uint32_t bm = b_first + bi;
    const float b = __uint_as_float(0x3f800000u | bm);
    const float y = 1.0f / b;
    unsigned long long nbad = 0;
    for (uint32_t am = threadIdx.x; am < (1u << 23); am += blockDim.x) {
      const float a = __uint_as_float(0x3f800000u | am);
      const float ref = a / b;
      const float q = a * y;
      const float r = __builtin_fmaf(-q, b, a);
      const float q2 = __builtin_fmaf(r, y, q);
      if (__float_as_uint(q2) != __float_as_uint(ref)) {
        ++nbad;
        if (atomicCAS(first_bad, 0xffffffffu, am) == 0xffffffffu) first_bad[1] = bm;
      }
    }
    if (nbad) atomicAdd(bad, nbad);
  }
}

int main(int argc, char** argv) {
  const uint32_t total = 1u << 23;
  const uint32_t chunk = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 16);
  unsigned long long* bad;
  uint32_t* fb;
  hipMalloc(&bad, 8);
  hipMalloc(&fb, 8);
  hipMemset(bad, 0, 8);
  hipMemset(fb, 0xff, 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (uint32_t b0 = 0; b0 < total; b0 += chunk) {
    hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, b0, chunk, bad, fb);
    hipDeviceSynchronize();
    if ((b0 / chunk) % 16 == 0) { printf("b significands done: %u / %u\n", b0 + chunk, total); fflush(stdout); }
  }
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long nbad;
  uint32_t f[2];
  hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost);
  hipMemcpy(f, fb, 8, hipMemcpyDeviceToHost);
  printf("pairs checked: %llu  mismatches: %llu  (first: a_sig=0x%06x b_sig=0x%06x)  %.1f s\n",
         (unsigned long long)total * total, nbad, f[0], f[1], ms / 1e3);
  return nbad ? 1 : 0;
}
