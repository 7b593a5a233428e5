// Instruction-throughput microbenchmark (tools only): cost of the integer / fp64 / division / logf
// building blocks of the integrator, in VALU issue slots relative to v_add_f32, at full occupancy.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../volume_path_tracer_amd/csrc/vpt_math.h"

constexpr int kIters = 4096;

template <int Op>
__global__ __launch_bounds__(256) void bench(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * 747796405u + seed, a1 = a0 ^ 0x9e3779b9u, a2 = a0 * 3u, a3 = a0 + 12345u;
  uint64_t s0 = a0 | 1ull << 40, s1 = a1 | 3ull << 33, s2 = a2 | 5ull << 35, s3 = a3 | 7ull << 37;
  float f0 = (a0 & 0xffff) * 1e-5f + 0.5f, f1 = f0 * 0.75f, f2 = f0 * 0.6f, f3 = f0 * 0.9f;
  double d0 = f0, d1 = f1, d2 = f2, d3 = f3;
#pragma unroll 1
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (Op == 0) { f0 = f0 + 1.5f; f1 = f1 + 1.25f; f2 = f2 + 0.75f; f3 = f3 + 0.5f; }
      if (Op == 1) { asm volatile("v_mul_lo_u32 %0, %0, %4\n v_mul_lo_u32 %1, %1, %4\n v_mul_lo_u32 %2, %2, %4\n v_mul_lo_u32 %3, %3, %4" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(seed)); }
      if (Op == 2) { asm volatile("v_mad_u64_u32 %0, vcc, %4, %5, %0\n v_mad_u64_u32 %1, vcc, %4, %5, %1\n v_mad_u64_u32 %2, vcc, %4, %5, %2\n v_mad_u64_u32 %3, vcc, %4, %5, %3" : "+v"(s0), "+v"(s1), "+v"(s2), "+v"(s3) : "v"(seed), "v"(a1) : "vcc"); }
      if (Op == 9) { asm volatile("v_mul_hi_u32 %0, %0, %4\n v_mul_hi_u32 %1, %1, %4\n v_mul_hi_u32 %2, %2, %4\n v_mul_hi_u32 %3, %3, %4" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(seed)); }
      if (Op == 10) { asm volatile("v_rcp_f32 %0, %0\n v_rcp_f32 %1, %1\n v_rcp_f32 %2, %2\n v_rcp_f32 %3, %3" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3)); }
      if (Op == 11) { asm volatile("v_add_f64 %0, %0, %0\n v_add_f64 %1, %1, %1\n v_add_f64 %2, %2, %2\n v_add_f64 %3, %3, %3" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3)); }
      if (Op == 12) { asm volatile("v_add_f32 %0, %0, %0\n v_add_f32 %1, %1, %1\n v_add_f32 %2, %2, %2\n v_add_f32 %3, %3, %3" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3)); }
      if (Op == 14) { asm volatile("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(seed)); }
      if (Op == 15) { asm volatile("v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n v_cndmask_b32 %2, %2, %4, vcc\n v_cndmask_b32 %3, %3, %4, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(seed) : "vcc"); }
      if (Op == 16) { asm volatile("v_cmp_lt_f32 vcc, %0, %4\n v_cmp_lt_f32 vcc, %1, %4\n v_cmp_lt_f32 vcc, %2, %4\n v_cmp_lt_f32 vcc, %3, %4" : : "v"(f0), "v"(f1), "v"(f2), "v"(f3), "v"(f0) : "vcc"); }
      if (Op == 17) { asm volatile("v_mul_f32 %0, %0, %0\n v_mul_f32 %1, %1, %1\n v_mul_f32 %2, %2, %2\n v_mul_f32 %3, %3, %3" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3)); }
      if (Op == 18) { asm volatile("v_fma_f32 %0, %0, %0, %0\n v_fma_f32 %1, %1, %1, %1\n v_fma_f32 %2, %2, %2, %2\n v_fma_f32 %3, %3, %3, %3" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3)); }
      if (Op == 19) { asm volatile("v_floor_f32 %0, %0\n v_floor_f32 %1, %1\n v_floor_f32 %2, %2\n v_floor_f32 %3, %3" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3)); }
      if (Op == 20) { asm volatile("v_and_b32 %0, %0, %4\n v_and_b32 %1, %1, %4\n v_and_b32 %2, %2, %4\n v_and_b32 %3, %3, %4" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(seed)); }
      if (Op == 21) { asm volatile("v_mov_b32 %0, %4\n v_mov_b32 %1, %4\n v_mov_b32 %2, %4\n v_mov_b32 %3, %4" : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3) : "v"(seed)); }
      if (Op == 22) { asm volatile("v_max_f32 %0, %0, %4\n v_max_f32 %1, %1, %4\n v_max_f32 %2, %2, %4\n v_max_f32 %3, %3, %4" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(f0)); }
      if (Op == 23) { asm volatile("v_xor_b32 %0, %0, %4\n v_xor_b32 %1, %1, %4\n v_xor_b32 %2, %2, %4\n v_xor_b32 %3, %3, %4" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(seed)); }
      if (Op == 24) { asm volatile("v_pk_add_f32 %0, %0, %0\n v_pk_add_f32 %1, %1, %1\n v_pk_add_f32 %2, %2, %2\n v_pk_add_f32 %3, %3, %3" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3)); }
      if (Op == 25) { asm volatile("v_cndmask_b32_e64 %0, %0, %4, s[8:9]\n v_cndmask_b32_e64 %1, %1, %4, s[8:9]\n v_cndmask_b32_e64 %2, %2, %4, s[8:9]\n v_cndmask_b32_e64 %3, %3, %4, s[8:9]" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(seed) : "s8", "s9"); }
      if (Op == 26) { asm volatile("v_cmp_lt_f32_e64 s[8:9], %0, %4\n v_cmp_lt_f32_e64 s[10:11], %1, %4\n v_cndmask_b32_e64 %2, %2, %4, s[8:9]\n v_cndmask_b32_e64 %3, %3, %4, s[10:11]" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(f0) : "s8", "s9", "s10", "s11"); }
      if (Op == 13) { asm volatile("v_cvt_f64_f32 %0, %4\n v_cvt_f64_f32 %1, %4\n v_cvt_f64_f32 %2, %4\n v_cvt_f64_f32 %3, %4" : "=v"(d0), "=v"(d1), "=v"(d2), "=v"(d3) : "v"(f0)); }
      if (Op == 3) { d0 = fma(d0, 0.999, 1e-3); d1 = fma(d1, 0.999, 1e-3); d2 = fma(d2, 0.999, 1e-3); d3 = fma(d3, 0.999, 1e-3); }
      if (Op == 4) { f0 = 1.0f / f0 + 0.5f; f1 = 1.0f / f1 + 0.5f; f2 = 1.0f / f2 + 0.5f; f3 = 1.0f / f3 + 0.5f; }
      if (Op == 5) { f0 = sqrtf(f0) + 0.5f; f1 = sqrtf(f1) + 0.5f; f2 = sqrtf(f2) + 0.5f; f3 = sqrtf(f3) + 0.5f; }
      if (Op == 6) { f0 = -vpt::math::logf_glibc_unit(f0 * 0.5f); f1 = -vpt::math::logf_glibc_unit(f1 * 0.5f); f2 = -vpt::math::logf_glibc_unit(f2 * 0.5f); f3 = -vpt::math::logf_glibc_unit(f3 * 0.5f); }
      if (Op == 7) { asm volatile("v_mul_u32_u24 %0, %0, %4\n v_mul_u32_u24 %1, %1, %4\n v_mul_u32_u24 %2, %2, %4\n v_mul_u32_u24 %3, %3, %4" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(seed)); }
      if (Op == 8) { asm volatile("v_cvt_f32_u32 %0, %4\n v_cvt_f32_u32 %1, %4\n v_cvt_f32_u32 %2, %4\n v_cvt_f32_u32 %3, %4" : "=v"(f0), "=v"(f1), "=v"(f2), "=v"(f3) : "v"(a0)); }
    }
  }
  uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ (uint32_t)(s0 ^ s1 ^ s2 ^ s3) ^ vpt::math::as_u32(f0 + f1 + f2 + f3) ^ (uint32_t)(int64_t)(d0 + d1 + d2 + d3);
  if (r == 0x12345678u) out[0] = r;
}

int main() {
  uint32_t* out;
  hipMalloc(&out, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"v_add_f32(c)", "v_mul_lo_u32", "v_mad_u64_u32", "fma_f64(c)", "div_f32(cr)", "sqrt_f32(cr)", "logf_glibc_unit", "v_mul_u32_u24", "v_cvt_f32_u32", "v_mul_hi_u32", "v_rcp_f32", "v_add_f64", "v_add_f32(asm)", "v_cvt_f64_f32", "v_add_u32", "v_cndmask_b32", "v_cmp_lt_f32", "v_mul_f32", "v_fma_f32", "v_floor_f32", "v_and_b32", "v_mov_b32", "v_max_f32", "v_xor_b32", "v_pk_add_f32", "v_cndmask_e64(sgpr)", "cmp+cndmask pairs"};
  void (*ks[])(uint32_t*, uint32_t) = {bench<0>, bench<1>, bench<2>, bench<3>, bench<4>, bench<5>, bench<6>, bench<7>, bench<8>, bench<9>, bench<10>, bench<11>, bench<12>, bench<13>, bench<14>, bench<15>, bench<16>, bench<17>, bench<18>, bench<19>, bench<20>, bench<21>, bench<22>, bench<23>, bench<24>, bench<25>, bench<26>};
  const int blocks = 256 * 8;
  double base = 1;
  for (int op = 0; op < 27; ++op) {
    hipLaunchKernelGGL(ks[op], dim3(blocks), dim3(256), 0, 0, out, 1u);
    hipEventRecord(e0);
    hipLaunchKernelGGL(ks[op], dim3(blocks), dim3(256), 0, 0, out, 2u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double ops = (double)blocks * 256 * kIters * 8 * 4;
    double per = ms * 1e-3 / ops * 1e12;  // ps per lane-op
    if (op == 12) base = per;
    printf("%-18s %8.3f ms  %7.4f ps/lane-op  %5.2f x v_add_f32\n", names[op], ms, per, per / 0.0151);
  }
  return 0;
}
