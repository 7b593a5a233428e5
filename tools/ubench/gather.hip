// Ceiling of divergent 4-byte per-lane gathers (tools only): the access pattern of the integrator's
// HDDA walk-word loads (one 4-byte word per lane from a table of ~1.2 MiB, each lane at a different
// line).  Every lane follows `Chains` independent random walks through the table (next = t[cur]),
// so a wavefront keeps Chains divergent loads in flight; occupancy is set with dynamic LDS.  Reports
// loads/s per CU for table sizes from L2-resident (1.2 MiB, the C3 walk table) to HBM-resident, and
// the memory-level parallelism (chains x waves/SIMD) the request rate saturates at.
//   hipcc -O3 --offload-arch=gfx950 -o gather gather.hip && ./gather [calib | width | pool MiB... | mix ...]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(x)                                                                              \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                           \
      std::exit(1);                                                                           \
    }                                                                                         \
  } while (0)

template <int Chains>
__global__ __launch_bounds__(256) void chase(const uint32_t* __restrict__ t, uint32_t n, int iters, uint32_t* out,
                                             int active) {
  extern __shared__ uint32_t occupancy_lds[];  // only sizes the block (waves per SIMD)
  uint32_t idx[Chains];
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if ((int)(threadIdx.x & 63) >= active) return;  // lanes of a wavefront that load (the rest idle)
#pragma unroll
  for (int c = 0; c < Chains; ++c) idx[c] = (g * 2654435761u + c * 40503u) % n;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < Chains; ++c) idx[c] = t[idx[c]];
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < Chains; ++c) r ^= idx[c];
  if (r == 0xFFFFFFFFu) out[0] = r + occupancy_lds[0];
}

// Wide gathers (the `width` mode): each lane loads one W-dword entry per step (W = 1, 2, 4, or 8 as two
// adjacent dwordx4 loads -- the stencil's 32-B piece), entries W*4-byte aligned; word 0 holds the next
// entry, the others zero, and the sum keeps every loaded dword live.
template <int W>
struct Entry;
template <>
struct Entry<1> {
  static __device__ __forceinline__ uint32_t next(const uint32_t* t, uint32_t i) { return t[i]; }
};
template <>
struct Entry<2> {
  static __device__ __forceinline__ uint32_t next(const uint32_t* t, uint32_t i) {
    const uint2 v = reinterpret_cast<const uint2*>(t)[i];
    return v.x + v.y;
  }
};
template <>
struct Entry<4> {
  static __device__ __forceinline__ uint32_t next(const uint32_t* t, uint32_t i) {
    const uint4 v = reinterpret_cast<const uint4*>(t)[i];
    return v.x + v.y + v.z + v.w;
  }
};
template <>
struct Entry<8> {
  static __device__ __forceinline__ uint32_t next(const uint32_t* t, uint32_t i) {
    const uint4 a = reinterpret_cast<const uint4*>(t)[2 * i], b = reinterpret_cast<const uint4*>(t)[2 * i + 1];
    return (a.x + a.y + a.z + a.w) + (b.x + b.y + b.z + b.w);
  }
};

template <int Chains, int W>
__global__ __launch_bounds__(256) void chase_wide(const uint32_t* __restrict__ t, uint32_t n, int iters, uint32_t* out) {
  extern __shared__ uint32_t occupancy_lds[];
  uint32_t idx[Chains];
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int c = 0; c < Chains; ++c) idx[c] = (g * 2654435761u + c * 40503u) % n;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < Chains; ++c) idx[c] = Entry<W>::next(t, idx[c]);
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < Chains; ++c) r ^= idx[c];
  if (r == 0xFFFFFFFFu) out[0] = r + occupancy_lds[0];
}

template <int Chains, int W>
double run_wide(const uint32_t* t, uint32_t n, int waves, int cus, uint32_t* out, size_t lds_total) {
  const int blocks = cus * waves;
  const size_t lds = lds_total / waves - 1024;
  const int iters = 256;
  CHECK(hipFuncSetAttribute((const void*)chase_wide<Chains, W>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((chase_wide<Chains, W>), dim3(blocks), dim3(256), lds, 0, t, n, iters, out);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((chase_wide<Chains, W>), dim3(blocks), dim3(256), lds, 0, t, n, iters, out);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  CHECK(hipGetLastError());
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  return (double)blocks * 256 * iters * Chains / (ms * 1e-3) / cus;  // lane entries per second per CU
}

template <int W>
void width_rows(size_t bytes, int cus, uint32_t* out, size_t lds_total) {
  const size_t n = bytes / (4 * W);
  std::vector<uint32_t> h(n * W, 0u);
  uint64_t s = 88172645463325252ull;
  for (size_t i = 0; i < n; ++i) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    h[i * W] = (uint32_t)(s % n);
  }
  uint32_t* t;
  CHECK(hipMalloc(&t, n * W * 4));
  CHECK(hipMemcpy(t, h.data(), n * W * 4, hipMemcpyHostToDevice));
  for (int waves : {4, 7})
    for (int chains : {1, 2}) {
      const double r = chains == 1 ? run_wide<1, W>(t, (uint32_t)n, waves, cus, out, lds_total)
                                   : run_wide<2, W>(t, (uint32_t)n, waves, cus, out, lds_total);
      std::printf("width %3d %10.2f %6d %6d %10.4f\n", W * 4, bytes / 1048576.0, chains, waves, r * 1e-9);
    }
  CHECK(hipFree(t));
}

// The C3 kernel's request mix in one chase (the `mix` mode, r05 -- a joint check of the two-class pipe model
// bench.py reports as pipe_frac): every lane runs one chain of divergent 4-B gathers through an L2-resident
// table (the walk words and cell entries: 81.6 per sample on C3) and, every `Period`-th step, one step of a
// second chain of 32-B gathers through a pool-sized table (the stencil pieces: 11.9 per sample), both
// dependent chains as in the kernel (a lane has at most one walk word and one stencil in flight); `active`
// lanes of each wavefront (the kernel's walk runs at ~32 of 64).
template <int Period>
__global__ __launch_bounds__(256) void chase_mix(const uint32_t* __restrict__ walk, uint32_t nw,
                                                 const uint32_t* __restrict__ pool, uint32_t np, int iters,
                                                 uint32_t* out, int active) {
  extern __shared__ uint32_t occupancy_lds[];
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if ((int)(threadIdx.x & 63) >= active) return;
  uint32_t w = (g * 2654435761u) % nw, p = (g * 40503u + 17u) % np;
  for (int i = 0; i < iters; ++i) {
    w = walk[w];
    if (i % Period == 0) p = Entry<8>::next(pool, p);
  }
  if ((w ^ p) == 0xFFFFFFFFu) out[0] = w + occupancy_lds[0];
}

template <int Period>
double run_mix(const uint32_t* walk, uint32_t nw, const uint32_t* pool, uint32_t np, int waves, int cus,
               uint32_t* out, size_t lds_total, int active) {
  const int blocks = cus * waves;
  const size_t lds = lds_total / waves - 1024;
  const int iters = 4096;
  CHECK(hipFuncSetAttribute((const void*)chase_mix<Period>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(chase_mix<Period>, dim3(blocks), dim3(256), lds, 0, walk, nw, pool, np, iters, out, active);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(chase_mix<Period>, dim3(blocks), dim3(256), lds, 0, walk, nw, pool, np, iters, out, active);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  CHECK(hipGetLastError());
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  return (double)blocks * 4 * active * iters / (ms * 1e-3);  // lane walk steps per second (whole device)
}

template <int Chains>
double run(const uint32_t* t, uint32_t n, int waves, int cus, uint32_t* out, size_t lds_total, int active = 64) {
  const int blocks = cus * waves;  // 256 threads = 4 waves per block, one per SIMD
  const size_t lds = lds_total / waves - 1024;
  const int iters = 512;
  CHECK(hipFuncSetAttribute((const void*)chase<Chains>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(chase<Chains>, dim3(blocks), dim3(256), lds, 0, t, n, iters, out, active);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(chase<Chains>, dim3(blocks), dim3(256), lds, 0, t, n, iters, out, active);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  CHECK(hipGetLastError());
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double loads = (double)blocks * 4 * active * iters * Chains;
  return loads / (ms * 1e-3) / cus;  // lane loads per second per CU
}

int main(int argc, char** argv) {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t lds_total = 160 * 1024;
  uint32_t* out;
  CHECK(hipMalloc(&out, 4));
  const bool calib = argc > 1 && std::string(argv[1]) == "calib";  // one config, for a --pmc pass
  if (argc > 1 && std::string(argv[1]) == "width") {  // lane entries/s per CU by entry width and table size
    std::printf("%5s %5s %10s %6s %6s %10s\n", "", "bytes", "table_MiB", "chains", "waves", "Gentry/s/CU");
    for (size_t bytes : {size_t(1228800), size_t(16) << 20, size_t(256) << 20, size_t(1536) << 20}) {
      width_rows<1>(bytes, cus, out, lds_total);
      width_rows<2>(bytes, cus, out, lds_total);
      width_rows<4>(bytes, cus, out, lds_total);
      width_rows<8>(bytes, cus, out, lds_total);
    }
    return 0;
  }
  if (argc > 2 && std::string(argv[1]) == "pool") {  // 32-B entries (a stencil's piece) from tables of the given MiB
    std::printf("%5s %5s %10s %6s %6s %10s\n", "", "bytes", "table_MiB", "chains", "waves", "Gentry/s/CU");
    for (int a = 2; a < argc; ++a) width_rows<8>((size_t)(std::atof(argv[a]) * 1048576.0) & ~size_t(31), cus, out, lds_total);
    return 0;
  }
  if (argc > 1 && std::string(argv[1]) == "mix") {  // mix [pool MiB] [walk KiB] [steps per sample] [samples] [period 4|7]
    const double pool_mib = argc > 2 ? std::atof(argv[2]) : 797.0, walk_kib = argc > 3 ? std::atof(argv[3]) : 1200.0;
    const double steps_per_sample = argc > 4 ? std::atof(argv[4]) : 81.6, samples = argc > 5 ? std::atof(argv[5]) : 530841600.0;
    const int period = argc > 6 ? std::atoi(argv[6]) : 7;
    auto table = [](size_t n, size_t stride) {
      std::vector<uint32_t> h(n * stride, 0u);
      uint64_t s = 88172645463325252ull;
      for (size_t i = 0; i < n; ++i) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        h[i * stride] = (uint32_t)(s % n);
      }
      uint32_t* d;
      CHECK(hipMalloc(&d, h.size() * 4));
      CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
      return d;
    };
    const uint32_t nw = (uint32_t)(walk_kib * 1024 / 4), np = (uint32_t)(pool_mib * 1048576.0 / 32);
    uint32_t* walk = table(nw, 1);
    uint32_t* pool = table(np, 8);
    std::printf("mix: %d CUs, walk table %.0f KiB, pool %.0f MiB, a 32-B step every %d walk steps; a sample = %.1f walk "
                "steps, frame = %.0f samples\n", cus, walk_kib, pool_mib, period, steps_per_sample, samples);
    std::printf("%6s %6s %14s %14s\n", "waves", "active", "Gsteps/s", "frame_ms");
    for (int waves : {7, 5})
      for (int act : {64, 32}) {
        const double r = period == 4 ? run_mix<4>(walk, nw, pool, np, waves, cus, out, lds_total, act)
                                     : run_mix<7>(walk, nw, pool, np, waves, cus, out, lds_total, act);
        std::printf("%6d %6d %14.3f %14.1f\n", waves, act, r * 1e-9, samples * steps_per_sample / r * 1e3);
      }
    return 0;
  }
  const size_t sizes[] = {307200, 1u << 22, 1u << 26};  // 1.2 MiB (L2), 16 MiB (MALL), 256 MiB (HBM)
  std::printf("gather ceiling: %d CUs, divergent 4-B loads, loads/s per CU (G)\n", cus);
  std::printf("%10s %6s %6s %10s\n", "table_MiB", "chains", "waves", "Gload/s/CU");
  for (size_t n : sizes) {
    std::vector<uint32_t> h(n);
    uint64_t s = 88172645463325252ull;
    for (size_t i = 0; i < n; ++i) {
      s ^= s << 13;
      s ^= s >> 7;
      s ^= s << 17;
      h[i] = (uint32_t)(s % n);
    }
    uint32_t* t;
    CHECK(hipMalloc(&t, n * 4));
    CHECK(hipMemcpy(t, h.data(), n * 4, hipMemcpyHostToDevice));
    if (calib) {  // 2 launches of chase<2>, 7 waves, 64 lanes: lane loads per launch below
      const double r = run<2>(t, (uint32_t)n, 7, cus, out, lds_total);
      std::printf("calib lane_loads_per_launch %.0f Gload/s/CU %.4f\n", (double)cus * 7 * 256 * 512 * 2, r * 1e-9);
      return 0;
    }
    for (int waves : {1, 2, 4, 7, 8}) {
      std::printf("%10.2f %6d %6d %10.4f\n", n * 4.0 / (1 << 20), 1, waves, run<1>(t, (uint32_t)n, waves, cus, out, lds_total) * 1e-9);
      std::printf("%10.2f %6d %6d %10.4f\n", n * 4.0 / (1 << 20), 2, waves, run<2>(t, (uint32_t)n, waves, cus, out, lds_total) * 1e-9);
      std::printf("%10.2f %6d %6d %10.4f\n", n * 4.0 / (1 << 20), 4, waves, run<4>(t, (uint32_t)n, waves, cus, out, lds_total) * 1e-9);
    }
    if (n == sizes[0]) {
      // Partly active wavefronts (a divergent walk keeps ~31 of 64 lanes walking): is the ceiling per
      // lane (line) or per wave instruction?  Lane loads/s and wave instructions/s per CU.
      std::printf("%10s %6s %6s %6s %10s %12s\n", "table_MiB", "chains", "waves", "active", "Gload/s/CU", "Ginst/s/CU");
      for (int act : {64, 48, 32, 16, 8, 1}) {
        const double r = run<2>(t, (uint32_t)n, 7, cus, out, lds_total, act);
        std::printf("%10.2f %6d %6d %6d %10.4f %12.4f\n", n * 4.0 / (1 << 20), 2, 7, act, r * 1e-9, r / act * 1e-9);
      }
    }
    CHECK(hipFree(t));
  }
  return 0;
}
