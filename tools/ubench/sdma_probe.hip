// Whether copies run beside a persistent kernel that holds every CU (tools only; r05, the drop-in's
// progressive film): a kernel of CUs x 8 blocks keeps every wave busy for `hold_ms` (fp32 atomics into a
// device film, a deadline from s_memrealtime, so the grid always ends), and while it runs the host times
// on a second stream: a device -> pinned-host copy of the film (the progressive film's snapshot), a
// pinned-host -> device copy of zeros (its clear), a device -> device copy and a memset (blit kernels,
// which need CUs).  A copy that finishes in about size / link bandwidth ran beside the kernel; one that
// finishes only near hold_ms waited for it.
//   hipcc -O3 --offload-arch=gfx950 -o sdma_probe sdma_probe.hip && ./sdma_probe [MiB] [hold_ms]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

__global__ __launch_bounds__(256) void busy(float* film, uint64_t n, uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2654435761ull;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    atomicAdd(film + (i % n), 1.0f);
    i += 7919;
    __builtin_amdgcn_s_sleep(32);
  }
}

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? (size_t)std::atol(argv[1]) : 32;
  const double hold_ms = argc > 2 ? std::atof(argv[2]) : 1000.0;
  const size_t bytes = mib << 20, n = bytes / sizeof(float);
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float *film = nullptr, *film2 = nullptr, *host = nullptr, *zeros = nullptr;
  CHECK(hipMalloc((void**)&film, bytes));
  CHECK(hipMalloc((void**)&film2, bytes));
  CHECK(hipMemset(film, 0, bytes));
  CHECK(hipHostMalloc((void**)&host, bytes, hipHostMallocDefault));
  CHECK(hipHostMalloc((void**)&zeros, bytes, hipHostMallocDefault));
  for (size_t i = 0; i < n; ++i) zeros[i] = 0.0f;
  hipStream_t a, b;
  CHECK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  // warm both copy paths and the kernel once (first-use costs)
  CHECK(hipMemcpyAsync(host, film, bytes, hipMemcpyDeviceToHost, b));
  CHECK(hipMemcpyAsync(film, zeros, bytes, hipMemcpyHostToDevice, b));
  CHECK(hipStreamSynchronize(b));
  auto tw = std::chrono::steady_clock::now();
  CHECK(hipMemcpyAsync(host, film, bytes, hipMemcpyDeviceToHost, b));
  CHECK(hipStreamSynchronize(b));
  std::printf("idle device: D2H %zu MiB %.2f ms\n", mib, ms_since(tw));
  const uint64_t ticks = (uint64_t)(hold_ms * 1e5);
  hipLaunchKernelGGL(busy, dim3(cus * 8), dim3(256), 0, a, film, (uint64_t)n, ticks);
  CHECK(hipGetLastError());
  const auto t0 = std::chrono::steady_clock::now();
  std::this_thread::sleep_for(std::chrono::milliseconds((int)(hold_ms / 10)));
  struct Op {
    const char* name;
    int kind;
  } ops[] = {{"D2H to pinned", 0}, {"H2D from pinned", 1}, {"D2H to pinned (again)", 0}, {"D2D", 2}, {"memset", 3}};
  for (const Op& op : ops) {
    const double start = ms_since(t0);
    const auto t = std::chrono::steady_clock::now();
    if (op.kind == 0) CHECK(hipMemcpyAsync(host, film, bytes, hipMemcpyDeviceToHost, b));
    if (op.kind == 1) CHECK(hipMemcpyAsync(film, zeros, bytes, hipMemcpyHostToDevice, b));
    if (op.kind == 2) CHECK(hipMemcpyAsync(film2, film, bytes, hipMemcpyDeviceToDevice, b));
    if (op.kind == 3) CHECK(hipMemsetAsync(film2, 0, bytes, b));
    CHECK(hipStreamSynchronize(b));
    const double took = ms_since(t);
    int running = hipStreamQuery(a) == hipErrorNotReady;
    std::printf("%-24s issued at %7.1f ms, took %8.2f ms (%6.1f GB/s), kernel still running after: %d\n", op.name, start,
                took, bytes / took / 1e6, running);
  }
  CHECK(hipStreamSynchronize(a));
  std::printf("kernel ended at %.1f ms (hold %.0f ms)\n", ms_since(t0), hold_ms);
  return 0;
}
