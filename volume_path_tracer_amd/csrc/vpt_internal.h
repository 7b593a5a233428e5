// vpt_internal.h — host-side internals shared by the C-ABI translation units.
#pragma once

#include <sys/mman.h>

#include <cstdint>
#include <cstdlib>
#include <memory>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "../../include/vpt_gpu.h"
#include "vpt_integrator.h"

namespace vpt {

// Thread-local error message behind vpt_last_error().
int set_error(int code, const std::string& msg);

// An allocator whose value-less construct() leaves the element uninitialised: resize() of a large buffer that
// is written in full afterwards (the stencil pool: 0.84 GB for the 512^3 cloud) skips a serial zero-fill, and its
// pages are first touched by the threads that fill them.  Buffers of 4 MiB and more are 2-MiB aligned and
// advised for transparent huge pages: the ~1 GB a 512^3 grid's flatten faults in (and its release unmaps) is then
// ~500 page operations instead of ~250 000 -- where the kernel grants them (THP "madvise" or "always").
constexpr size_t kHugeAllocBytes = size_t(4) << 20, kHugePage = size_t(2) << 20;
template <class T>
struct NoInitAllocator : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInitAllocator<U>;
  };
  NoInitAllocator() = default;
  template <class U>
  NoInitAllocator(const NoInitAllocator<U>&) noexcept {}
  T* allocate(size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes < kHugeAllocBytes) return std::allocator<T>::allocate(n);
    void* p = std::aligned_alloc(kHugePage, (bytes + kHugePage - 1) / kHugePage * kHugePage);
    if (!p) throw std::bad_alloc();
    (void)madvise(p, bytes, MADV_HUGEPAGE);  // advice only: the buffer works either way
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_t n) noexcept {
    if (n * sizeof(T) < kHugeAllocBytes)
      std::allocator<T>::deallocate(p, n);
    else
      std::free(p);
  }
  template <class U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};

// A grid flattened for the GPU (host copies; vpt_gpu.hip uploads them).
struct HostGrid {
  DevGrid dev{};  // pointers are filled in after upload
  std::vector<int2> cells8, cells128;
  std::vector<RootTileDev> root;
  std::vector<float, NoInitAllocator<float>> bricks;  // [leaf][kBrickVox] square rows (built via [leaf][729] aprons)
  std::vector<float> leaf_max;   // fixed majorants
  std::vector<uint8_t> runs8;    // run radius per cells8 entry (compute_runs; empty until then)
  std::vector<uint32_t> walk8;   // HDDA fast-path table (build_walk_table)
  double run_fraction = 0.0;     // share of interior cells with a run radius >= 2
};

// Run radii of the cells8 table (DevGrid::runs8): r(c) = the largest r <= 15 such that every cell
// within Chebyshev distance r of c is in the table, interior, and has c's majorant (same bits,
// not NaN).  Sets h.runs8, h.dev.runs8 and h.run_fraction.
void compute_runs(HostGrid& h, int threads);

// The HDDA fast-path table of the cells8 entries (DevGrid::walk8): the majorant's bits for interior
// cells (a +0 majorant: the zero-run radius), kWalkSlow for the others.  Sets h.walk8 and h.dev.walk8
// (build_host_grid calls it).
void build_walk_table(HostGrid& h, int threads);

// Zero-run radius per cells8 entry: the largest r <= kZeroRunMax such that every cell within
// Chebyshev distance r lies in the table, is interior and has majorant +0 (0 for other cells).
std::vector<uint8_t> zero_run_radii(const HostGrid& h, int threads);

// Builds the leaf-slot tables, the walk table and the stencil brick pool; fixes the majorants
// (fix_majorants_for_interpolation, volume.cpp:104-160) when fix == true.
int build_host_grid(const vpt_grid_desc& d, bool fix, int threads, HostGrid& out);

// Host getValue on a built grid (same tables the device reads).
float host_value_at(const HostGrid& g, int32_t i, int32_t j, int32_t k);

// Fills the scene constants (camera matrix, light terms, ...) for a configuration.
int build_scene(const vpt_configuration& cfg, DevScene& S);

// Blackbody table from the embedded CIE 1931 data (init_blackbody_radiation_xyz).
void blackbody_table(float* out_500x3);
const float* cie_table();  // [471][3]
float cie_y_integral();

int default_threads();

// 1 when every blackbody lookup of the temperature grid reads rows < rows of the table: the
// trilinear value is a convex combination of getValue()s (leaf voxels, tile values, background), so
// T = value * scale + offset (worker.cpp:152-157) lies between the extremes of those; one row of margin
// covers the rounding of the lerps and of the two float operations.  0 for non-finite values.
struct ValueRange {
  float lo = 0, hi = 0;  // extremes of every getValue() of the grid (background, leaf voxels, tile values)
  bool finite = true;    // all of them finite (lo / hi are then meaningful)
};
ValueRange value_range(const vpt_grid_desc& t, int threads);  // (threads <= 0: default_threads())
int blackbody_rows_suffice(const ValueRange& r, float scale, float offset, int rows);

// A vpt_grid_desc that owns its arrays (vpt_synth_grid, vpt_grid_from_nanovdb, vpt_grid_read_nvdb;
// released by vpt_synth_free / vpt_grid_free).  d must stay the first member.
struct OwnedGrid {
  vpt_grid_desc d{};
  std::vector<int32_t> leaf_origin, tile_origin, tile_level, lower_origin, upper_origin;
  std::vector<float, NoInitAllocator<float>> leaf_values;  // (filled by copies: no zero-fill first)
  std::vector<float> leaf_max, tile_value;
  std::vector<uint64_t, NoInitAllocator<uint64_t>> leaf_mask;
  std::vector<uint8_t> tile_active;
  void finish();  // points d's arrays at the vectors
};
OwnedGrid* owned_grid_new();

}  // namespace vpt
