// vpt_scene.cpp — host-side scene constants: camera matrix, light terms, blackbody table.
//
// Everything here runs once per context on the host, with the reference's float formulas and
// operation order (Eigen fixed-size products/reductions restated as a0*b0 + (a1*b1 + a2*b2)),
// so the device integrator receives bit-identical constants.
#include <sched.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "vpt_internal.h"

namespace vpt {
namespace {

#include "cie_data.inc"  // kCIE[471][3] (double literals), kYIntegral — generated from data/cie1931_xyz.csv

struct CieTable {
  float v[471 * 3];
  float yint;
  CieTable() {
    // std::array<float,471> initialised from double literals (src/spectral_data/xyz.hpp:17-314).
    for (int i = 0; i < 471; ++i)
      for (int c = 0; c < 3; ++c) v[i * 3 + c] = (float)kCIE[i][c];
    yint = (float)kYIntegral;
  }
};
const CieTable& cie() {
  static CieTable t;
  return t;
}

// detail::planck_law (src/spectral.cpp:7-20)
float planck_law(float lambda_m, float temperature_k) {
  if (temperature_k <= 0.0f) return 0.0f;
  const float c = 299792458.f;
  const float h = 6.62606957e-34f;
  const float kb = 1.3806488e-23f;
  const float num = 2 * h * c * c;
  float lambda5 = (float)std::pow((double)lambda_m, 5.0);  // std::pow(float, int) promotes to double
  float e = std::exp((h * c) / (lambda_m * kb * temperature_k));
  float den = lambda5 * (e - 1);
  return num / den;
}

// spectrum_to_xyz(BlackbodyEmittedRadianceSpectrum(T)) (include/vpt/spectral.hpp:62-75)
void spectrum_to_xyz(float t, float out[3]) {
  const CieTable& C = cie();
  for (int c = 0; c < 3; ++c) {
    float integral = 0.0f;
    for (int i = 0; i < 471; ++i) integral += C.v[i * 3 + c] * planck_law(static_cast<float>(360 + i) * 1e-9f, t);
    out[c] = integral;
  }
  for (int c = 0; c < 3; ++c) out[c] = out[c] / C.yint;
}

struct F3 {
  float x, y, z;
};
F3 normalized(F3 a) {  // Eigen MatrixBase::normalized()
  float z = a.x * a.x + (a.y * a.y + a.z * a.z);
  if (z > 0.0f) {
    float s = std::sqrt(z);
    return F3{a.x / s, a.y / s, a.z / s};
  }
  return a;
}
F3 cross(F3 a, F3 b) { return F3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }

// 3x3 lazy product coefficient (Eigen coeff-based product: redux over the inner dimension).
void mat3_mul(const float* A, const float* B, float* O) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      O[i * 3 + j] = A[i * 3] * B[j] + (A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j]);
}
void mat3_vec(const float* A, const float* v, float* o) {
  for (int i = 0; i < 3; ++i) o[i] = A[i * 3] * v[0] + (A[i * 3 + 1] * v[1] + A[i * 3 + 2] * v[2]);
}

}  // namespace

const float* cie_table() { return cie().v; }
float cie_y_integral() { return cie().yint; }

void blackbody_table(float* out) {  // init_blackbody_radiation_xyz (precompute_blackbody.cpp:18-22)
  for (int i = 0; i < VPT_BLACKBODY_ROWS; ++i) spectrum_to_xyz((i - 1) * 100.0f, out + i * 3);
}

// Host worker threads for the grid build: the CPUs this process may run on (its affinity mask), capped by the
// cgroup's CPU quota (cpu.max: the GPU box grants a job 16 of its 256 CPUs -- 64 threads there time-slice on 16)
// and at 64.  Computed once.
int default_threads() {
  static const int n = [] {
    unsigned c = std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0 && CPU_COUNT(&set) > 0) c = (unsigned)CPU_COUNT(&set);
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char quota[32] = {};
      long long period = 0;
      if (std::fscanf(f, "%31s %lld", quota, &period) == 2 && std::strcmp(quota, "max") != 0 && period > 0) {
        const long long q = std::atoll(quota);
        const unsigned cap = (unsigned)std::max(1LL, (q + period - 1) / period);
        c = std::min(c, cap);
      }
      std::fclose(f);
    }
    if (c == 0) c = 4;
    return (int)std::min(c, 64u);
  }();
  return n;
}

// Camera::Camera (src/camera.cpp:45-57) and the constant terms of vpt::run / sample_Ld.
int build_scene(const vpt_configuration& cfg, DevScene& S) {
  std::memset(&S, 0, sizeof S);
  const int64_t W = cfg.output_size[0], H = cfg.output_size[1];
  const int64_t tw = cfg.tile_size[0], th = cfg.tile_size[1];
  if (W <= 0 || H <= 0 || tw <= 0 || th <= 0) return set_error(VPT_E_INVALID, "output_size and tile_size must be positive");
  if (W > (1 << 24) || H > (1 << 24) || tw > (1 << 16) || th > (1 << 16) || tw * th >= (1 << 29))
    return set_error(VPT_E_INVALID, "output_size / tile_size too large");
  S.seed = cfg.seed;
  S.W = (int32_t)W;
  S.H = (int32_t)H;
  S.tw = (int32_t)tw;
  S.th = (int32_t)th;
  uint64_t ntx = (uint64_t)(W / tw + (W % tw != 0)), nty = (uint64_t)(H / th + (H % th != 0));
  S.ntx = (uint32_t)ntx;
  S.T = ntx * nty;
  const vpt_worker_params& P = cfg.worker_parameters;
  const vpt_volume_params& V = cfg.volume_parameters;
  S.max_depth = P.max_depth;
  S.single_pixel_enabled = P.single_pixel_enabled ? 1 : 0;
  S.sp_x = (int32_t)P.single_pixel_coord[0];
  S.sp_y = (int32_t)P.single_pixel_coord[1];
  S.jitter_scale = P.use_jitter ? 0.5f : 0.0f;

  // camera_to_world (camera.cpp:5-19)
  const vpt_camera_params& cp = cfg.camera_parameters;
  F3 pos{cp.position[0], cp.position[1], cp.position[2]};
  F3 look{cp.look[0], cp.look[1], cp.look[2]};
  F3 up{cp.up[0], cp.up[1], cp.up[2]};
  F3 dir = normalized(F3{look.x - pos.x, look.y - pos.y, look.z - pos.z});
  F3 left = cross(normalized(up), dir);
  F3 new_up = cross(dir, left);
  float Cm[9] = {left.x, new_up.x, dir.x, left.y, new_up.y, dir.y, left.z, new_up.z, dir.z};
  // screen_to_camera (camera.cpp:34-43), raster_to_screen (camera.cpp:21-32)
  float ar = static_cast<float>(W) / static_cast<float>(H);
  float vfov_rad = 3.14159274f * cp.vfov_deg / 180.0f;
  float tv = std::tan(vfov_rad / 2);
  float Sl[9] = {ar * tv, 0, 0, 0, tv, 0, 0, 0, 0}, St[3] = {0.0f, 0.0f, 1.0f};
  float hx = static_cast<float>(W) / 2.0f, hy = static_cast<float>(H) / 2.0f;
  float Rl[9] = {-(1.0f / hx), 0, 0, 0, -(1.0f / hy), 0, 0, 0, 0}, Rt[3] = {1.0f, 1.0f, 0.0f};
  // m_screen_to_world_dir = c2w.linear() * s2c ; m_raster_to_world_dir = m_screen_to_world_dir * r2s
  float SWl[9], SWt[3], tmp[3];
  mat3_mul(Cm, Sl, SWl);
  mat3_vec(Cm, St, SWt);
  mat3_mul(SWl, Rl, S.cam_L);
  mat3_vec(SWl, Rt, tmp);
  for (int i = 0; i < 3; ++i) S.cam_t[i] = tmp[i] + SWt[i];
  S.cam_pos[0] = pos.x;
  S.cam_pos[1] = pos.y;
  S.cam_pos[2] = pos.z;
  S.imaging_ratio = cp.imaging_ratio;

  for (int i = 0; i < 3; ++i) {
    S.le_inf[i] = P.infinite_light_xyz[i] * P.infinite_light_multiplier;  // worker.cpp:199
    S.Li[i] = P.distant_light_xyz[i] * P.distant_light_multiplier;        // worker.cpp:55
  }
  S.li_zero = (S.Li[0] == 0.0f && S.Li[1] == 0.0f && S.Li[2] == 0.0f) ? 1 : 0;
  F3 wi = normalized(F3{P.distant_light_inv_direction[0], P.distant_light_inv_direction[1], P.distant_light_inv_direction[2]});
  S.wi[0] = wi.x;
  S.wi[1] = wi.y;
  S.wi[2] = wi.z;
  S.sigma_a = V.sigma_a;
  S.sigma_s = V.sigma_s;
  S.sigma_t = V.sigma_a + V.sigma_s;
  S.g_hg = V.henyey_greenstein_g;
  S.le_scale = V.le_scale;
  S.temp_scale = V.temperature_scale;
  S.temp_offset = V.temperature_offset;
  S.y_integral = cie().yint;
  return VPT_OK;
}

}  // namespace vpt

extern "C" int vpt_blackbody_table(float* out) {
  if (!out) return vpt::set_error(VPT_E_INVALID, "vpt_blackbody_table: null output");
  vpt::blackbody_table(out);
  return VPT_OK;
}

namespace vpt {
int blackbody_rows_suffice(const ValueRange& r, float scale, float offset, int rows) {
  if (!r.finite) return 0;
  const float tmax = std::max(r.lo * scale, r.hi * scale) + offset;
  // rows dn and dn + 1 with dn <= floor(T / 100) + 1 (the search loops of blackbody_xyz), plus margin
  return std::isfinite(tmax) && tmax < (float)(rows - 3) * 100.0f ? 1 : 0;
}
}  // namespace vpt

extern "C" int vpt_blackbody_xyz(const float* table, float t, float* out) {
  if (!table || !out) return vpt::set_error(VPT_E_INVALID, "vpt_blackbody_xyz: null argument");
  std::vector<float> bb(501 * 3, 0.0f);
  std::memcpy(bb.data(), table, 500 * 3 * sizeof(float));
  vpt::DevScene S;
  std::memset(&S, 0, sizeof S);
  S.bb = bb.data();
  S.cie = vpt::cie_table();
  S.y_integral = vpt::cie_y_integral();
  if (t >= 49900.0f && std::isfinite(t)) {  // host: the reference's exact spectral integration
    vpt::spectrum_to_xyz(t, out);
    return VPT_OK;
  }
  vpt::blackbody_xyz(S, S.bb, t, out[0], out[1], out[2]);
  return VPT_OK;
}
