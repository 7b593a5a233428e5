// vpt_image.cpp — film -> 8-bit sRGB, as the reference writes its output image.
//
// film_to_image (src/main.cpp:12-24): xyz = film.xyz / film.w; linsrgb = M * xyz with the
// xyz_to_linsrgb matrix (include/vpt/color.hpp:8-18, double literals rounded to float; Eigen's
// 3x3 * 3x1 product as m0*x + (m1*y + m2*z)); sRGB OETF (color.hpp:20-30, std::pow on floats);
// clamp to [0, 1]; * 255; cast to unsigned char (truncation).  Host code, run after the render.
#include <cmath>
#include <cstdint>

#include "vpt_internal.h"

namespace vpt {
namespace {
const float kM[9] = {(float)3.240479, (float)-1.537150, (float)-0.498535,  //
                     (float)-0.969256, (float)1.875991, (float)0.041556,   //
                     (float)0.055648, (float)-0.204043, (float)1.057311};
inline float srgb_oetf(float x) { return x <= 0.0031308f ? (12.92f * x) : (1.055f * std::pow(x, 1.0f / 2.4f) - 0.055f); }
inline uint8_t to_u8(float v) {
  // srgb.cwiseMax(0).cwiseMin(1) * 255 -> cast<unsigned char>; NaN (pixels without samples: 0/0)
  // goes through max/min unchanged and converts like x86 cvttss2si (0x80000000 -> low byte 0).
  v = (v < 0.0f) ? 0.0f : v;
  v = (1.0f < v) ? 1.0f : v;
  v = v * 255.0f;
  if (!(v == v)) return 0;
  return (uint8_t)(int32_t)v;
}
}  // namespace
}  // namespace vpt

extern "C" int vpt_film_to_srgb8(const float* film, int64_t w, int64_t h, uint8_t* out) {
  if (!film || !out || w <= 0 || h <= 0) return vpt::set_error(VPT_E_INVALID, "vpt_film_to_srgb8: bad argument");
  for (int64_t i = 0; i < w * h; ++i) {
    const float* p = film + i * 4;
    const float x = p[0] / p[3], y = p[1] / p[3], z = p[2] / p[3];
    for (int c = 0; c < 3; ++c) {
      const float* m = vpt::kM + 3 * c;
      const float lin = m[0] * x + (m[1] * y + m[2] * z);
      out[i * 3 + c] = vpt::to_u8(vpt::srgb_oetf(lin));
    }
  }
  return VPT_OK;
}
