// Per-element noise arithmetic shared by the noise kernels (noise.hip) and the fused
// noise -> filter kernels (stencil_u8.hip), on the Philox stream described in noise.hip:
// skimage.util.random_noise's float64 apply in numpy's op order plus the caller's U8 cast; for
// gaussian / speckle the U8 cast itself runs on the 0..255 scale in fp32 (floor(clip(v + 255 n)),
// the same law; the float64 value is still produced for callers that keep it).  Files that
// include this are compiled with -ffp-contract=off.
#pragma once

#include "idn_common.hpp"

namespace idn {

__device__ __forceinline__ double img_as_float(uint32_t v) { return __dmul_rn((double)v, 1.0 / 255.0); }

// np.clip(v, 0, 1) for non-NaN v (v_max_f64 / v_min_f64)
__device__ __forceinline__ double clip01(double v) { return __builtin_fmin(__builtin_fmax(v, 0.0), 1.0); }

// (255 * out).astype(np.uint8) for out in [0, 1]: truncation (out is never negative here)
__device__ __forceinline__ uint8_t u8_of(double out) { return (uint8_t)(int)__dmul_rn(out, 255.0); }

// two standard normals from one Philox block (Box-Muller, fp32 hardware transcendentals:
// v_log/v_sqrt/v_sin/v_cos; sin/cos take revolutions, so theta = u2 needs no 2*pi multiply, and
// the raw v_sqrt_f32 (1 ulp) replaces the 13-instruction correctly rounded sqrtf sequence)
__device__ __forceinline__ void normal2(const u32x4& r, float& z0, float& z1) {
  const float u1 = ((float)(r.x >> 8) + 1.0f) * (1.0f / 16777216.0f);  // (0, 1]
  const float u2 = (float)(r.y >> 8) * (1.0f / 16777216.0f);           // [0, 1)
  const float rad =
      __builtin_amdgcn_sqrtf(-2.0f * 0.6931471805599453f * __builtin_amdgcn_logf(u1));
  z0 = rad * __builtin_amdgcn_cosf(u2);
  z1 = rad * __builtin_amdgcn_sinf(u2);
}


// two standard normals from two 16-bit uniforms (the halves of one Philox word): u1 in
// (0, 1] on a 2^-16 grid (so |z| <= sqrt(2 ln 2^16) = 4.71: every level the reference uses has
// sd > 0.21, where |n| > 4.71 sd saturates the clip in [0, 1] anyway), u2 in [0, 1)
__device__ __forceinline__ void normal2_16(uint32_t w, float& z0, float& z1) {
  const float u1 = ((float)(w & 0xFFFFu) + 1.0f) * (1.0f / 65536.0f);
  const float u2 = (float)(w >> 16) * (1.0f / 65536.0f);
  const float rad =
      __builtin_amdgcn_sqrtf(-2.0f * 0.6931471805599453f * __builtin_amdgcn_logf(u1));
  z0 = rad * __builtin_amdgcn_cosf(u2);
  z1 = rad * __builtin_amdgcn_sinf(u2);
}
__device__ __forceinline__ void normal8_16(const u32x4& r, float (&z)[8]) {
  normal2_16(r.x, z[0], z[1]);
  normal2_16(r.y, z[2], z[3]);
  normal2_16(r.z, z[4], z[5]);
  normal2_16(r.w, z[6], z[7]);
}

// 16 consecutive elements e0 = 16 * chunk .. e0 + 15 of image `gimg` (compact layout, flat
// element index): the flat16 stream --
//   gaussian / speckle  counter (e/8, 0, image id) -> Philox4x32-7 -> 8 16-bit uniforms -> four
//                       Box-Muller pairs -> the 8 normals of elements 8q..8q+7
//   s&p                 counter (e/4, 1, image id) -> Philox4x32-7 -> word b holds (U1, U2) of
//                       element 4q+b as 16-bit uniforms compared against integer thresholds
//                       (|P - p| < 2^-16); round 1 spent one Philox4x32-10 block per 2 elements
// MEAN0: mean == 0.0, so mean + sd*z is sd*z exactly up to the sign of a zero, which the
// following x + n / x + x*n (x >= 0) cannot see: one float64 add per element less.
// Returns the U8 bytes; `of` (nullable) receives the 16 float64 values.
template <int KIND, bool MEAN0>
__device__ __forceinline__ v4u noise16_u8(const v4u raw, uint32_t chunk, uint64_t gimg,
                                          uint64_t key, double p0, double p1, uint32_t t_flip,
                                          uint32_t t_salt, double* of) {
  const uint32_t in[4] = {raw.x, raw.y, raw.z, raw.w};
  uint32_t o[4] = {0u, 0u, 0u, 0u};
  float z8[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // elements 4k .. 4k+3
    double outv[4];
    if constexpr (KIND == IDN_NOISE_SAP) {
      // one Philox4x32-7 block per 4 elements (e / 4 = chunk * 4 + k): element b takes word b,
      // low 16 bits the `flipped` uniform, high 16 bits the `salted` one
      const uint32_t q = chunk * 4u + (uint32_t)k;
      const u32x4 r = philox4x32<7>(u32x4{q, 1u, (uint32_t)gimg, (uint32_t)(gimg >> 32)}, key);
      const uint32_t wd[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const double xv = img_as_float((in[k] >> (8 * b)) & 0xFFu);
        outv[b] = (wd[b] & 0xFFFFu) < t_flip ? ((wd[b] >> 16) < t_salt ? 1.0 : 0.0) : xv;
      }
    } else {
      // one Philox4x32-7 block -> 8 16-bit uniforms -> 4 Box-Muller pairs -> 8 normals, for
      // elements 8j .. 8j+7 (j = chunk * 2 + k / 2)
      if ((k & 1) == 0) {
        const uint32_t q = chunk * 2u + (uint32_t)(k >> 1);
        const u32x4 r = philox4x32<7>(u32x4{q, 0u, (uint32_t)gimg, (uint32_t)(gimg >> 32)}, key);
        normal8_16(r, z8);
      }
      const float* z = z8 + 4 * (k & 1);
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        // the U8 result on the 0..255 scale in fp32: floor(clip(v + 255 n)) (gaussian) or
        // floor(clip(v + v n)) (speckle) -- the law of (255 * clip(x + n)).astype(uint8) up to
        // fp32 rounding next to integers; fewer than half the float64 apply's instructions
        const float v = (float)((in[k] >> (8 * b)) & 0xFFu);
        float ov;
        if constexpr (KIND == IDN_NOISE_GAUSSIAN) {
          ov = __builtin_fmaf((float)(255.0 * p1), z[b], MEAN0 ? v : v + (float)(255.0 * p0));
        } else {
          const float n = MEAN0 ? (float)p1 * z[b] : __builtin_fmaf((float)p1, z[b], (float)p0);
          ov = __builtin_fmaf(v, n, v);
        }
        o[k] |= (uint32_t)__builtin_amdgcn_fmed3f(ov, 0.0f, 255.0f) << (8 * b);
        if (of) {  // the float64 result (numpy's op order) for callers that keep it
          const double sz = __dmul_rn(p1, (double)z[b]);
          const double nz = MEAN0 ? sz : __dadd_rn(p0, sz);
          const double xv = img_as_float((in[k] >> (8 * b)) & 0xFFu);
          of[4 * k + b] = KIND == IDN_NOISE_GAUSSIAN ? clip01(__dadd_rn(xv, nz))
                                                     : clip01(__dadd_rn(xv, __dmul_rn(xv, nz)));
        }
      }
      continue;
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      o[k] |= (uint32_t)u8_of(outv[b]) << (8 * b);
      if (of) of[4 * k + b] = outv[b];
    }
  }
  return v4u{o[0], o[1], o[2], o[3]};
}

// 16-bit uniform thresholds of the s&p flat stream: P(u < t / 2^16) within 2^-16 of cdf0
inline uint32_t sap_threshold(double pp) {
  const double t = ceil(pp * 65536.0);
  return t <= 0.0 ? 0u : t >= 65536.0 ? 65536u : (uint32_t)t;
}

}  // namespace idn
