// Per-element noise arithmetic of the u8 noise kernels (noise.hip), on the Philox streams described
// there: skimage.util.random_noise's apply followed by the caller's U8 cast (255 * out).astype(
// uint8).  Two Gaussian streams:
//   * u8-only outputs (the denoise branches' input): 16-bit uniforms, fp32 Box-Muller, the U8
//     cast computed on the 0..255 scale in fp32 -- floor(clip(v + 255 n)) / floor(clip(v + v n))
//     -- which differs from numpy's float64 apply + cast only where 255 * out lies within ~3e-4 of
//     an integer (a boundary shift of ~1e-5 LSB: invisible in the law, tests/test_noise_gpu.py
//     chi-square tests it at the reference's levels).  The extreme radius cell of the 16-bit grid
//     (u1 = 2^-16, |z| >= 4.71, probability 2^-16) is refined to 32 bits from a second block, so
//     |z| reaches 6.66 (P(|z| > 6.66) ~ 3e-11).
//   * float64 outputs (the plain branches, which hand the float64 image on): 53-bit uniforms and
//     an fp64 Box-Muller (noise.hip normal2_f64), numpy's op order, U8 = trunc(255 * out) exactly.
// Files that include this are compiled with -ffp-contract=off.
#pragma once

#include "idn_common.hpp"

namespace idn {

__device__ __forceinline__ double img_as_float(uint32_t v) { return __dmul_rn((double)v, 1.0 / 255.0); }

// np.clip(v, 0, 1) for non-NaN v (v_max_f64 / v_min_f64)
__device__ __forceinline__ double clip01(double v) { return __builtin_fmin(__builtin_fmax(v, 0.0), 1.0); }

// (255 * out).astype(np.uint8) for out in [0, 1]: truncation (out is never negative here)
__device__ __forceinline__ uint8_t u8_of(double out) { return (uint8_t)(int)__dmul_rn(out, 255.0); }

// eight standard normals from one Philox block (counter (q, 0, image id)): word p holds the pair's
// u1 (low 16 bits, (k + 1) 2^-16 in (0, 1]) and u2 (high 16 bits, in [0, 1)); Box-Muller on the
// fp32 hardware transcendentals (v_log / v_sqrt / v_sin / v_cos; sin / cos take revolutions, so
// theta = u2 needs no 2 pi multiply).  A pair in the cell k = 0 takes u1 = (j + 1) 2^-32 with j the
// low 16 bits of word p of the refinement block (counter (q, 3, image id)): a 32-bit uniform
// conditioned on that cell (rare: one lane block in 2^14 takes the branch).
__device__ __forceinline__ void normal8_16(const u32x4& r, uint32_t q, uint64_t gimg, uint64_t key,
                                           float (&z)[8]) {
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
  float u1[4];
  bool deep = false;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    u1[p] = ((float)(w[p] & 0xFFFFu) + 1.0f) * (1.0f / 65536.0f);
    deep |= (w[p] & 0xFFFFu) == 0u;
  }
  if (deep) {
    const u32x4 f = philox4x32<7>(u32x4{q, 3u, (uint32_t)gimg, (uint32_t)(gimg >> 32)}, key);
    const uint32_t fw[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
    for (int p = 0; p < 4; ++p)
      if ((w[p] & 0xFFFFu) == 0u) u1[p] = ((float)(fw[p] & 0xFFFFu) + 1.0f) * 0x1p-32f;
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float u2 = (float)(w[p] >> 16) * (1.0f / 65536.0f);
    const float rad =
        __builtin_amdgcn_sqrtf(-2.0f * 0.6931471805599453f * __builtin_amdgcn_logf(u1[p]));
    z[2 * p] = rad * __builtin_amdgcn_cosf(u2);
    z[2 * p + 1] = rad * __builtin_amdgcn_sinf(u2);
  }
}

// 16 consecutive elements e0 = 16 * chunk .. e0 + 15 of image `gimg` (flat element index): the
// u8 stream --
//   gaussian / speckle  counter (e/8, 0, image id) -> Philox4x32-7 -> normal8_16 -> the 8 normals
//                       of elements 8q..8q+7
//   s&p                 counter (e/4, 1, image id) -> Philox4x32-7 -> word b holds (U1, U2) of
//                       element 4q+b as 16-bit uniforms compared against integer thresholds
//                       (|P - p| < 2^-16)
// MEAN0: mean == 0.0 (one add per element less).  Returns the U8 bytes; s&p only: `of`
// (nullable) receives the 16 float64 values (1 / 0 / x, so U8 == trunc(255 * of) exactly).
template <int KIND, bool MEAN0>
__device__ __forceinline__ v4u noise16_u8(const v4u raw, uint32_t chunk, uint64_t gimg,
                                          uint64_t key, double p0, double p1, uint32_t t_flip,
                                          uint32_t t_salt, double* of) {
  const uint32_t in[4] = {raw.x, raw.y, raw.z, raw.w};
  uint32_t o[4] = {0u, 0u, 0u, 0u};
  float z8[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // elements 4k .. 4k+3
    if constexpr (KIND == IDN_NOISE_SAP) {
      // one Philox4x32-7 block per 4 elements (e / 4 = chunk * 4 + k): element b takes word b,
      // low 16 bits the `flipped` uniform, high 16 bits the `salted` one
      const uint32_t q = chunk * 4u + (uint32_t)k;
      const u32x4 r = philox4x32<7>(u32x4{q, 1u, (uint32_t)gimg, (uint32_t)(gimg >> 32)}, key);
      const uint32_t wd[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t v = (in[k] >> (8 * b)) & 0xFFu;
        const bool flip = (wd[b] & 0xFFFFu) < t_flip, salt = (wd[b] >> 16) < t_salt;
        // U8(255 * x) = trunc(255 * (v * (1/255))): v, or v - 1 for the 24 values that do not
        // round-trip (SURVEY 8 conventions)
        const uint32_t keep = u8_of(img_as_float(v));
        o[k] |= (flip ? (salt ? 255u : 0u) : keep) << (8 * b);
        if (of) of[4 * k + b] = flip ? (salt ? 1.0 : 0.0) : img_as_float(v);
      }
    } else {
      // one Philox4x32-7 block -> 8 normals for elements 8j .. 8j+7 (j = chunk * 2 + k / 2)
      if ((k & 1) == 0) {
        const uint32_t q = chunk * 2u + (uint32_t)(k >> 1);
        const u32x4 r = philox4x32<7>(u32x4{q, 0u, (uint32_t)gimg, (uint32_t)(gimg >> 32)}, key);
        normal8_16(r, q, gimg, key, z8);
      }
      const float* z = z8 + 4 * (k & 1);
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        // floor(clip(v + 255 n)) (gaussian) or floor(clip(v + v n)) (speckle) in fp32
        const float v = (float)((in[k] >> (8 * b)) & 0xFFu);
        float ov;
        if constexpr (KIND == IDN_NOISE_GAUSSIAN) {
          ov = __builtin_fmaf((float)(255.0 * p1), z[b], MEAN0 ? v : v + (float)(255.0 * p0));
        } else {
          const float n = MEAN0 ? (float)p1 * z[b] : __builtin_fmaf((float)p1, z[b], (float)p0);
          ov = __builtin_fmaf(v, n, v);
        }
        o[k] |= (uint32_t)__builtin_amdgcn_fmed3f(ov, 0.0f, 255.0f) << (8 * b);
      }
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
