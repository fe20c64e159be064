// skimage.util.random_noise modes used by the reference's noise closures, on u8 HxWxC batches:
//   gaussian  lib/model/test.py:193-307, minibatch.py:87-201   out = clip(x + N(mean, sd), 0, 1)
//   speckle   lib/model/test.py:476-590, minibatch.py:374-490  out = clip(x + x*N(mean, sd), 0, 1)
//   s&p       lib/model/test.py:357-474, minibatch.py:253-372  out = 1 / 0 / x by two uniforms
//   poisson   lib/model/test.py:309-355, minibatch.py:203-251  out = clip(P(x*vals)/vals, 0, 1)
// with x = v * (1/255) in float64 (img_as_float) and the caller's U8 cast (255*out).astype(uint8).
// The float64 op order is numpy's (file compiled with -ffp-contract=off; explicit _rn ops), so
// with a replayed random field (numpy's own draws) the outputs are bit-exact; with the Philox
// stream they are statistically equivalent (tests/test_noise_gpu.py).
//
// RNG: Philox4x32 keyed by (seed ^ kind tag); counter = (element group, stream tag, image id).
// Gaussian / speckle have two streams (noise_apply.hpp): u8-only outputs draw 16-bit uniforms
// (fp32 Box-Muller, fp32 apply on the 0..255 scale, tag 0, refinement tag 3); float64 outputs
// draw 53-bit uniforms with an fp64 Box-Muller (tag 2) and apply in numpy's float64 order, the
// U8 then being trunc(255 * out) of that value.  s&p (tag 1) and Poisson have one stream each.
// Every layout (flat 16-element kernels for compact rows, element kernels for strided ones) draws
// the same values.  Image id = offset + image index (or an id array), so a rank that owns images
// [a, b) of a batch draws exactly what a single GPU would for those images.
//
// Also: periodic noise pattern (add_periodic_noise, test.py:1128-1298) and cv2.add(u8, u8).
#include "idn_common.hpp"
#include "f64_math.hpp"
#include "noise_apply.hpp"
#include "ycc.hpp"

#include <math.h>

#include <algorithm>
#include <mutex>

namespace idn {

constexpr uint64_t KIND_TAG = 0x9E3779B97F4A7C15ull;

struct NoiseArgs {
  const uint8_t* src;
  uint8_t* out_u8;
  double* out_f64;
  const double* replay;
  const uint32_t* vals;  // poisson: per-image vals (power of two), workspace
  int n, h, w, c;
  int64_t row_stride;
  int64_t elems;  // h*w*c
  double p0, p1;  // mean/sd (gaussian, speckle), sap thresholds
  uint64_t key, offset;
  const uint64_t* ids;  // optional per-image ids (device); else id = offset + image index
  const int64_t* slots;  // optional batch positions (device): image i of the launch reads and
                         // writes image slots[i] of src / out_u8 / out_f64; else slot = i
  unsigned long long* ycc;  // noise_gauss_ycc_kernel: per image the colour range keys (ycc.hpp)
};
__device__ __forceinline__ uint64_t image_id(const NoiseArgs& a, int img) {
  return a.ids ? a.ids[img] : a.offset + (uint64_t)img;
}
__device__ __forceinline__ int64_t slot_of(const NoiseArgs& a, int img) {
  return a.slots ? a.slots[img] : (int64_t)img;
}

__device__ __forceinline__ void store_out(const NoiseArgs& a, int img, int64_t e, int64_t boff,
                                          double out) {
  if (a.out_f64) a.out_f64[slot_of(a, img) * a.elems + e] = out;
  if (a.out_u8) a.out_u8[boff] = u8_of(out);
}

// two standard normals in float64 from one Philox4x32-10 block (counter (pair, 2, image id)):
// 53-bit uniforms u1 = (a + 1) 2^-53 in (0, 1], u2 = b 2^-53 in [0, 1) (|z| <= 8.57),
// rad = sqrt(-2 ln u1), (cos, sin)(2 pi u2).  ln and (sin, cos) from the integers a + 1, b by the
// table-driven forms of f64_math.hpp (within ~1.4 ulp; the library log / sincospi, ~130 fp64
// operations per pair, made the float64 stream fp64-issue-bound)
// The tables live in LDS (F64mLds, staged once per workgroup): per-lane gathers from the
// __constant__ copies went through the vector L1 at one cache line per lane and cost more than
// the fp64 work they save.
struct F64mLds {
  double ln[f64m::LN_TAB_N];
  double sc[f64m::SC_TAB_N];
};
__device__ __forceinline__ void stage_f64m(F64mLds& t) {
  for (int i = threadIdx.x; i < f64m::LN_TAB_N; i += blockDim.x) t.ln[i] = f64m::LN_TAB[i];
  for (int i = threadIdx.x; i < f64m::SC_TAB_N; i += blockDim.x) t.sc[i] = f64m::SC_TAB[i];
  __syncthreads();
}
__device__ __forceinline__ void normal2_f64(const u32x4& r, const F64mLds& t, double& z0,
                                            double& z1) {
  const uint64_t a = ((uint64_t)r.x << 21) | (r.y >> 11), b = ((uint64_t)r.z << 21) | (r.w >> 11);
  const double rad = sqrt(fmax(-2.0 * f64m::ln_u53(a + 1, t.ln), 0.0));
  double sn, cs;
  f64m::sincos2pi_u53(b, t.sc, &sn, &cs);
  z0 = rad * cs;
  z1 = rad * sn;
}

// element form, one thread per element pair: the noise value n of each element is numpy's own
// draw (SRC_REPLAY: N(mean, sd) field, bit-exact with the reference) or mean + sd * z from the
// float64 stream (SRC_F64); out = clip(x + n) / clip(x + x n) in numpy's op order, U8 = trunc(255
// out).  Any row stride and slot layout.
enum NoiseSrc { SRC_REPLAY = 0, SRC_F64 = 1 };
template <int KIND, int SRC>
__global__ __launch_bounds__(256) void noise_gauss_kernel(NoiseArgs a) {
  __shared__ F64mLds tab;
  if constexpr (SRC == SRC_F64) stage_f64m(tab);
  const int64_t pairs = (a.elems + 1) / 2;
  const int64_t total = pairs * a.n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int img = (int)(t / pairs);
    const int64_t pr = t - (int64_t)img * pairs;
    double nz[2];
    if constexpr (SRC == SRC_REPLAY) {
      const int64_t e0 = 2 * pr;
      nz[0] = a.replay[(int64_t)img * a.elems + e0];
      nz[1] = (e0 + 1 < a.elems) ? a.replay[(int64_t)img * a.elems + e0 + 1] : 0.0;
    } else {
      const uint64_t gimg = image_id(a, img);
      const u32x4 r = philox4x32(u32x4{(uint32_t)pr, 2u ^ ((uint32_t)(pr >> 32) << 8),
                                       (uint32_t)gimg, (uint32_t)(gimg >> 32)},
                                 a.key);
      double z0, z1;
      normal2_f64(r, tab, z0, z1);
      // np.random.normal(mean, sd): loc + scale * gauss
      nz[0] = __dadd_rn(a.p0, __dmul_rn(a.p1, z0));
      nz[1] = __dadd_rn(a.p0, __dmul_rn(a.p1, z1));
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int64_t e = 2 * pr + s;
      if (e >= a.elems) break;
      const int64_t pix = e / a.c;
      const int ch = (int)(e - pix * a.c);
      const int y = (int)(pix / a.w), x = (int)(pix - (int64_t)y * a.w);
      const int64_t boff = slot_of(a, img) * a.h * a.row_stride + (int64_t)y * a.row_stride +
                           (int64_t)x * a.c + ch;
      const double xv = img_as_float(a.src[boff]);
      double out;
      if (KIND == IDN_NOISE_GAUSSIAN) out = clip01(__dadd_rn(xv, nz[s]));
      else out = clip01(__dadd_rn(xv, __dmul_rn(xv, nz[s])));
      store_out(a, img, e, boff, out);
    }
  }
}

// Float64 gaussian / speckle on compact 3-channel images, with the bior1.5 / Haar wavelet's colour
// range reduced on the fly (the live test path: random_noise's float64 image goes straight to
// denoise_wavelet, lib/model/test.py:1678-1684 -> 1807-1810).  One thread per pixel pair = the
// three element pairs 3q .. 3q+2 of noise_gauss_kernel (the same draws, the same op order: the
// image is bit-identical), plus per image the fp64 min / max of skimage rgb2ycbcr's three dot
// products of the output (ycc_dots, wl_color_minmax's chain), reduced per workgroup and folded
// into ycc[6 img ..] as order-preserving keys with the offsets added after the reduction -- what
// wl_color_minmax would compute from the stored image, without reading its 24 B/pixel back.
template <int KIND, int SRC>
__global__ __launch_bounds__(256) void noise_gauss_ycc_kernel(NoiseArgs a) {
  const int img = blockIdx.y;
  const int64_t npp = a.elems / 6;
  const int64_t slot = slot_of(a, img);
  const uint8_t* s = a.src + slot * a.elems;
  double* of = a.out_f64 + slot * a.elems;
  uint8_t* ou = a.out_u8 ? a.out_u8 + slot * a.elems : nullptr;
  const uint64_t gimg = image_id(a, img);
  __shared__ F64mLds tab;
  if constexpr (SRC == SRC_F64) stage_f64m(tab);
  double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < npp;
       q += (int64_t)gridDim.x * blockDim.x) {
    double nz[6];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int64_t pr = 3 * q + k;
      if constexpr (SRC == SRC_REPLAY) {
        nz[2 * k] = a.replay[(int64_t)img * a.elems + 2 * pr];
        nz[2 * k + 1] = a.replay[(int64_t)img * a.elems + 2 * pr + 1];
      } else {
        const u32x4 r = philox4x32(u32x4{(uint32_t)pr, 2u ^ ((uint32_t)(pr >> 32) << 8),
                                         (uint32_t)gimg, (uint32_t)(gimg >> 32)},
                                   a.key);
        double z0, z1;
        normal2_f64(r, tab, z0, z1);
        nz[2 * k] = __dadd_rn(a.p0, __dmul_rn(a.p1, z0));
        nz[2 * k + 1] = __dadd_rn(a.p0, __dmul_rn(a.p1, z1));
      }
    }
    const uint16_t* s2 = reinterpret_cast<const uint16_t*>(s + 6 * q);  // 2-byte aligned
    const uint32_t b01 = s2[0], b23 = s2[1], b45 = s2[2];
    const uint32_t bytes[6] = {b01 & 0xFFu, b01 >> 8, b23 & 0xFFu, b23 >> 8, b45 & 0xFFu, b45 >> 8};
    double out[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      const double xv = img_as_float(bytes[e]);
      out[e] = KIND == IDN_NOISE_GAUSSIAN ? clip01(__dadd_rn(xv, nz[e]))
                                          : clip01(__dadd_rn(xv, __dmul_rn(xv, nz[e])));
    }
    double2* o2 = reinterpret_cast<double2*>(of + 6 * q);  // 16-byte aligned (48 q bytes)
    o2[0] = make_double2(out[0], out[1]);
    o2[1] = make_double2(out[2], out[3]);
    o2[2] = make_double2(out[4], out[5]);
    if (ou) {
      uint16_t* u2 = reinterpret_cast<uint16_t*>(ou + 6 * q);
      u2[0] = (uint16_t)(u8_of(out[0]) | (u8_of(out[1]) << 8));
      u2[1] = (uint16_t)(u8_of(out[2]) | (u8_of(out[3]) << 8));
      u2[2] = (uint16_t)(u8_of(out[4]) | (u8_of(out[5]) << 8));
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      double d[3];
      ycc_dots(out[3 * p], out[3 * p + 1], out[3 * p + 2], d);
#pragma unroll
      for (int c = 0; c < 3; ++c) {  // finite values: fmin / fmax are plain selects
        mn[c] = fmin(mn[c], d[c]);
        mx[c] = fmax(mx[c], d[c]);
      }
    }
  }
  __shared__ double red[2][3][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double da = mn[c], db = mx[c];
    for (int o = 32; o > 0; o >>= 1) {
      da = fmin(da, __shfl_xor(da, o));
      db = fmax(db, __shfl_xor(db, o));
    }
    if (lane == 0) {
      red[0][c][wave] = da;
      red[1][c][wave] = db;
    }
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int c = threadIdx.x;
    double da = red[0][c][0], db = red[1][c][0];
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) {
      da = fmin(da, red[0][c][k]);
      db = fmax(db, red[1][c][k]);
    }
    if (da <= db) {  // a workgroup with no pixel leaves the keys alone
      atomicMin(a.ycc + 6 * img + c, dkey(__dadd_rn(da, ycc_offset(c))));
      atomicMax(a.ycc + 6 * img + 3 + c, dkey(__dadd_rn(db, ycc_offset(c))));
    }
  }
}

__global__ void ycc_keys_init(unsigned long long* keys, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 6 * n) keys[i] = (i % 6) < 3 ? ~0ull : 0ull;
}

// ---- u8 stream, flat form (compact rows): 16 consecutive elements per thread ------------------
// One 16-byte load / store per lane, image = blockIdx.y, no 64-bit index division; the stream is
// noise16_u8 (noise_apply.hpp).
template <int KIND, bool MEAN0 = false>
__global__ __launch_bounds__(256) void noise_flat16_kernel(NoiseArgs a, uint32_t t_flip,
                                                           uint32_t t_salt) {
  const int img = blockIdx.y;
  const uint32_t chunk = blockIdx.x * 256u + threadIdx.x;
  const int64_t e0 = (int64_t)chunk * 16;
  if (e0 >= a.elems) return;
  const uint64_t gimg = image_id(a, img);
  const int64_t base = slot_of(a, img) * a.elems + e0;
  const v4u raw = *reinterpret_cast<const v4u*>(a.src + base);
  const v4u o = noise16_u8<KIND, MEAN0>(raw, chunk, gimg, a.key, a.p0, a.p1, t_flip, t_salt,
                                        a.out_f64 ? a.out_f64 + base : nullptr);
  if (a.out_u8) *reinterpret_cast<v4u*>(a.out_u8 + base) = o;
}

// ---- u8 stream, element form (any layout): the same 16-element chunks gathered byte by byte ---
template <int KIND, bool MEAN0 = false>
__global__ __launch_bounds__(256) void noise_elem16_kernel(NoiseArgs a, uint32_t t_flip,
                                                           uint32_t t_salt) {
  const int64_t chunks = (a.elems + 15) / 16;
  const int64_t total = chunks * a.n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int img = (int)(t / chunks);
    const uint32_t chunk = (uint32_t)(t - (int64_t)img * chunks);
    const int64_t e0 = (int64_t)chunk * 16;
    int64_t off[16];
    uint32_t in[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int64_t e = e0 + i;
      off[i] = -1;
      if (e < a.elems) {
        const int64_t pix = e / a.c;
        const int ch = (int)(e - pix * a.c);
        const int y = (int)(pix / a.w), x = (int)(pix - (int64_t)y * a.w);
        off[i] = slot_of(a, img) * a.h * a.row_stride + (int64_t)y * a.row_stride +
                 (int64_t)x * a.c + ch;
        in[i >> 2] |= (uint32_t)a.src[off[i]] << (8 * (i & 3));
      }
    }
    double of[16];
    const v4u o = noise16_u8<KIND, MEAN0>(v4u{in[0], in[1], in[2], in[3]}, chunk, image_id(a, img),
                                          a.key, a.p0, a.p1, t_flip, t_salt,
                                          (KIND == IDN_NOISE_SAP && a.out_f64) ? of : nullptr);
    const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (off[i] < 0) continue;
      if (a.out_u8) a.out_u8[off[i]] = (uint8_t)(ow[i >> 2] >> (8 * (i & 3)));
      if (KIND == IDN_NOISE_SAP && a.out_f64) a.out_f64[slot_of(a, img) * a.elems + e0 + i] = of[i];
    }
  }
}

// salt & pepper, replay: flipped = U1 < cdf0(amount), salted = U2 < cdf0(salt_vs_pepper) on
// numpy's own random_sample fields
__global__ __launch_bounds__(256) void noise_sap_kernel(NoiseArgs a) {
  const int64_t total = a.elems * a.n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int img = (int)(t / a.elems);
    const int64_t e = t - (int64_t)img * a.elems;
    const double u1 = a.replay[t], u2 = a.replay[total + t];
    const int64_t pix = e / a.c;
    const int ch = (int)(e - pix * a.c);
    const int y = (int)(pix / a.w), x = (int)(pix - (int64_t)y * a.w);
    const int64_t boff =
        slot_of(a, img) * a.h * a.row_stride + (int64_t)y * a.row_stride + (int64_t)x * a.c + ch;
    double out = img_as_float(a.src[boff]);
    if (u1 < a.p0) out = (u2 < a.p1) ? 1.0 : 0.0;
    store_out(a, img, e, boff, out);
  }
}

// per-image distinct-value mask (256 bits) -> vals = 2^ceil(log2(#distinct))
__global__ __launch_bounds__(256) void unique_mask_kernel(const uint8_t* __restrict__ src, int h,
                                                          int rowbytes, int64_t row_stride,
                                                          const int64_t* __restrict__ slots,
                                                          uint32_t* __restrict__ mask) {
  __shared__ uint32_t m[8];
  if (threadIdx.x < 8) m[threadIdx.x] = 0;
  __syncthreads();
  const int img = blockIdx.y;
  const uint8_t* s = src + (slots ? slots[img] : (int64_t)img) * h * row_stride;
  const int64_t total = (int64_t)h * rowbytes;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int y = (int)(i / rowbytes);
    const uint32_t v = s[(int64_t)y * row_stride + (i - (int64_t)y * rowbytes)];
    atomicOr(&m[v >> 5], 1u << (v & 31));
  }
  __syncthreads();
  if (threadIdx.x < 8 && m[threadIdx.x]) atomicOr(&mask[img * 8 + threadIdx.x], m[threadIdx.x]);
}

__global__ void vals_from_mask_kernel(uint32_t* mask, int n) {
  const int img = blockIdx.x * blockDim.x + threadIdx.x;
  if (img >= n) return;
  int cnt = 0;
  for (int k = 0; k < 8; ++k) cnt += __popc(mask[img * 8 + k]);
  uint32_t v = 1;
  while ((int)v < cnt) v <<= 1;  // 2**ceil(log2(cnt)); cnt == 1 -> 1
  mask[8 * n + img] = v;
}

// Philox-stream Poisson by inversion of the exact CDF.  lambda = img_as_float(v) * vals takes one
// of 256 values per power-of-two vals (vals <= 256), so the CDF row of every
// (vals, v) is tabulated per call (POIS_KMAX entries; P(X >= 512) < 1e-25 at lambda = 256, the
// largest).  A draw's 32-bit Philox word w gives u = (w + 1/2) / 2^32 and the count
//   k = min { k : cdf[k] > u }  =  min { k : w < t_k },   t_k = ceil(cdf[k] * 2^32 - 1/2)
// (the integer thresholds t_k are exact restatements of the double compares).  The law is
// numpy's (Knuth / PTRS sample the same Poisson(lambda)); the replay mode takes numpy's own draws
// bit-exactly.
//
// The tables depend on nothing but vals, so they are built once per device (pois_tables_for)
// and kept.  Flat kernel (round 2): per vals level a 154 KB block staged in LDS, per v
//   * the thresholds t_k over the window [lo_v, hi_v + 2], hi_v - lo_v = the counts of u in
//     [2^-16, 1 - 2^-16]  (+-4.2 sd; 23.4 K u32 over the 256 v at vals = 256)
//   * a guide over the bins of w, geometric towards both ends: per side, the octaves
//     [2^p, 2^(p+1)) of the distance x from the nearer end for p = 16 .. 30, each split in
//     POIS_S, and one deep bin (x < 2^16); it holds each bin's first count.  Every bin spans
//     <= 3 counts, so k = first + [w >= t_first] + [w >= t_first+1] + [w >= t_first+2]:
//     thresholds past the bin's last count exceed every w of the bin, so the sum needs no span.
//   * a header: the LDS dword index of t_0 for v (window start - lo_v, biased by the T offset).
// A draw is a header, a guide and 3 threshold reads -- branch-free.
// The deep bins (u < 2^-16 or u > 1 - 2^-16, 1 draw in 32 K) bisect the global CDF row.
// Round 1 bisected the global rows for every draw (1 guide + 1-3 CDF probes in L2, 64-byte
// transactions for 4-8 useful bytes): L2-bound at 1.96 ms per 256 images.
constexpr int POIS_NV = 9;       // vals = 1, 2, 4, ..., 256
constexpr int POIS_KMAX = 512;   // CDF entries per lambda
constexpr int POIS_PMIN = 16;    // smallest octave exponent of a guided bin (x >= 2^16)
constexpr int POIS_LS = 2;       // log2 of the bins per octave
constexpr int POIS_S = 1 << POIS_LS;
constexpr int POIS_NBH = 1 + (31 - POIS_PMIN) * POIS_S;  // bins per side, deep bin 0 (61)
constexpr int POIS_NG = 2 * POIS_NBH;                    // guide entries per v (122)
constexpr int POIS_SPAN = 3;                             // max counts per bin
constexpr int POIS_TCAP = 23552;                         // window thresholds per level
// level block: HDR[256] u32 (T_BASE + window start - lo_v), GUIDE[256][POIS_NG] u16 (first
// count; side-major: [side][j]), T[POIS_TCAP] u32
constexpr size_t POIS_LVL_G = 256 * sizeof(uint32_t);
constexpr size_t POIS_LVL_T = (POIS_LVL_G + 256 * POIS_NG * sizeof(uint16_t) + 15) & ~(size_t)15;
constexpr size_t POIS_LVL_BYTES = POIS_LVL_T + POIS_TCAP * sizeof(uint32_t);  // 157696
constexpr uint32_t POIS_T_BASE = POIS_LVL_T / 4;
struct PoisTables {
  double* cdf;       // [POIS_NV][256][POIS_KMAX]
  uint8_t* levels;   // [POIS_NV] blocks of POIS_LVL_BYTES
  uint32_t* ntab;    // [POIS_NV] thresholds used per level (> POIS_TCAP: level not staged)
};
__device__ __forceinline__ double pois_u(uint32_t w) {
  return fma((double)w, 0x1p-32, 0x1p-33);  // exact: 33 significant bits
}
__device__ __forceinline__ int pois_first_above(const double* cdf, double q) {
  int lo = 0, hi = POIS_KMAX - 1;  // cdf[KMAX-1] = 1 > q
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cdf[mid] > q) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}
// guide position of a word: side * POIS_NBH + j, j = 0 the deep bin.  x >> 7 < 2^24 converts to
// float exactly; its exponent and top POIS_LS mantissa bits are the octave and the split.
__device__ __forceinline__ uint32_t pois_side(uint32_t w) { return w >> 31; }
__device__ __forceinline__ int pois_bin(uint32_t w) {
  const uint32_t x = w ^ (uint32_t)((int32_t)w >> 31);  // distance from the nearer end, < 2^31
  const int eb = (int)(__float_as_uint((float)(x >> 7)) >> (23 - POIS_LS));
  return max(eb - (((127 - 7 + POIS_PMIN) << POIS_LS) - 1), 0);
}
// first distance x of bin j >= 1 (the octave 2^p, p = POIS_PMIN + (j-1) / S, split (j-1) % S)
__device__ __forceinline__ uint32_t pois_x_start(int j) {
  const int p = POIS_PMIN + (j - 1) / POIS_S, m = (j - 1) % POIS_S;
  return (1u << p) + ((uint32_t)m << (p - POIS_LS));
}
__device__ __forceinline__ uint32_t pois_x_end(int j) {
  return j == POIS_NBH - 1 ? 0x7FFFFFFFu : pois_x_start(j + 1) - 1u;
}
// the i-th bin endpoint in increasing w: side 0 bins j = 1 .. NBH-1 (start, end), then side 1
// bins j = NBH-1 .. 1 (start, end) where side 1's w = ~x
constexpr int POIS_NEP = 4 * (POIS_NBH - 1);
__device__ __forceinline__ uint32_t pois_endpoint(int i) {
  const int bin = i >> 1;
  if (bin < POIS_NBH - 1) {
    const int j = bin + 1;
    return (i & 1) ? pois_x_end(j) : pois_x_start(j);
  }
  const int j = POIS_NBH - 1 - (bin - (POIS_NBH - 1));
  return (i & 1) ? ~pois_x_start(j) : ~pois_x_end(j);
}
__device__ __forceinline__ uint32_t pois_threshold(double c) {
  const double t = ceil(fma(c, 0x1p32, -0.5));  // exact: c * 2^32 <= 2^32 has ulp <= 2^-20
  return t <= 0.0 ? 0u : t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}
// one workgroup per vals level, thread = v: the CDF row by the recurrence
// p(k+1) = p(k) * lambda / (k+1) (written to global for the element kernel and the deep bins),
// with a two-pointer pass over the bin endpoints in the same loop; then the guide, the window
// starts (prefix sum over v) and the thresholds
__global__ __launch_bounds__(256) void pois_level_kernel(PoisTables t) {
  __shared__ uint32_t scan[256];
  __shared__ int bad;
  const int vi = blockIdx.x, v = threadIdx.x;
  double* cdf = t.cdf + ((size_t)vi * 256 + v) * POIS_KMAX;
  uint8_t* lvl = t.levels + (size_t)vi * POIS_LVL_BYTES;
  uint16_t* guide = reinterpret_cast<uint16_t*>(lvl + POIS_LVL_G) + (size_t)v * POIS_NG;
  if (v == 0) bad = 0;
  const double lam = __dmul_rn(img_as_float((uint32_t)v), (double)(1u << vi));
  double p = exp(-lam), acc = 0.0;
  int ep = 0, lo = 0, first = 0, hi = 0;
  bool fits = true;
  double ue = pois_u(pois_endpoint(0));
  for (int k = 0; k < POIS_KMAX; ++k) {
    acc += p;
    const double c = k == POIS_KMAX - 1 ? 1.0 : fmin(acc, 1.0);
    cdf[k] = c;
    p = p * lam / (double)(k + 1);
    while (ep < POIS_NEP && c > ue) {  // endpoint ep's count is k
      if (ep == 0) lo = k;
      if (!(ep & 1)) {
        first = k;
      } else {  // bin ep/2 spans counts [first, k]
        const int bin = ep >> 1;
        const int pos = bin < POIS_NBH - 1 ? bin + 1 : POIS_NG - 1 - (bin - (POIS_NBH - 1));
        fits &= k - first <= POIS_SPAN;
        guide[pos] = (uint16_t)first;
        hi = k;
      }
      if (++ep < POIS_NEP) ue = pois_u(pois_endpoint(ep));
    }
  }
  guide[0] = (uint16_t)lo;
  guide[POIS_NBH] = (uint16_t)lo;  // deep bins: any in-window read, the result is replaced
  __syncthreads();
  if (!fits) bad = 1;
  const uint32_t width = (uint32_t)(hi - lo + 3);  // thresholds lo .. hi + 2
  scan[v] = width;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {  // inclusive scan
    const uint32_t add = v >= d ? scan[v - d] : 0u;
    __syncthreads();
    scan[v] += add;
    __syncthreads();
  }
  const uint32_t start = scan[v] - width, total = scan[255];
  reinterpret_cast<uint32_t*>(lvl)[v] = POIS_T_BASE + start - (uint32_t)lo;
  if (total > POIS_TCAP || bad || hi + 2 >= POIS_KMAX) {
    if (v == 0) t.ntab[vi] = POIS_TCAP + 1;  // not staged: the flat kernel bisects the rows
    return;
  }
  if (v == 0) t.ntab[vi] = total;
  uint32_t* T = reinterpret_cast<uint32_t*>(lvl + POIS_LVL_T);
  for (uint32_t i = 0; i < width; ++i) T[start + i] = pois_threshold(cdf[lo + i]);
}

// element e's uniform: 4 consecutive elements share one Philox block (counter (e/4, tag, image
// id)), element e takes word e % 4
__device__ __forceinline__ u32x4 pois_block(uint64_t key, uint64_t q, uint64_t gimg) {
  return philox4x32<7>(u32x4{(uint32_t)q, (uint32_t)(q >> 32) ^ 0x80000000u, (uint32_t)gimg,
                             (uint32_t)(gimg >> 32)}, key);
}
__device__ __forceinline__ int vals_index(uint32_t vals) { return __ffs((int)vals) - 1; }

// the element form: the definition, bisecting the CDF row in global memory
__global__ __launch_bounds__(256) void noise_poisson_kernel(NoiseArgs a, PoisTables pt) {
  const int64_t total = a.elems * a.n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int img = (int)(t / a.elems);
    const int64_t e = t - (int64_t)img * a.elems;
    const int64_t pix = e / a.c;
    const int ch = (int)(e - pix * a.c);
    const int y = (int)(pix / a.w), x = (int)(pix - (int64_t)y * a.w);
    const int64_t boff =
        slot_of(a, img) * a.h * a.row_stride + (int64_t)y * a.row_stride + (int64_t)x * a.c + ch;
    const double vals = (double)a.vals[img];
    double k;
    if (a.replay) {
      k = a.replay[t];
    } else {
      const u32x4 r = pois_block(a.key, (uint64_t)e >> 2, image_id(a, img));
      const int q = (int)(e & 3);
      const uint32_t w = q == 0 ? r.x : q == 1 ? r.y : q == 2 ? r.z : r.w;
      const double* cdf =
          pt.cdf + ((size_t)vals_index(a.vals[img]) * 256 + a.src[boff]) * POIS_KMAX;
      k = (double)pois_first_above(cdf, pois_u(w));
    }
    store_out(a, img, e, boff, clip01(k / vals));
  }
}

// flat Poisson (compact rows, Philox stream): work units = (image, part) pairs over a grid of one
// workgroup per CU, the unit's level block staged in LDS (re-staged only when the level changes),
// 16 consecutive elements per thread per step; the same uniforms and the same inversion as
// noise_poisson_kernel, so the two forms agree bit for bit
constexpr int POIS_FLAT_WGT = 1024;
__global__ __launch_bounds__(POIS_FLAT_WGT) void noise_poisson_flat_kernel(NoiseArgs a,
                                                                           PoisTables pt,
                                                                           int parts) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[POIS_LVL_BYTES];
  const uint32_t* HDR = reinterpret_cast<const uint32_t*>(lds);
  const uint16_t* GUIDE = reinterpret_cast<const uint16_t*>(lds + POIS_LVL_G);
  const uint32_t* L32 = reinterpret_cast<const uint32_t*>(lds);  // T[k] of v: L32[HDR[v] + k]
  const int64_t nq = a.elems / 16;
  const int units = a.n * parts;
  int staged = -1;
  for (int unit = blockIdx.x; unit < units; unit += gridDim.x) {
    const int img = unit / parts, part = unit - img * parts;
    const uint32_t vraw = a.vals[img];
    const int vi = vals_index(vraw);
    const bool in_lds = pt.ntab[vi] <= (uint32_t)POIS_TCAP;
    if (vi != staged) {  // uniform over the workgroup
      __syncthreads();
      if (in_lds) {
        const v4u* src = reinterpret_cast<const v4u*>(pt.levels + (size_t)vi * POIS_LVL_BYTES);
        const int n16 = (int)((POIS_LVL_T + pt.ntab[vi] * sizeof(uint32_t) + 15) / 16);
        v4u* dst = reinterpret_cast<v4u*>(lds);
        for (int i = threadIdx.x; i < n16; i += POIS_FLAT_WGT) dst[i] = src[i];
      }
      __syncthreads();
      staged = vi;
    }
    const double* cdf_lvl = pt.cdf + (size_t)vi * 256 * POIS_KMAX;
    const double inv_vals = 1.0 / (double)vraw;  // power of two: k * inv_vals == k / vals
    const uint64_t gimg = image_id(a, img);
    const int64_t q0 = nq * part / parts, q1 = nq * (part + 1) / parts;
    for (int64_t q = q0 + threadIdx.x; q < q1; q += POIS_FLAT_WGT) {
      const int64_t e0 = q * 16;
      const int64_t base = slot_of(a, img) * a.elems + e0;
      const v4u raw = *reinterpret_cast<const v4u*>(a.src + base);
      const uint32_t in[4] = {raw.x, raw.y, raw.z, raw.w};
      double* of = a.out_f64 ? a.out_f64 + base : nullptr;
      uint32_t o[4];
#pragma unroll
      for (int hf = 0; hf < 4; ++hf) {  // 4 groups of 4 elements, one Philox block each
        const u32x4 r = pois_block(a.key, (uint64_t)(e0 >> 2) + hf, gimg);
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
        int k[4], jmin = POIS_NBH;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t v = (in[hf] >> (8 * i)) & 0xFFu;
          const int j = pois_bin(w[i]);
          jmin = min(jmin, j);
          const uint32_t k0 = GUIDE[v * POIS_NG + pois_side(w[i]) * POIS_NBH + j];
          const uint32_t* t = L32 + HDR[v] + k0;
          const uint32_t t0 = t[0], t1 = t[1], t2 = t[2];
          k[i] = (int)k0 + (w[i] >= t0) + (w[i] >= t1) + (w[i] >= t2);
        }
        if (!in_lds || __any(jmin == 0)) {  // deep bins (1 draw in 32 K) or an unstaged level
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (!in_lds || pois_bin(w[i]) == 0) {
              const uint32_t v = (in[hf] >> (8 * i)) & 0xFFu;
              k[i] = pois_first_above(cdf_lvl + (size_t)v * POIS_KMAX, pois_u(w[i]));
            }
          }
        }
        o[hf] = 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // trunc(255 * min(k / vals, 1)), exact in integers
          o[hf] |= min((uint32_t)(255 * k[i]) >> vi, 255u) << (8 * i);
          if (of) of[4 * hf + i] = clip01(__dmul_rn((double)k[i], inv_vals));
        }
      }
      if (a.out_u8) *reinterpret_cast<v4u*>(a.out_u8 + base) = v4u{o[0], o[1], o[2], o[3]};
    }
  }
}

// flat per-image distinct-value mask: 16 bytes per thread per step, a private 256-bit mask per
// thread, OR-reduced over the wave before one LDS atomic per word.  vals only needs the count
// up to 2^ceil(log2(count)): once a block's own mask holds more than 128 values, vals = 256 is
// certain whatever the rest of the image holds, so the block stops (checked every 4 steps).
__global__ __launch_bounds__(256) void unique_mask_flat_kernel(const uint8_t* __restrict__ src,
                                                               int64_t per_img,
                                                               const int64_t* __restrict__ slots,
                                                               uint32_t* __restrict__ mask) {
  __shared__ uint32_t m[8];
  __shared__ int full;
  if (threadIdx.x < 8) m[threadIdx.x] = 0;
  __syncthreads();
  const int img = blockIdx.y;
  const v4u* s =
      reinterpret_cast<const v4u*>(src + (slots ? slots[img] : (int64_t)img) * per_img);
  const int64_t nq = per_img / 16;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  uint32_t mk[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // block-uniform trip count: every thread reaches the __syncthreads of the checks
  const int64_t q0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t steps = q0 < nq ? (nq - q0 + stride - 1) / stride : 0;
  for (int64_t it = 0; it < steps; ++it, q += stride) {
    if (q < nq) {
      const v4u v = s[q];
      const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int b = 0; b < 16; ++b) {
        const uint32_t x = (d[b >> 2] >> (8 * (b & 3))) & 0xFFu;
        const uint32_t bit = 1u << (x & 31u), word = x >> 5;
#pragma unroll
        for (int k = 0; k < 8; ++k) mk[k] |= word == (uint32_t)k ? bit : 0u;
      }
    }
    if ((it & 3) == 3 && it + 1 < steps) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        uint32_t v = mk[k];
        for (int off = 32; off > 0; off >>= 1) v |= (uint32_t)__shfl_xor((int)v, off);
        if ((threadIdx.x & 63) == 0 && v) atomicOr(&m[k], v);
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        int cnt = 0;
        for (int k = 0; k < 8; ++k) cnt += __popc(m[k]);
        full = cnt > 128;
      }
      __syncthreads();
      if (full) break;
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint32_t v = mk[k];
    for (int off = 32; off > 0; off >>= 1) v |= (uint32_t)__shfl_xor((int)v, off);
    if ((threadIdx.x & 63) == 0 && v) atomicOr(&m[k], v);
  }
  __syncthreads();
  if (threadIdx.x < 8 && m[threadIdx.x]) atomicOr(&mask[img * 8 + threadIdx.x], m[threadIdx.x]);
}

// cv2.add(u8, u8) on compact rows, 16 bytes per thread: SWAR saturating byte add
__device__ __forceinline__ uint32_t addsat_u8x4(uint32_t a, uint32_t b) {
  const uint32_t low7 = (a & 0x7F7F7F7Fu) + (b & 0x7F7F7F7Fu);  // no carry out of any byte
  const uint32_t sum = low7 ^ ((a ^ b) & 0x80808080u);          // byte sums mod 256
  const uint32_t carry = ((a & b) | ((a | b) & ~sum)) & 0x80808080u;
  return sum | ((carry >> 7) * 0xFFu);
}
__global__ __launch_bounds__(256) void add_pattern_flat_kernel(const uint8_t* __restrict__ src,
                                                               const uint8_t* __restrict__ pat,
                                                               uint8_t* __restrict__ dst,
                                                               int64_t per_img,
                                                               const int64_t* __restrict__ slots) {
  const int img = blockIdx.y;
  const int64_t nq = per_img / 16;
  const int64_t base = (slots ? slots[img] : (int64_t)img) * per_img;
  const v4u* s = reinterpret_cast<const v4u*>(src + base);
  const v4u* p = reinterpret_cast<const v4u*>(pat);
  v4u* d = reinterpret_cast<v4u*>(dst + base);
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq;
       q += (int64_t)gridDim.x * blockDim.x) {
    const v4u a = s[q], b = p[q];
    d[q] = v4u{addsat_u8x4(a.x, b.x), addsat_u8x4(a.y, b.y), addsat_u8x4(a.z, b.z),
               addsat_u8x4(a.w, b.w)};
  }
}

// periodic pattern: t_i = i*step + (-A) (numpy linspace op order), t_last = A
__global__ __launch_bounds__(256) void periodic_kernel(uint8_t* __restrict__ pat, int64_t size,
                                                       double amp, double step) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < size;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double t = (i == size - 1) ? amp : __dadd_rn(__dmul_rn((double)i, step), -amp);
    const double y = __dmul_rn(sin(t), 255.0);
    // (uint8)(int32)trunc(y): truncate toward zero, wrap mod 256
    pat[i] = (uint8_t)(int)y;
  }
}

// cv2.add(u8, u8) = min(a + b, 255), 16 bytes per thread where aligned
__global__ __launch_bounds__(256) void add_pattern_kernel(const uint8_t* __restrict__ src,
                                                          const uint8_t* __restrict__ pat,
                                                          uint8_t* __restrict__ dst, int n, int h,
                                                          int rowbytes, int64_t row_stride,
                                                          const int64_t* __restrict__ slots) {
  const int64_t per_img = (int64_t)h * rowbytes;
  const int64_t total = per_img * n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int img = (int)(i / per_img);
    const int64_t e = i - (int64_t)img * per_img;
    const int y = (int)(e / rowbytes);
    const int64_t off = (slots ? slots[img] : (int64_t)img) * h * row_stride +
                        (int64_t)y * row_stride + (e - (int64_t)y * rowbytes);
    const uint32_t s = (uint32_t)src[off] + (uint32_t)pat[e];
    dst[off] = (uint8_t)(s > 255u ? 255u : s);
  }
}

static unsigned grid_for(int64_t work, int64_t cap = 65536) {
  int64_t b = (work + 255) / 256;
  if (b < 1) b = 1;
  return (unsigned)(b > cap ? cap : b);
}

}  // namespace idn

// poisson: per-image distinct-value masks + vals, then the inversion tables (256-byte aligned)
static size_t pois_tables_off(int n) {
  return ((size_t)n * 9 * sizeof(uint32_t) + 255) & ~(size_t)255;
}
extern "C" size_t idn_noise_workspace_size(int kind, int n) {
  if (kind != IDN_NOISE_POISSON || n <= 0) return 0;
  return pois_tables_off(n);  // per-image distinct-value masks and vals
}

namespace idn {
// the Poisson tables of the current device, built on first use (on `st`, then synchronised) and
// kept for the life of the process: 9.4 MB of CDF rows + 9 level blocks of 154 KB
static int pois_tables_for(hipStream_t st, PoisTables* out) {
  static std::mutex mu;
  static PoisTables cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
    return set_error(IDN_EHIP, "poisson tables: no device");
  std::lock_guard<std::mutex> lock(mu);
  if (!cache[dev].cdf) {
    PoisTables pt;
    const size_t cdf_bytes = (size_t)POIS_NV * 256 * POIS_KMAX * sizeof(double);
    const size_t bytes = cdf_bytes + (size_t)POIS_NV * POIS_LVL_BYTES + 16 * sizeof(uint32_t);
    void* mem = nullptr;
    if (hipMalloc(&mem, bytes) != hipSuccess)
      return set_error(IDN_EHIP, "poisson tables: hipMalloc(%zu) failed", bytes);
    pt.cdf = reinterpret_cast<double*>(mem);
    pt.levels = reinterpret_cast<uint8_t*>(mem) + cdf_bytes;
    pt.ntab = reinterpret_cast<uint32_t*>(pt.levels + (size_t)POIS_NV * POIS_LVL_BYTES);
    hipLaunchKernelGGL(pois_level_kernel, dim3(POIS_NV), dim3(256), 0, st, pt);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
      (void)hipFree(mem);
      return set_error(IDN_EHIP, "poisson tables: build failed");
    }
    cache[dev] = pt;
  }
  *out = cache[dev];
  return IDN_OK;
}
}  // namespace idn

extern "C" int idn_poisson_levels(uint32_t* ntab_out, uint32_t* cap_out, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(ntab_out && cap_out, "idn_poisson_levels: null pointer");
  hipStream_t st = as_stream(stream);
  PoisTables pt;
  const int rc = pois_tables_for(st, &pt);
  if (rc != IDN_OK) return rc;
  if (hipMemcpyAsync(ntab_out, pt.ntab, POIS_NV * sizeof(uint32_t), hipMemcpyDeviceToHost, st) !=
          hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return set_error(IDN_EHIP, "idn_poisson_levels: copy failed");
  cap_out[0] = POIS_TCAP;
  return IDN_OK;
}

namespace idn {
static int noise_u8_impl(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n, int h, int w,
                         int c, int64_t row_stride, int kind, double p0, double p1, uint64_t seed,
                         uint64_t offset, const uint64_t* ids, const int64_t* slots,
                         const double* replay,
                         void* workspace, size_t ws_bytes, void* stream) {
  IDN_CHECK_ARG(src, "idn_noise_u8: null src");
  IDN_CHECK_ARG(out_u8 || out_f64, "idn_noise_u8: at least one of out_u8 / out_f64 is required");
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0 && c >= 1 && c <= 4, "idn_noise_u8: bad shape");
  // the per-image kernels put the image on gridDim.y
  IDN_CHECK_ARG(n <= 65535, "idn_noise_u8: at most 65535 images per call (got %d)", n);
  IDN_CHECK_ARG(row_stride >= (int64_t)w * c, "idn_noise_u8: row_stride < w*c");
  IDN_CHECK_ARG(kind >= 0 && kind <= 3, "idn_noise_u8: unknown noise kind %d", kind);
  IDN_CHECK_ARG((const void*)out_u8 != (const void*)src || kind != IDN_NOISE_POISSON,
                "idn_noise_u8: poisson cannot run in place");
  if (n == 0) return IDN_OK;
  hipStream_t st = as_stream(stream);
  NoiseArgs a;
  a.src = src;
  a.out_u8 = out_u8;
  a.out_f64 = out_f64;
  a.replay = replay;
  a.vals = nullptr;
  a.n = n;
  a.h = h;
  a.w = w;
  a.c = c;
  a.row_stride = row_stride;
  a.elems = (int64_t)h * w * c;
  a.key = seed ^ (KIND_TAG * (uint64_t)(kind + 1));
  a.offset = offset;
  a.ids = ids;
  a.slots = slots;
  // flat form: Philox stream, compact rows, 16-element chunks that never straddle images
  const bool flat = !replay && row_stride == (int64_t)w * c && a.elems % 16 == 0 &&
                    ((uintptr_t)src & 15) == 0 && ((uintptr_t)out_u8 & 15) == 0 &&
                    ((uintptr_t)out_f64 & 7) == 0 && a.elems / 16 < ((int64_t)1 << 31);
  IDN_CHECK_ARG((a.elems + 15) / 16 < ((int64_t)1 << 32), "idn_noise_u8: image too large");
  const unsigned g16 = grid_for((a.elems + 15) / 16 * n);
  switch (kind) {
    case IDN_NOISE_GAUSSIAN:
    case IDN_NOISE_SPECKLE: {
      IDN_CHECK_ARG(p1 >= 0.0, "idn_noise_u8: var must be >= 0");
      a.p0 = p0;             // mean
      a.p1 = pow(p1, 0.5);   // var ** 0.5 (random_noise)
      const int64_t work = (a.elems + 1) / 2 * n;
      const bool g = kind == IDN_NOISE_GAUSSIAN, m0 = a.p0 == 0.0;
      if (replay || out_f64) {  // numpy's field, or the float64 stream: float64 apply
        if (replay && g)
          hipLaunchKernelGGL((noise_gauss_kernel<IDN_NOISE_GAUSSIAN, SRC_REPLAY>), dim3(grid_for(work)), dim3(256), 0, st, a);
        else if (replay)
          hipLaunchKernelGGL((noise_gauss_kernel<IDN_NOISE_SPECKLE, SRC_REPLAY>), dim3(grid_for(work)), dim3(256), 0, st, a);
        else if (g)
          hipLaunchKernelGGL((noise_gauss_kernel<IDN_NOISE_GAUSSIAN, SRC_F64>), dim3(grid_for(work)), dim3(256), 0, st, a);
        else
          hipLaunchKernelGGL((noise_gauss_kernel<IDN_NOISE_SPECKLE, SRC_F64>), dim3(grid_for(work)), dim3(256), 0, st, a);
      } else if (flat) {
        const dim3 grid((unsigned)((a.elems / 16 + 255) / 256), (unsigned)n);
        if (g && m0)
          hipLaunchKernelGGL((noise_flat16_kernel<IDN_NOISE_GAUSSIAN, true>), grid, dim3(256), 0, st, a, 0u, 0u);
        else if (g)
          hipLaunchKernelGGL(noise_flat16_kernel<IDN_NOISE_GAUSSIAN>, grid, dim3(256), 0, st, a, 0u, 0u);
        else if (m0)
          hipLaunchKernelGGL((noise_flat16_kernel<IDN_NOISE_SPECKLE, true>), grid, dim3(256), 0, st, a, 0u, 0u);
        else
          hipLaunchKernelGGL(noise_flat16_kernel<IDN_NOISE_SPECKLE>, grid, dim3(256), 0, st, a, 0u, 0u);
      } else if (g && m0) {
        hipLaunchKernelGGL((noise_elem16_kernel<IDN_NOISE_GAUSSIAN, true>), dim3(g16), dim3(256), 0, st, a, 0u, 0u);
      } else if (g) {
        hipLaunchKernelGGL(noise_elem16_kernel<IDN_NOISE_GAUSSIAN>, dim3(g16), dim3(256), 0, st, a, 0u, 0u);
      } else if (m0) {
        hipLaunchKernelGGL((noise_elem16_kernel<IDN_NOISE_SPECKLE, true>), dim3(g16), dim3(256), 0, st, a, 0u, 0u);
      } else {
        hipLaunchKernelGGL(noise_elem16_kernel<IDN_NOISE_SPECKLE>, dim3(g16), dim3(256), 0, st, a, 0u, 0u);
      }
      break;
    }
    case IDN_NOISE_SAP: {
      IDN_CHECK_ARG(p0 >= 0.0 && p0 <= 1.0 && p1 >= 0.0 && p1 <= 1.0,
                    "idn_noise_u8: amount / salt_vs_pepper must be in [0, 1]");
      // np.random.choice([True, False], p=[p, 1-p]): True iff random_sample < cdf[0]
      a.p0 = p0 / (p0 + (1.0 - p0));
      a.p1 = p1 / (p1 + (1.0 - p1));
      const uint32_t tf = sap_threshold(a.p0), ts = sap_threshold(a.p1);
      if (replay) {
        hipLaunchKernelGGL(noise_sap_kernel, dim3(grid_for(a.elems * n)), dim3(256), 0, st, a);
      } else if (flat) {
        // 16-bit uniform thresholds: P(u < t / 2^16) within 2^-16 of cdf0
        const dim3 grid((unsigned)((a.elems / 16 + 255) / 256), (unsigned)n);
        hipLaunchKernelGGL(noise_flat16_kernel<IDN_NOISE_SAP>, grid, dim3(256), 0, st, a, tf, ts);
      } else {
        hipLaunchKernelGGL(noise_elem16_kernel<IDN_NOISE_SAP>, dim3(g16), dim3(256), 0, st, a, tf, ts);
      }
      break;
    }
    default: {  // POISSON
      const size_t need = idn_noise_workspace_size(kind, n);
      IDN_CHECK_ARG(workspace && ws_bytes >= need,
                    "idn_noise_u8: poisson needs %zu workspace bytes (got %zu)", need, ws_bytes);
      uint32_t* mask = (uint32_t*)workspace;
      if (hipMemsetAsync(mask, 0, (size_t)n * 8 * sizeof(uint32_t), st) != hipSuccess)
        return set_error(IDN_EHIP, "idn_noise_u8: memset failed");
      const int64_t per_img = (int64_t)h * w * c;
      const bool compact = row_stride == (int64_t)w * c && per_img % 16 == 0 &&
                           ((uintptr_t)src & 15) == 0;
      if (compact) {
        hipLaunchKernelGGL(unique_mask_flat_kernel, dim3(16, (unsigned)n), dim3(256), 0, st, src,
                           per_img, slots, mask);
      } else {
        unsigned gx = grid_for(per_img, 64);
        hipLaunchKernelGGL(unique_mask_kernel, dim3(gx, (unsigned)n), dim3(256), 0, st, src, h,
                           w * c, row_stride, slots, mask);
      }
      hipLaunchKernelGGL(vals_from_mask_kernel, dim3((n + 255) / 256), dim3(256), 0, st, mask, n);
      a.vals = mask + 8 * n;
      PoisTables pt{};
      if (!replay) {
        const int rc = pois_tables_for(st, &pt);
        if (rc != IDN_OK) return rc;
      }
      if (flat) {
        // one 154 KB-LDS workgroup per CU, looping over (image, part) units; ~8 units per
        // workgroup keeps the tail short
        const int cus = cu_count();
        const int64_t nq = a.elems / 16;
        const int parts = (int)std::max<int64_t>(
            1, std::min<int64_t>((8LL * cus + n - 1) / n, (nq + POIS_FLAT_WGT - 1) / POIS_FLAT_WGT));
        const int units = n * parts;
        hipLaunchKernelGGL(noise_poisson_flat_kernel, dim3((unsigned)std::min(units, cus)),
                           dim3(POIS_FLAT_WGT), 0, st, a, pt, parts);
      } else {
        hipLaunchKernelGGL(noise_poisson_kernel, dim3(grid_for(a.elems * n)), dim3(256), 0, st, a,
                           pt);
      }
      break;
    }
  }
  IDN_CHECK_LAUNCH("idn_noise_u8");
  return IDN_OK;
}
}  // namespace idn

extern "C" int idn_noise_u8(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n, int h,
                            int w, int c, int64_t row_stride, int kind, double p0, double p1,
                            uint64_t seed, uint64_t offset, const double* replay, void* workspace,
                            size_t ws_bytes, void* stream) {
  return idn::noise_u8_impl(src, out_u8, out_f64, n, h, w, c, row_stride, kind, p0, p1, seed,
                            offset, nullptr, nullptr, replay, workspace, ws_bytes, stream);
}

extern "C" int idn_noise_ids_u8(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n,
                                int h, int w, int c, int64_t row_stride, int kind, double p0,
                                double p1, uint64_t seed, const uint64_t* image_ids,
                                void* workspace, size_t ws_bytes, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(image_ids || n == 0, "idn_noise_ids_u8: null image_ids");
  return noise_u8_impl(src, out_u8, out_f64, n, h, w, c, row_stride, kind, p0, p1, seed, 0,
                       image_ids, nullptr, nullptr, workspace, ws_bytes, stream);
}

extern "C" int idn_noise_slots_u8(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n,
                                  int h, int w, int c, int64_t row_stride, int kind, double p0,
                                  double p1, uint64_t seed, const uint64_t* image_ids,
                                  const int64_t* slots, void* workspace, size_t ws_bytes,
                                  void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(image_ids || n == 0, "idn_noise_slots_u8: null image_ids");
  IDN_CHECK_ARG(slots || n == 0, "idn_noise_slots_u8: null slots");
  IDN_CHECK_ARG(row_stride == (int64_t)w * c, "idn_noise_slots_u8: slots need compact rows "
                "(row_stride %lld != w*c)", (long long)row_stride);
  return noise_u8_impl(src, out_u8, out_f64, n, h, w, c, row_stride, kind, p0, p1, seed, 0,
                       image_ids, slots, nullptr, workspace, ws_bytes, stream);
}

extern "C" int idn_noise_ycc_u8(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n,
                                int h, int w, int kind, double p0, double p1, uint64_t seed,
                                uint64_t offset, const uint64_t* image_ids, const double* replay,
                                uint64_t* ycc_keys, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(src && out_f64 && ycc_keys, "idn_noise_ycc_u8: null src / out_f64 / ycc_keys");
  IDN_CHECK_ARG(kind == IDN_NOISE_GAUSSIAN || kind == IDN_NOISE_SPECKLE,
                "idn_noise_ycc_u8: gaussian or speckle only (got %d)", kind);
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0, "idn_noise_ycc_u8: bad shape");
  IDN_CHECK_ARG(p1 >= 0.0, "idn_noise_ycc_u8: var must be >= 0");
  if (n == 0) return IDN_OK;
  const int64_t elems = (int64_t)h * w * 3;
  if (elems % 6 != 0 || ((uintptr_t)src & 1) || ((uintptr_t)out_f64 & 15) ||
      ((uintptr_t)out_u8 & 1) || n > 65535)
    return set_error(IDN_EUNSUPPORTED, "idn_noise_ycc_u8: needs an even pixel count per image, "
                     "2-byte aligned u8 and 16-byte aligned float64 buffers");
  hipStream_t st = as_stream(stream);
  NoiseArgs a{};
  a.src = src;
  a.out_u8 = out_u8;
  a.out_f64 = out_f64;
  a.replay = replay;
  a.n = n;
  a.h = h;
  a.w = w;
  a.c = 3;
  a.row_stride = (int64_t)w * 3;
  a.elems = elems;
  a.key = seed ^ (KIND_TAG * (uint64_t)(kind + 1));
  a.offset = offset;
  a.ids = image_ids;
  a.p0 = p0;
  a.p1 = pow(p1, 0.5);
  a.ycc = reinterpret_cast<unsigned long long*>(ycc_keys);
  hipLaunchKernelGGL(ycc_keys_init, dim3((6 * n + 255) / 256), dim3(256), 0, st, a.ycc, n);
  // about 2048 workgroups in all: one image alone spreads over the chip, a batch keeps the
  // per-workgroup atomics few
  const int64_t npp = elems / 6;
  const unsigned gx = (unsigned)std::max<int64_t>(
      1, std::min<int64_t>((npp + 255) / 256, (2048 + n - 1) / n));
  const dim3 grid(gx, (unsigned)n);
  const bool g = kind == IDN_NOISE_GAUSSIAN;
  if (replay && g)
    hipLaunchKernelGGL((noise_gauss_ycc_kernel<IDN_NOISE_GAUSSIAN, SRC_REPLAY>), grid, dim3(256), 0, st, a);
  else if (replay)
    hipLaunchKernelGGL((noise_gauss_ycc_kernel<IDN_NOISE_SPECKLE, SRC_REPLAY>), grid, dim3(256), 0, st, a);
  else if (g)
    hipLaunchKernelGGL((noise_gauss_ycc_kernel<IDN_NOISE_GAUSSIAN, SRC_F64>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((noise_gauss_ycc_kernel<IDN_NOISE_SPECKLE, SRC_F64>), grid, dim3(256), 0, st, a);
  IDN_CHECK_LAUNCH("idn_noise_ycc_u8");
  return IDN_OK;
}

extern "C" int idn_periodic_pattern_u8(uint8_t* pattern, int h, int w, int c, double amplitude,
                                       void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(pattern, "idn_periodic_pattern_u8: null pattern");
  IDN_CHECK_ARG(h > 0 && w > 0 && c > 0, "idn_periodic_pattern_u8: bad shape");
  const int64_t size = (int64_t)h * w * c;
  // numpy.linspace(-A, A, size): step = (A - (-A)) / (size - 1)
  const double step = size > 1 ? (amplitude - (-amplitude)) / (double)(size - 1) : 0.0;
  hipLaunchKernelGGL(periodic_kernel, dim3(grid_for(size)), dim3(256), 0, as_stream(stream),
                     pattern, size, amplitude, step);
  IDN_CHECK_LAUNCH("idn_periodic_pattern_u8");
  return IDN_OK;
}

namespace idn {
static int add_pattern_impl(const uint8_t* src, const uint8_t* pattern, uint8_t* dst, int n,
                            int h, int w, int c, int64_t row_stride, const int64_t* slots,
                            void* stream) {
  IDN_CHECK_ARG(src && pattern && dst, "idn_add_pattern_u8: null pointer");
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0 && c > 0, "idn_add_pattern_u8: bad shape");
  IDN_CHECK_ARG(row_stride >= (int64_t)w * c, "idn_add_pattern_u8: row_stride < w*c");
  if (n == 0) return IDN_OK;
  const int64_t per_img = (int64_t)h * w * c;
  if (row_stride == (int64_t)w * c && per_img % 16 == 0 && n <= 65535 &&
      (((uintptr_t)src | (uintptr_t)pattern | (uintptr_t)dst) & 15) == 0) {
    const int64_t nq = per_img / 16;
    const unsigned gx = (unsigned)std::min<int64_t>((nq + 255) / 256, 1024);
    hipLaunchKernelGGL(add_pattern_flat_kernel, dim3(gx, (unsigned)n), dim3(256), 0,
                       as_stream(stream), src, pattern, dst, per_img, slots);
  } else {
    hipLaunchKernelGGL(add_pattern_kernel, dim3(grid_for((int64_t)n * h * w * c)), dim3(256), 0,
                       as_stream(stream), src, pattern, dst, n, h, w * c, row_stride, slots);
  }
  IDN_CHECK_LAUNCH("idn_add_pattern_u8");
  return IDN_OK;
}

// dst image slots[i] = src image slots[i] (compact images, 16 bytes per thread where aligned)
__global__ __launch_bounds__(256) void copy_slots_kernel(const uint8_t* __restrict__ src,
                                                         uint8_t* __restrict__ dst,
                                                         int64_t per_img,
                                                         const int64_t* __restrict__ slots) {
  const int64_t base = slots[blockIdx.y] * per_img;
  if ((per_img & 15) == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const v4u* s = reinterpret_cast<const v4u*>(src + base);
    v4u* d = reinterpret_cast<v4u*>(dst + base);
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < per_img / 16;
         q += (int64_t)gridDim.x * blockDim.x)
      d[q] = s[q];
  } else {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < per_img;
         i += (int64_t)gridDim.x * blockDim.x)
      dst[base + i] = src[base + i];
  }
}
}  // namespace idn

extern "C" int idn_add_pattern_u8(const uint8_t* src, const uint8_t* pattern, uint8_t* dst, int n,
                                  int h, int w, int c, int64_t row_stride, void* stream) {
  return idn::add_pattern_impl(src, pattern, dst, n, h, w, c, row_stride, nullptr, stream);
}

extern "C" int idn_add_pattern_slots_u8(const uint8_t* src, const uint8_t* pattern, uint8_t* dst,
                                        int n, int h, int w, int c, const int64_t* slots,
                                        void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(slots || n == 0, "idn_add_pattern_slots_u8: null slots");
  return add_pattern_impl(src, pattern, dst, n, h, w, c, (int64_t)w * c, slots, stream);
}

extern "C" int idn_copy_slots_u8(const uint8_t* src, uint8_t* dst, int n, int64_t per_img,
                                 const int64_t* slots, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(src && dst && (slots || n == 0), "idn_copy_slots_u8: null pointer");
  IDN_CHECK_ARG(n >= 0 && n <= 65535 && per_img > 0, "idn_copy_slots_u8: bad shape");
  if (n == 0 || src == dst) return IDN_OK;
  const unsigned gx = (unsigned)std::min<int64_t>((per_img / 16 + 255) / 256, 1024);
  hipLaunchKernelGGL(copy_slots_kernel, dim3(gx < 1 ? 1 : gx, (unsigned)n), dim3(256), 0,
                     as_stream(stream), src, dst, per_img, slots);
  IDN_CHECK_LAUNCH("idn_copy_slots_u8");
  return IDN_OK;
}
