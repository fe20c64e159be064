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
// RNG: Philox4x32-10 keyed by (seed ^ kind tag); counter = (element pair / draw, image id).
// Image id = offset + image index, so a rank that owns images [a, b) of a batch draws exactly
// what a single GPU would for those images.
//
// Also: periodic noise pattern (add_periodic_noise, test.py:1128-1298) and cv2.add(u8, u8).
#include "idn_common.hpp"

#include <math.h>

#include <algorithm>

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
};
__device__ __forceinline__ uint64_t image_id(const NoiseArgs& a, int img) {
  return a.ids ? a.ids[img] : a.offset + (uint64_t)img;
}

__device__ __forceinline__ void store_out(const NoiseArgs& a, int img, int64_t e, int64_t boff,
                                          double out) {
  if (a.out_f64) a.out_f64[(int64_t)img * a.elems + e] = out;
  if (a.out_u8) a.out_u8[boff] = u8_of(out);
}

// one thread per element pair (2 normals per Philox block)
template <int KIND>
__global__ __launch_bounds__(256) void noise_gauss_kernel(NoiseArgs a) {
  const int64_t pairs = (a.elems + 1) / 2;
  const int64_t total = pairs * a.n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int img = (int)(t / pairs);
    const int64_t pr = t - (int64_t)img * pairs;
    double nz[2];
    if (a.replay) {
      const int64_t e0 = 2 * pr;
      nz[0] = a.replay[(int64_t)img * a.elems + e0];
      nz[1] = (e0 + 1 < a.elems) ? a.replay[(int64_t)img * a.elems + e0 + 1] : 0.0;
    } else {
      const uint64_t gimg = image_id(a, img);
      const u32x4 r = philox4x32(u32x4{(uint32_t)pr, (uint32_t)(pr >> 32), (uint32_t)gimg,
                                       (uint32_t)(gimg >> 32)},
                                 a.key);
      float z0, z1;
      normal2(r, z0, z1);
      nz[0] = __dadd_rn(a.p0, __dmul_rn(a.p1, (double)z0));
      nz[1] = __dadd_rn(a.p0, __dmul_rn(a.p1, (double)z1));
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int64_t e = 2 * pr + s;
      if (e >= a.elems) break;
      const int64_t pix = e / a.c;
      const int ch = (int)(e - pix * a.c);
      const int y = (int)(pix / a.w), x = (int)(pix - (int64_t)y * a.w);
      const int64_t boff = (int64_t)img * a.h * a.row_stride + (int64_t)y * a.row_stride +
                           (int64_t)x * a.c + ch;
      const double xv = img_as_float(a.src[boff]);
      double out;
      if (KIND == IDN_NOISE_GAUSSIAN) out = clip01(__dadd_rn(xv, nz[s]));
      else out = clip01(__dadd_rn(xv, __dmul_rn(xv, nz[s])));
      store_out(a, img, e, boff, out);
    }
  }
}

// ---- flat form (compact rows, Philox stream): 16 consecutive elements per thread -------------
// One 16-byte load / store per lane, image = blockIdx.y, no 64-bit index division.  Stream:
//   gaussian / speckle  counter (e/4, 0, image id) -> 4 u32 -> two Box-Muller pairs -> the 4
//                       normals of elements 4q..4q+3
//   s&p                 counter (e/2, 1, image id) -> (U1, U2) of elements 2q and 2q+1 as 32-bit
//                       uniforms compared against integer thresholds (|P - p| < 2^-32)
// The apply is the same float64 expression as the element kernels above.
__device__ __forceinline__ void normal4(const u32x4& r, float (&z)[4]) {
  normal2(r, z[0], z[1]);
  const u32x4 r2{r.z, r.w, 0u, 0u};
  normal2(r2, z[2], z[3]);
}

// MEAN0: mean == 0.0, so mean + sd*z is sd*z exactly up to the sign of a zero, which the
// following x + n / x + x*n (x >= 0) cannot see: one float64 add per element less
template <int KIND, bool MEAN0 = false>
__global__ __launch_bounds__(256) void noise_flat16_kernel(NoiseArgs a, uint32_t t_flip,
                                                           uint32_t t_salt) {
  const int img = blockIdx.y;
  const uint32_t chunk = blockIdx.x * 256u + threadIdx.x;
  const int64_t e0 = (int64_t)chunk * 16;
  if (e0 >= a.elems) return;
  const uint64_t gimg = image_id(a, img);
  const uint8_t* src = a.src + (int64_t)img * a.elems + e0;
  const v4u raw = *reinterpret_cast<const v4u*>(src);
  const uint32_t in[4] = {raw.x, raw.y, raw.z, raw.w};
  uint32_t o[4] = {0u, 0u, 0u, 0u};
  double* of = a.out_f64 ? a.out_f64 + (int64_t)img * a.elems + e0 : nullptr;
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // elements 4k .. 4k+3
    double outv[4];
    if constexpr (KIND == IDN_NOISE_SAP) {
#pragma unroll
      for (int hlf = 0; hlf < 2; ++hlf) {
        const uint32_t q = chunk * 8u + (uint32_t)(2 * k + hlf);
        const u32x4 r = philox4x32(u32x4{q, 1u, (uint32_t)gimg, (uint32_t)(gimg >> 32)}, a.key);
        const uint32_t u1[2] = {r.x, r.z}, u2[2] = {r.y, r.w};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int b = 2 * hlf + j;
          const double xv = img_as_float((in[k] >> (8 * b)) & 0xFFu);
          outv[b] = u1[j] < t_flip ? (u2[j] < t_salt ? 1.0 : 0.0) : xv;
        }
      }
    } else {
      const uint32_t q = chunk * 4u + (uint32_t)k;
      const u32x4 r = philox4x32(u32x4{q, 0u, (uint32_t)gimg, (uint32_t)(gimg >> 32)}, a.key);
      float z[4];
      normal4(r, z);
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const double sz = __dmul_rn(a.p1, (double)z[b]);
        const double nz = MEAN0 ? sz : __dadd_rn(a.p0, sz);
        const double xv = img_as_float((in[k] >> (8 * b)) & 0xFFu);
        if (KIND == IDN_NOISE_GAUSSIAN) outv[b] = clip01(__dadd_rn(xv, nz));
        else outv[b] = clip01(__dadd_rn(xv, __dmul_rn(xv, nz)));
      }
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      o[k] |= (uint32_t)u8_of(outv[b]) << (8 * b);
      if (of) of[4 * k + b] = outv[b];
    }
  }
  if (a.out_u8)
    *reinterpret_cast<v4u*>(a.out_u8 + (int64_t)img * a.elems + e0) = v4u{o[0], o[1], o[2], o[3]};
}

// salt & pepper: flipped = U1 < cdf0(amount), salted = U2 < cdf0(salt_vs_pepper)
__global__ __launch_bounds__(256) void noise_sap_kernel(NoiseArgs a) {
  const int64_t total = a.elems * a.n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int img = (int)(t / a.elems);
    const int64_t e = t - (int64_t)img * a.elems;
    double u1, u2;
    if (a.replay) {
      u1 = a.replay[t];
      u2 = a.replay[total + t];
    } else {
      const uint64_t gimg = image_id(a, img);
      const u32x4 r = philox4x32(
          u32x4{(uint32_t)e, (uint32_t)(e >> 32), (uint32_t)gimg, (uint32_t)(gimg >> 32)}, a.key);
      u1 = u01_closed_open(r.x, r.y);
      u2 = u01_closed_open(r.z, r.w);
    }
    const int64_t pix = e / a.c;
    const int ch = (int)(e - pix * a.c);
    const int y = (int)(pix / a.w), x = (int)(pix - (int64_t)y * a.w);
    const int64_t boff =
        (int64_t)img * a.h * a.row_stride + (int64_t)y * a.row_stride + (int64_t)x * a.c + ch;
    double out = img_as_float(a.src[boff]);
    if (u1 < a.p0) out = (u2 < a.p1) ? 1.0 : 0.0;
    store_out(a, img, e, boff, out);
  }
}

// per-image distinct-value mask (256 bits) -> vals = 2^ceil(log2(#distinct))
__global__ __launch_bounds__(256) void unique_mask_kernel(const uint8_t* __restrict__ src, int h,
                                                          int rowbytes, int64_t row_stride,
                                                          uint32_t* __restrict__ mask) {
  __shared__ uint32_t m[8];
  if (threadIdx.x < 8) m[threadIdx.x] = 0;
  __syncthreads();
  const int img = blockIdx.y;
  const uint8_t* s = src + (int64_t)img * h * row_stride;
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

// numpy legacy Poisson: multiplication method for lam < 10, PTRS (Hormann 1993) otherwise, with
// numpy's own loggam in the acceptance test
struct PhiloxStream {
  uint64_t key;
  uint32_t e_lo, e_hi, g_lo, g_hi;
  uint32_t blk = 0;
  u32x4 cur;
  int used = 2;
  __device__ __forceinline__ double next() {
    if (used == 2) {
      cur = philox4x32(u32x4{e_lo, e_hi ^ (blk << 20), g_lo, g_hi}, key);
      ++blk;
      used = 0;
    }
    const double u = (used == 0) ? u01_closed_open(cur.x, cur.y) : u01_closed_open(cur.z, cur.w);
    ++used;
    return u;
  }
};

// the per-lambda constants of numpy's samplers (lambda depends only on the u8 value and the
// image's vals: the flat kernel tabulates them once per workgroup)
struct PoisConst {
  double lam, enlam, slam, loglam, b, a, invalpha, vr, loginvalpha;
};
__device__ __forceinline__ PoisConst pois_const(double lam) {
  PoisConst p{};
  p.lam = lam;
  if (lam < 10.0) {
    p.enlam = exp(-lam);
  } else {
    p.slam = sqrt(lam);
    p.loglam = log(lam);
    p.b = 0.931 + 2.53 * p.slam;
    p.a = -0.059 + 0.02483 * p.b;
    p.invalpha = 1.1239 + 1.1328 / (p.b - 3.4);
    p.vr = 0.9277 - 3.6224 / (p.b - 2);
    p.loginvalpha = log(p.invalpha);
  }
  return p;
}

// numpy's legacy random_loggam (log Gamma(x), Stirling series with the recursion below 7): the
// function numpy's PTRS acceptance test evaluates at k + 1
__device__ double np_loggam(double x) {
  constexpr double a[10] = {8.333333333333333e-02, -2.777777777777778e-03, 7.936507936507937e-04,
                            -5.952380952380952e-04, 8.417508417508418e-04, -1.917526917526918e-03,
                            6.410256410256410e-03, -2.955065359477124e-02, 1.796443723688307e-01,
                            -1.39243221690590e+00};
  if (x == 1.0 || x == 2.0) return 0.0;
  const int n = x < 7.0 ? (int)(7 - x) : 0;
  double x0 = x + n;
  const double x2 = (1.0 / x0) * (1.0 / x0);
  double gl0 = a[9];
#pragma unroll
  for (int k = 8; k >= 0; --k) {
    gl0 *= x2;
    gl0 += a[k];
  }
  double gl = gl0 / x0 + 0.5 * 1.8378770664093453e+00 + (x0 - 0.5) * log(x0) - x0;
  for (int k = 1; k <= n; ++k) {
    gl -= log(x0 - 1.0);
    x0 -= 1.0;
  }
  return gl;
}

constexpr int LOGGAM_TAB = 1024;  // loggam(k + 1) for k < 1024 (a workgroup table in LDS)

__device__ double poisson_sample(const PoisConst& p, PhiloxStream& rs,
                                 const double* loggam_tab = nullptr) {
  const double lam = p.lam;
  if (lam == 0.0) return 0.0;
  if (lam < 10.0) {
    double prod = 1.0;
    int x = 0;
    for (int it = 0; it < 1000; ++it) {
      prod *= rs.next();
      if (prod > p.enlam) ++x;
      else return (double)x;
    }
    return (double)x;
  }
  for (int it = 0; it < 1000; ++it) {
    const double U = rs.next() - 0.5;
    const double V = rs.next();
    const double us = 0.5 - fabs(U);
    const double k = floor((2 * p.a / us + p.b) * U + lam + 0.43);
    if (us >= 0.07 && V <= p.vr) return k;
    if (k < 0 || (us < 0.013 && V > us)) continue;
    const double lg = (loggam_tab && k < LOGGAM_TAB) ? loggam_tab[(int)k] : np_loggam(k + 1);
    if (log(V) + p.loginvalpha - log(p.a / (us * us) + p.b) <= -lam + k * p.loglam - lg)
      return k;
  }
  return floor(lam);  // unreachable in practice (bounded loop)
}

__global__ __launch_bounds__(256) void noise_poisson_kernel(NoiseArgs a) {
  const int64_t total = a.elems * a.n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int img = (int)(t / a.elems);
    const int64_t e = t - (int64_t)img * a.elems;
    const int64_t pix = e / a.c;
    const int ch = (int)(e - pix * a.c);
    const int y = (int)(pix / a.w), x = (int)(pix - (int64_t)y * a.w);
    const int64_t boff =
        (int64_t)img * a.h * a.row_stride + (int64_t)y * a.row_stride + (int64_t)x * a.c + ch;
    const double vals = (double)a.vals[img];
    double k;
    if (a.replay) {
      k = a.replay[t];
    } else {
      const uint64_t gimg = image_id(a, img);
      PhiloxStream rs{a.key, (uint32_t)e, (uint32_t)(e >> 32), (uint32_t)gimg,
                      (uint32_t)(gimg >> 32)};
      k = poisson_sample(pois_const(__dmul_rn(img_as_float(a.src[boff]), vals)), rs);
    }
    store_out(a, img, e, boff, clip01(k / vals));
  }
}

// flat Poisson (compact rows, Philox stream): 16 consecutive elements per thread, image =
// blockIdx.y, the 256 per-value lambda constants tabulated in LDS; same streams and arithmetic
// as noise_poisson_kernel, so the two forms agree bit for bit
__global__ __launch_bounds__(256) void noise_poisson_flat_kernel(NoiseArgs a) {
  __shared__ PoisConst tab[256];
  __shared__ double lgt[LOGGAM_TAB];
  const int img = blockIdx.y;
  const double vals = (double)a.vals[img];
  tab[threadIdx.x] = pois_const(__dmul_rn(img_as_float(threadIdx.x), vals));
  for (int k = threadIdx.x; k < LOGGAM_TAB; k += 256) lgt[k] = np_loggam((double)k + 1.0);
  __syncthreads();
  const uint32_t chunk = blockIdx.x * 256u + threadIdx.x;
  const int64_t e0 = (int64_t)chunk * 16;
  if (e0 >= a.elems) return;
  const uint64_t gimg = image_id(a, img);
  const v4u raw = *reinterpret_cast<const v4u*>(a.src + (int64_t)img * a.elems + e0);
  const uint32_t in[4] = {raw.x, raw.y, raw.z, raw.w};
  double* of = a.out_f64 ? a.out_f64 + (int64_t)img * a.elems + e0 : nullptr;
  uint32_t* o8 = a.out_u8 ? reinterpret_cast<uint32_t*>(a.out_u8 + (int64_t)img * a.elems + e0) : nullptr;
  // Each lane walks its 16 elements with its own rejection state: one loop iteration is one
  // attempt (PTRS) or one factor (multiplication method) of the lane's current element, and a
  // lane moves on as soon as its element is accepted -- the wave never waits for the unluckiest
  // lane of every element (the element kernel's max over 64 geometric attempt counts).
  // Per element the draws and arithmetic are exactly poisson_sample's.
  auto byte_of = [&](int j) -> uint32_t {
    const uint32_t dw = (j >> 2) == 0 ? in[0] : (j >> 2) == 1 ? in[1] : (j >> 2) == 2 ? in[2] : in[3];
    return (dw >> (8 * (j & 3))) & 0xFFu;
  };
  int j = 0, it = 0, x = 0;
  double prod = 1.0;
  PoisConst pc = tab[byte_of(0)];
  PhiloxStream rs{a.key, (uint32_t)e0, (uint32_t)(e0 >> 32), (uint32_t)gimg, (uint32_t)(gimg >> 32)};
  uint32_t o = 0u;
  while (j < 16) {
    bool done = false;
    double k = 0.0;
    if (pc.lam == 0.0) {
      done = true;
    } else if (pc.lam < 10.0) {
      prod *= rs.next();
      if (prod > pc.enlam) {
        ++x;
        if (++it >= 1000) done = true;
      } else {
        done = true;
      }
      k = (double)x;
    } else {
      const double U = rs.next() - 0.5;
      const double V = rs.next();
      const double us = 0.5 - fabs(U);
      k = floor((2 * pc.a / us + pc.b) * U + pc.lam + 0.43);
      if (us >= 0.07 && V <= pc.vr) {
        done = true;
      } else if (!(k < 0 || (us < 0.013 && V > us))) {
        const double lg = k < LOGGAM_TAB ? lgt[(int)k] : np_loggam(k + 1);
        done = log(V) + pc.loginvalpha - log(pc.a / (us * us) + pc.b) <= -pc.lam + k * pc.loglam - lg;
      }
      if (!done && ++it >= 1000) {
        done = true;
        k = floor(pc.lam);
      }
    }
    if (done) {
      const double out = clip01(k / vals);
      o |= (uint32_t)u8_of(out) << (8 * (j & 3));
      if (of) of[j] = out;
      if ((j & 3) == 3) {
        if (o8) o8[j >> 2] = o;
        o = 0u;
      }
      ++j;
      if (j < 16) {
        const int64_t e = e0 + j;
        pc = tab[byte_of(j)];
        rs = PhiloxStream{a.key, (uint32_t)e, (uint32_t)(e >> 32), (uint32_t)gimg,
                          (uint32_t)(gimg >> 32)};
        it = 0;
        x = 0;
        prod = 1.0;
      }
    }
  }
}

// flat per-image distinct-value mask: 16 bytes per thread per step, a private 256-bit mask per
// thread, OR-reduced over the wave before one LDS atomic per word
__global__ __launch_bounds__(256) void unique_mask_flat_kernel(const uint8_t* __restrict__ src,
                                                               int64_t per_img,
                                                               uint32_t* __restrict__ mask) {
  __shared__ uint32_t m[8];
  if (threadIdx.x < 8) m[threadIdx.x] = 0;
  __syncthreads();
  const int img = blockIdx.y;
  const v4u* s = reinterpret_cast<const v4u*>(src + (int64_t)img * per_img);
  const int64_t nq = per_img / 16;
  uint32_t mk[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq;
       q += (int64_t)gridDim.x * blockDim.x) {
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
                                                               int64_t per_img) {
  const int img = blockIdx.y;
  const int64_t nq = per_img / 16;
  const v4u* s = reinterpret_cast<const v4u*>(src + (int64_t)img * per_img);
  const v4u* p = reinterpret_cast<const v4u*>(pat);
  v4u* d = reinterpret_cast<v4u*>(dst + (int64_t)img * per_img);
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
                                                          int rowbytes, int64_t row_stride) {
  const int64_t per_img = (int64_t)h * rowbytes;
  const int64_t total = per_img * n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int img = (int)(i / per_img);
    const int64_t e = i - (int64_t)img * per_img;
    const int y = (int)(e / rowbytes);
    const int64_t off = (int64_t)img * h * row_stride + (int64_t)y * row_stride + (e - (int64_t)y * rowbytes);
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

extern "C" size_t idn_noise_workspace_size(int kind, int n) {
  if (kind != IDN_NOISE_POISSON || n <= 0) return 0;
  return (size_t)n * 9 * sizeof(uint32_t);
}

namespace idn {
static int noise_u8_impl(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n, int h, int w,
                         int c, int64_t row_stride, int kind, double p0, double p1, uint64_t seed,
                         uint64_t offset, const uint64_t* ids, const double* replay,
                         void* workspace, size_t ws_bytes, void* stream) {
  IDN_CHECK_ARG(src, "idn_noise_u8: null src");
  IDN_CHECK_ARG(out_u8 || out_f64, "idn_noise_u8: at least one of out_u8 / out_f64 is required");
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0 && c >= 1 && c <= 4, "idn_noise_u8: bad shape");
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
  // flat form: Philox stream, compact rows, 16-element chunks that never straddle images
  const bool flat = !replay && row_stride == (int64_t)w * c && a.elems % 16 == 0 &&
                    ((uintptr_t)src & 15) == 0 && ((uintptr_t)out_u8 & 15) == 0 &&
                    ((uintptr_t)out_f64 & 7) == 0 && a.elems / 16 < ((int64_t)1 << 31) &&
                    env_int("IDN_NOISE_FLAT", 1) != 0;
  switch (kind) {
    case IDN_NOISE_GAUSSIAN:
    case IDN_NOISE_SPECKLE: {
      IDN_CHECK_ARG(p1 >= 0.0, "idn_noise_u8: var must be >= 0");
      a.p0 = p0;             // mean
      a.p1 = pow(p1, 0.5);   // var ** 0.5 (random_noise)
      const int64_t work = (a.elems + 1) / 2 * n;
      if (flat) {
        const dim3 grid((unsigned)((a.elems / 16 + 255) / 256), (unsigned)n);
        const bool m0 = a.p0 == 0.0;
        if (kind == IDN_NOISE_GAUSSIAN && m0)
          hipLaunchKernelGGL((noise_flat16_kernel<IDN_NOISE_GAUSSIAN, true>), grid, dim3(256), 0, st, a, 0u, 0u);
        else if (kind == IDN_NOISE_GAUSSIAN)
          hipLaunchKernelGGL(noise_flat16_kernel<IDN_NOISE_GAUSSIAN>, grid, dim3(256), 0, st, a, 0u, 0u);
        else if (m0)
          hipLaunchKernelGGL((noise_flat16_kernel<IDN_NOISE_SPECKLE, true>), grid, dim3(256), 0, st, a, 0u, 0u);
        else
          hipLaunchKernelGGL(noise_flat16_kernel<IDN_NOISE_SPECKLE>, grid, dim3(256), 0, st, a, 0u, 0u);
      } else if (kind == IDN_NOISE_GAUSSIAN)
        hipLaunchKernelGGL(noise_gauss_kernel<IDN_NOISE_GAUSSIAN>, dim3(grid_for(work)), dim3(256), 0, st, a);
      else
        hipLaunchKernelGGL(noise_gauss_kernel<IDN_NOISE_SPECKLE>, dim3(grid_for(work)), dim3(256), 0, st, a);
      break;
    }
    case IDN_NOISE_SAP: {
      IDN_CHECK_ARG(p0 >= 0.0 && p0 <= 1.0 && p1 >= 0.0 && p1 <= 1.0,
                    "idn_noise_u8: amount / salt_vs_pepper must be in [0, 1]");
      // np.random.choice([True, False], p=[p, 1-p]): True iff random_sample < cdf[0]
      a.p0 = p0 / (p0 + (1.0 - p0));
      a.p1 = p1 / (p1 + (1.0 - p1));
      if (flat) {
        // 32-bit uniform thresholds: P(u < t / 2^32) within 2^-32 of cdf0
        auto thr = [](double pp) -> uint32_t {
          const double t = ceil(pp * 4294967296.0);
          return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
        };
        const dim3 grid((unsigned)((a.elems / 16 + 255) / 256), (unsigned)n);
        hipLaunchKernelGGL(noise_flat16_kernel<IDN_NOISE_SAP>, grid, dim3(256), 0, st, a,
                           thr(a.p0), thr(a.p1));
      } else {
        hipLaunchKernelGGL(noise_sap_kernel, dim3(grid_for(a.elems * n)), dim3(256), 0, st, a);
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
                           per_img, mask);
      } else {
        unsigned gx = grid_for(per_img, 64);
        hipLaunchKernelGGL(unique_mask_kernel, dim3(gx, (unsigned)n), dim3(256), 0, st, src, h,
                           w * c, row_stride, mask);
      }
      hipLaunchKernelGGL(vals_from_mask_kernel, dim3((n + 255) / 256), dim3(256), 0, st, mask, n);
      a.vals = mask + 8 * n;
      if (flat) {
        const dim3 grid((unsigned)((a.elems / 16 + 255) / 256), (unsigned)n);
        hipLaunchKernelGGL(noise_poisson_flat_kernel, grid, dim3(256), 0, st, a);
      } else {
        hipLaunchKernelGGL(noise_poisson_kernel, dim3(grid_for(a.elems * n)), dim3(256), 0, st, a);
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
                            offset, nullptr, replay, workspace, ws_bytes, stream);
}

extern "C" int idn_noise_ids_u8(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n,
                                int h, int w, int c, int64_t row_stride, int kind, double p0,
                                double p1, uint64_t seed, const uint64_t* image_ids,
                                void* workspace, size_t ws_bytes, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(image_ids || n == 0, "idn_noise_ids_u8: null image_ids");
  return noise_u8_impl(src, out_u8, out_f64, n, h, w, c, row_stride, kind, p0, p1, seed, 0,
                       image_ids, nullptr, workspace, ws_bytes, stream);
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

extern "C" int idn_add_pattern_u8(const uint8_t* src, const uint8_t* pattern, uint8_t* dst, int n,
                                  int h, int w, int c, int64_t row_stride, void* stream) {
  using namespace idn;
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
                       as_stream(stream), src, pattern, dst, per_img);
  } else {
    hipLaunchKernelGGL(add_pattern_kernel, dim3(grid_for((int64_t)n * h * w * c)), dim3(256), 0,
                       as_stream(stream), src, pattern, dst, n, h, w * c, row_stride);
  }
  IDN_CHECK_LAUNCH("idn_add_pattern_u8");
  return IDN_OK;
}
