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
// RNG: Philox4x32 keyed by (seed ^ kind tag); counter = (element group / draw, image id)
// (the flat Gaussian / speckle stream: Philox4x32-7 and 16-bit uniforms, noise_apply.hpp).
// Image id = offset + image index, so a rank that owns images [a, b) of a batch draws exactly
// what a single GPU would for those images.
//
// Also: periodic noise pattern (add_periodic_noise, test.py:1128-1298) and cv2.add(u8, u8).
#include "idn_common.hpp"
#include "noise_apply.hpp"

#include <math.h>

#include <algorithm>

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

// ---- flat form (compact rows, Philox stream): 16 consecutive elements per thread -------------
// One 16-byte load / store per lane, image = blockIdx.y, no 64-bit index division; the stream and
// the float64 apply are noise16_u8 (noise_apply.hpp), shared with the fused noise -> filter
// kernel (stencil_u8.hip), so the fused and two-step results are identical.
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
// of 256 values per power-of-two vals (vals <= 256), so the CDF of every
// (vals, v) pair is tabulated once per call (POIS_KMAX entries; P(X >= 512) < 1e-25 at
// lambda = 256) with a 1024-entry guide table.  A draw is one 53-bit uniform; the guide entries
// of its quantile interval bracket the answer (usually to one or two candidates) and a bisection
// of the bracket finishes it.  The same law as numpy's multiplication / PTRS samplers (the replay
// mode takes numpy's own draws), without their rejection loops.
constexpr int POIS_NV = 9;       // vals = 1, 2, 4, ..., 256
constexpr int POIS_KMAX = 512;   // CDF entries per lambda
constexpr int POIS_G = 1024;     // guide entries per lambda
struct PoisTables {
  double* cdf;      // [POIS_NV][256][POIS_KMAX]
  uint32_t* guide;  // [POIS_NV][256][POIS_G]: g(j) | g(j + 1) << 16, g(j) = smallest k with
                    // cdf[k] > j / POIS_G (g(POIS_G) = POIS_KMAX - 1): one load per bracket
};
// one thread per (vals, v): the CDF by the recurrence p(k+1) = p(k) * lambda / (k+1)
__global__ __launch_bounds__(64) void pois_cdf_kernel(PoisTables t) {
  const int id = blockIdx.x * 64 + threadIdx.x;  // vi * 256 + v
  if (id >= POIS_NV * 256) return;
  const int vi = id >> 8, v = id & 255;
  const double lam = __dmul_rn(img_as_float((uint32_t)v), (double)(1u << vi));
  double* cdf = t.cdf + (size_t)id * POIS_KMAX;
  double p = exp(-lam), acc = 0.0;
  for (int k = 0; k < POIS_KMAX; ++k) {
    acc += p;
    cdf[k] = k == POIS_KMAX - 1 ? 1.0 : fmin(acc, 1.0);
    p = p * lam / (double)(k + 1);
  }
}
// one thread per guide entry: g(j) and g(j + 1) by bisection of the CDF row
__device__ __forceinline__ int pois_first_above(const double* cdf, double q) {
  int lo = 0, hi = POIS_KMAX - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cdf[mid] > q) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}
__global__ __launch_bounds__(256) void pois_guide_kernel(PoisTables t) {
  const int id = blockIdx.x * 256 + threadIdx.x;  // (vi * 256 + v) * POIS_G + j
  if (id >= POIS_NV * 256 * POIS_G) return;
  const int row = id / POIS_G, j = id % POIS_G;
  const double* cdf = t.cdf + (size_t)row * POIS_KMAX;
  const uint32_t g0 = (uint32_t)pois_first_above(cdf, (double)j / POIS_G);
  const uint32_t g1 =
      j + 1 < POIS_G ? (uint32_t)pois_first_above(cdf, (double)(j + 1) / POIS_G) : POIS_KMAX - 1;
  t.guide[id] = g0 | (g1 << 16);
}

// element e's uniform: 4 consecutive elements share one Philox block (counter (e/4, tag, image
// id)), element e takes word e % 4 as u = (word + 1/2) / 2^32 in (0, 1).  The 2^-32 grid changes
// the law only on events of probability below 2^-32 (as the float Box-Muller of the Gaussian
// kind does), and the top 10 bits of the word are the guide index directly.
__device__ __forceinline__ double pois_u(uint32_t w) {
  return fma((double)w, 0x1p-32, 0x1p-33);  // exact: 33 significant bits
}
__device__ __forceinline__ u32x4 pois_block(uint64_t key, uint64_t q, uint64_t gimg) {
  return philox4x32(u32x4{(uint32_t)q, (uint32_t)(q >> 32) ^ 0x80000000u, (uint32_t)gimg,
                          (uint32_t)(gimg >> 32)}, key);
}
__device__ __forceinline__ int vals_index(uint32_t vals) { return __ffs((int)vals) - 1; }

// NE elements of one thread (row = vals index * 256 + u8 value, 32-bit offsets off the uniform
// table bases): bracket from the guide (all reads issued together), then bisection rounds in
// lockstep, each round issuing the probes of every unfinished element at once
template <int NE>
__device__ __forceinline__ void pois_invert_n(const PoisTables& pt, const uint32_t (&row)[NE],
                                              const uint32_t (&w)[NE], int (&lo)[NE]) {
  static_assert(POIS_G == 1024, "guide index = top 10 bits of the uniform word");
  int hi[NE];
  double u[NE];
#pragma unroll
  for (int jj = 0; jj < NE; ++jj) {
    u[jj] = pois_u(w[jj]);
    const uint32_t g = pt.guide[row[jj] * POIS_G + (w[jj] >> 22)];
    lo[jj] = (int)(g & 0xFFFFu);
    hi[jj] = (int)(g >> 16);
  }
  for (int round = 0; round < 10; ++round) {  // brackets are < 512 wide: at most 9 rounds
    double c[NE];
#pragma unroll
    for (int jj = 0; jj < NE; ++jj)
      c[jj] = lo[jj] < hi[jj] ? pt.cdf[row[jj] * POIS_KMAX + (uint32_t)((lo[jj] + hi[jj]) >> 1)]
                              : 0.0;
    bool open = false;
#pragma unroll
    for (int jj = 0; jj < NE; ++jj) {
      if (lo[jj] < hi[jj]) {
        const int mid = (lo[jj] + hi[jj]) >> 1;
        if (c[jj] <= u[jj]) lo[jj] = mid + 1;
        else hi[jj] = mid;
        open |= lo[jj] < hi[jj];
      }
    }
    if (!__any(open)) break;
  }
}

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
      const uint32_t u[1] = {q == 0 ? r.x : q == 1 ? r.y : q == 2 ? r.z : r.w};
      const uint32_t row[1] = {(uint32_t)vals_index(a.vals[img]) * 256u + a.src[boff]};
      int lo[1];
      pois_invert_n<1>(pt, row, u, lo);
      k = (double)lo[0];
    }
    store_out(a, img, e, boff, clip01(k / vals));
  }
}

// flat Poisson (compact rows, Philox stream): 16 consecutive elements per thread, image =
// blockIdx.y; the same uniforms and tables as noise_poisson_kernel, so the two forms agree bit
// for bit
__global__ __launch_bounds__(256) void noise_poisson_flat_kernel(NoiseArgs a, PoisTables pt) {
  const int img = blockIdx.y;
  const uint32_t chunk = blockIdx.x * 256u + threadIdx.x;
  const int64_t e0 = (int64_t)chunk * 16;
  if (__all(e0 >= a.elems)) return;
  const bool live = e0 < a.elems;  // dead lanes still take part in the lockstep rounds
  const uint32_t vraw = a.vals[img];
  const double vals = (double)vraw;
  const uint64_t gimg = image_id(a, img);
  v4u raw = {0u, 0u, 0u, 0u};
  const int64_t base = slot_of(a, img) * a.elems + e0;
  if (live) raw = *reinterpret_cast<const v4u*>(a.src + base);
  const uint32_t in[4] = {raw.x, raw.y, raw.z, raw.w};
  const uint32_t tab0 = (uint32_t)vals_index(vraw) * 256u;
  const double inv_vals = 1.0 / vals;  // vals is a power of two: k * inv_vals == k / vals
  double* of = a.out_f64 && live ? a.out_f64 + base : nullptr;
  uint32_t o[4] = {0u, 0u, 0u, 0u};
  // PQ groups of 16 / PQ elements (fewer live registers than 16 at once, so more waves per SIMD
  // to hide the table reads)
  constexpr int PQ = 4, PE = 16 / PQ;
#pragma unroll
  for (int hf = 0; hf < PQ; ++hf) {
    static_assert(PE == 4, "one Philox block per group");
    const u32x4 r = pois_block(a.key, (uint64_t)(e0 >> 2) + hf, gimg);
    const uint32_t u[PE] = {r.x, r.y, r.z, r.w};
    uint32_t row[PE];
#pragma unroll
    for (int jj = 0; jj < PE; ++jj) {
      const int el = PE * hf + jj;
      row[jj] = tab0 + ((in[el >> 2] >> (8 * (el & 3))) & 0xFFu);
    }
    int lo[PE];
    pois_invert_n<PE>(pt, row, u, lo);
#pragma unroll
    for (int jj = 0; jj < PE; ++jj) {
      const int el = PE * hf + jj;
      const double out = clip01(__dmul_rn((double)lo[jj], inv_vals));
      o[el >> 2] |= (uint32_t)u8_of(out) << (8 * (el & 3));
      if (of) of[el] = out;
    }
  }
  if (!live) return;
  if (a.out_u8)
    *reinterpret_cast<v4u*>(a.out_u8 + base) = v4u{o[0], o[1], o[2], o[3]};
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
  return pois_tables_off(n) + (size_t)idn::POIS_NV * 256 *
                                  (idn::POIS_KMAX * sizeof(double) + idn::POIS_G * sizeof(uint32_t));
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
        const dim3 grid((unsigned)((a.elems / 16 + 255) / 256), (unsigned)n);
        hipLaunchKernelGGL(noise_flat16_kernel<IDN_NOISE_SAP>, grid, dim3(256), 0, st, a,
                           sap_threshold(a.p0), sap_threshold(a.p1));
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
                           per_img, slots, mask);
      } else {
        unsigned gx = grid_for(per_img, 64);
        hipLaunchKernelGGL(unique_mask_kernel, dim3(gx, (unsigned)n), dim3(256), 0, st, src, h,
                           w * c, row_stride, slots, mask);
      }
      hipLaunchKernelGGL(vals_from_mask_kernel, dim3((n + 255) / 256), dim3(256), 0, st, mask, n);
      a.vals = mask + 8 * n;
      PoisTables pt;
      pt.cdf = reinterpret_cast<double*>((char*)workspace + pois_tables_off(n));
      pt.guide = reinterpret_cast<uint32_t*>(pt.cdf + (size_t)POIS_NV * 256 * POIS_KMAX);
      if (!replay) {
        hipLaunchKernelGGL(pois_cdf_kernel, dim3(POIS_NV * 256 / 64), dim3(64), 0, st, pt);
        hipLaunchKernelGGL(pois_guide_kernel, dim3(POIS_NV * 256 * POIS_G / 256), dim3(256), 0, st,
                           pt);
      }
      if (flat) {
        const dim3 grid((unsigned)((a.elems / 16 + 255) / 256), (unsigned)n);
        hipLaunchKernelGGL(noise_poisson_flat_kernel, grid, dim3(256), 0, st, a, pt);
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
