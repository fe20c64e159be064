// The reference's own additive noise closures (not skimage): SURVEY §8f row 1.
//   uniform   lib/model/test.py:767-903   x = img_as_float(img); out = cv2.add(x, U(0, high))
//   gamma     lib/model/test.py:1300-1437 out = cv2.add(x, scipy gamma.rvs(1.99, scale=s))
//   rayleigh  lib/model/test.py:1439-1572 out = cv2.add(x, scipy rayleigh.rvs(scale=s))
//   brownian  lib/model/test.py:905-1126  B = concat([0], cumsum(sqrt(dt) * N(0,1)[n-1]))
//                                          out = cv2.add(img, (B * 255).astype(uint8))
// cv2.add on two float64 arrays is a plain add (no clamp), and the caller's
// (255 * out).astype(np.uint8) wraps modulo 256, so out_u8 = U8(255 * out) with the C-cast rule
// (uint8)(int32)trunc(y), |y| >= 2^31 -> 0.  Brownian adds two u8 images with saturation.
//
// Draws: replay mode takes numpy's own unit draws (random_sample / standard_gamma /
// sqrt(chisquare(2)) / standard_normal); Philox mode draws them from counter streams keyed by
// (seed ^ kind tag, image id), so a batch split or a rank count never changes an image's noise.
// Brownian's cumulative sum runs as a three-pass scan (per-block sums, per-image block offsets,
// per-element prefix), fp64 throughout; its summation order differs from np.cumsum's strictly
// sequential one by rounding only.
#include "idn_common.hpp"

#include <math.h>

#include <algorithm>

namespace idn {

constexpr uint64_t ADD_TAG = 0xD1B54A32D192ED03ull;

struct AddArgs {
  const uint8_t* src;
  uint8_t* out_u8;
  double* out_f64;
  const double* replay;
  double* blk;  // brownian: per-image block sums / offsets (workspace)
  int n, h, w, c;
  int64_t row_stride;
  int64_t elems;
  double p0, p1;
  uint64_t key, offset;
  const uint64_t* ids;  // optional per-image ids (device); else id = offset + image index
  int nblk;  // brownian blocks per image
};
__device__ __forceinline__ uint64_t image_id(const AddArgs& a, int img) {
  return a.ids ? a.ids[img] : a.offset + (uint64_t)img;
}

__device__ __forceinline__ double img_as_float_(uint32_t v) { return __dmul_rn((double)v, 1.0 / 255.0); }

// (y).astype(np.uint8) for float64 y: (uint8)(int32)trunc(y); out of int32 range or NaN -> 0
__device__ __forceinline__ uint32_t u8_wrap(double y) {
  if (!(__builtin_fabs(y) < 2147483648.0)) return 0u;
  return (uint32_t)(int)y & 0xFFu;
}

__device__ __forceinline__ int64_t elem_offset(const AddArgs& a, int img, int64_t e) {
  const int64_t pix = e / a.c;
  const int ch = (int)(e - pix * a.c);
  const int y = (int)(pix / a.w), x = (int)(pix - (int64_t)y * a.w);
  return (int64_t)img * a.h * a.row_stride + (int64_t)y * a.row_stride + (int64_t)x * a.c + ch;
}

// ---- unit draws from the Philox stream ----------------------------------------------------------
__device__ __forceinline__ float box_muller0(uint32_t a, uint32_t b) {
  const float u1 = ((float)(a >> 8) + 1.0f) * (1.0f / 16777216.0f);
  const float u2 = (float)(b >> 8) * (1.0f / 16777216.0f);
  return __builtin_sqrtf(-2.0f * 0.6931471805599453f * __builtin_amdgcn_logf(u1)) *
         __builtin_amdgcn_cosf(u2);
}
// u in (0, 1] with full relative precision near 0 (for the log of the exponential tails)
__device__ __forceinline__ float u01_tail(uint32_t r) { return ((float)r + 0.5f) * 2.3283064365386963e-10f; }

// standard gamma(a) by Marsaglia-Tsang (a >= 1; a < 1 via G(a+1) * U^(1/a)), one Philox block per
// attempt: counter (e, attempt, image)
__device__ float std_gamma(double a_d, uint64_t key, uint32_t e_lo, uint32_t e_hi, uint64_t gimg) {
  float a = (float)a_d;
  float boost = 1.0f;
  uint32_t att = 0;
  if (a < 1.0f) {
    const u32x4 r = philox4x32(u32x4{e_lo, (e_hi << 8) | 0xFFu, (uint32_t)gimg, (uint32_t)(gimg >> 32)}, key);
    boost = __builtin_expf(__builtin_logf(u01_tail(r.x)) / a);
    a += 1.0f;
  }
  const float d = a - 1.0f / 3.0f, cc = 1.0f / __builtin_sqrtf(9.0f * d);
  for (; att < 64; ++att) {
    const u32x4 r = philox4x32(u32x4{e_lo, (e_hi << 8) | att, (uint32_t)gimg, (uint32_t)(gimg >> 32)}, key);
    const float z = box_muller0(r.x, r.y);
    float v = 1.0f + cc * z;
    if (v <= 0.0f) continue;
    v = v * v * v;
    const float u = u01_tail(r.z);
    if (__builtin_logf(u) < 0.5f * z * z + d - d * v + d * __builtin_logf(v)) return d * v * boost;
  }
  return d * boost;  // not reached in practice (acceptance ~98% per attempt at a = 1.99)
}

template <int KIND>
__device__ __forceinline__ double unit_draw(const AddArgs& a, int img, int64_t e, int64_t flat) {
  if (a.replay) return a.replay[flat];
  const uint64_t gimg = image_id(a, img);
  if constexpr (KIND == IDN_NOISE_GAMMA) {
    return (double)std_gamma(a.p0, a.key, (uint32_t)e, (uint32_t)(e >> 32), gimg);
  } else {
    const u32x4 r = philox4x32(u32x4{(uint32_t)e, (uint32_t)(e >> 32), (uint32_t)gimg,
                                     (uint32_t)(gimg >> 32)}, a.key);
    if constexpr (KIND == IDN_NOISE_UNIFORM) {
      const uint64_t v = ((uint64_t)(r.x >> 5) << 26) | (r.y >> 6);  // random_sample: 53 bits
      return (double)v * (1.0 / 9007199254740992.0);
    } else {  // RAYLEIGH unit draw: sqrt(chisquare(2)) = sqrt(-2 ln U)
      return (double)__builtin_sqrtf(-2.0f * __builtin_logf(u01_tail(r.x)));
    }
  }
}

// noise value from the unit draw: scipy rvs computes vals * scale + loc (loc = 0);
// np.random.uniform(0, high) computes low + (high - low) * random_sample()
template <int KIND>
__device__ __forceinline__ double noise_of(const AddArgs& a, double u) {
  if constexpr (KIND == IDN_NOISE_UNIFORM) return __dadd_rn(0.0, __dmul_rn(a.p0, u));
  else if constexpr (KIND == IDN_NOISE_GAMMA) return __dadd_rn(__dmul_rn(u, a.p1), 0.0);
  else return __dadd_rn(__dmul_rn(u, a.p0), 0.0);
}

// one element per thread (any stride, replay or Philox)
template <int KIND>
__global__ __launch_bounds__(256) void noise_add_kernel(AddArgs a) {
  const int img = blockIdx.y;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < a.elems;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t flat = (int64_t)img * a.elems + e;
    const double u = unit_draw<KIND>(a, img, e, flat);
    const int64_t boff = elem_offset(a, img, e);
    const double out = __dadd_rn(img_as_float_(a.src[boff]), noise_of<KIND>(a, u));
    if (a.out_f64) a.out_f64[flat] = out;
    if (a.out_u8) a.out_u8[boff] = (uint8_t)u8_wrap(__dmul_rn(255.0, out));
  }
}

// ---- brownian ---------------------------------------------------------------------------------
// increment of element e (e >= 1): sqrt(dt) * z_{e-1}; element 0 contributes 0 (B_0 = 0)
constexpr int BR_THREADS = 256, BR_PER_THREAD = 16, BR_BLOCK = BR_THREADS * BR_PER_THREAD;

__device__ __forceinline__ void brownian_incs(const AddArgs& a, int img, int64_t e0, double sdt,
                                              double (&inc)[BR_PER_THREAD]) {
  const uint64_t gimg = image_id(a, img);
#pragma unroll
  for (int q = 0; q < BR_PER_THREAD / 4; ++q) {
    float z[4] = {0.f, 0.f, 0.f, 0.f};
    if (!a.replay) {
      const uint64_t c = (uint64_t)(e0 / 4 + q);
      const u32x4 r = philox4x32(u32x4{(uint32_t)c, (uint32_t)(c >> 32), (uint32_t)gimg,
                                       (uint32_t)(gimg >> 32)}, a.key);
      const float u1a = ((float)(r.x >> 8) + 1.0f) * (1.0f / 16777216.0f);
      const float u2a = (float)(r.y >> 8) * (1.0f / 16777216.0f);
      const float ra = __builtin_sqrtf(-2.0f * 0.6931471805599453f * __builtin_amdgcn_logf(u1a));
      const float u1b = ((float)(r.z >> 8) + 1.0f) * (1.0f / 16777216.0f);
      const float u2b = (float)(r.w >> 8) * (1.0f / 16777216.0f);
      const float rb = __builtin_sqrtf(-2.0f * 0.6931471805599453f * __builtin_amdgcn_logf(u1b));
      z[0] = ra * __builtin_amdgcn_cosf(u2a);
      z[1] = ra * __builtin_amdgcn_sinf(u2a);
      z[2] = rb * __builtin_amdgcn_cosf(u2b);
      z[3] = rb * __builtin_amdgcn_sinf(u2b);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t e = e0 + 4 * q + j;
      double v = 0.0;
      if (e >= 1 && e < a.elems) {
        const double zz = a.replay ? a.replay[(int64_t)img * a.elems + e] : (double)z[j];
        v = __dmul_rn(sdt, zz);
      }
      inc[4 * q + j] = v;
    }
  }
}

// exclusive prefix over the block's 256 values (Hillis-Steele in LDS, fp64); total = block sum
__device__ __forceinline__ double block_exclusive_scan(double v, double* lds, double& total) {
  const int t = threadIdx.x;
  lds[t] = v;
  __syncthreads();
  for (int off = 1; off < BR_THREADS; off <<= 1) {
    const double add = t >= off ? lds[t - off] : 0.0;
    __syncthreads();
    lds[t] = __dadd_rn(lds[t], add);
    __syncthreads();
  }
  total = lds[BR_THREADS - 1];
  const double excl = t > 0 ? lds[t - 1] : 0.0;
  __syncthreads();
  return excl;
}

__global__ __launch_bounds__(BR_THREADS) void brownian_sums_kernel(AddArgs a, double sdt) {
  __shared__ double lds[BR_THREADS];
  const int img = blockIdx.y;
  const int64_t e0 = (int64_t)blockIdx.x * BR_BLOCK + (int64_t)threadIdx.x * BR_PER_THREAD;
  double inc[BR_PER_THREAD];
  brownian_incs(a, img, e0, sdt, inc);
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < BR_PER_THREAD; ++i) s = __dadd_rn(s, inc[i]);
  double total;
  block_exclusive_scan(s, lds, total);
  if (threadIdx.x == 0) a.blk[(int64_t)img * a.nblk + blockIdx.x] = total;
}

// per image: exclusive scan of its block sums, in place (one 256-thread block per image)
__global__ __launch_bounds__(BR_THREADS) void brownian_offsets_kernel(AddArgs a) {
  __shared__ double lds[BR_THREADS];
  const int img = blockIdx.x;
  double* b = a.blk + (int64_t)img * a.nblk;
  const int per = (a.nblk + BR_THREADS - 1) / BR_THREADS;
  const int lo = threadIdx.x * per, hi = min(lo + per, a.nblk);
  double s = 0.0;
  for (int i = lo; i < hi; ++i) s = __dadd_rn(s, b[i]);
  double total;
  const double base = block_exclusive_scan(s, lds, total);
  double run = base;
  for (int i = lo; i < hi; ++i) {
    const double v = b[i];
    b[i] = run;
    run = __dadd_rn(run, v);
  }
}

__global__ __launch_bounds__(BR_THREADS) void brownian_apply_kernel(AddArgs a, double sdt) {
  __shared__ double lds[BR_THREADS];
  const int img = blockIdx.y;
  const int64_t e0 = (int64_t)blockIdx.x * BR_BLOCK + (int64_t)threadIdx.x * BR_PER_THREAD;
  double inc[BR_PER_THREAD];
  brownian_incs(a, img, e0, sdt, inc);
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < BR_PER_THREAD; ++i) s = __dadd_rn(s, inc[i]);
  double total;
  const double excl = block_exclusive_scan(s, lds, total);
  double B = __dadd_rn(a.blk[(int64_t)img * a.nblk + blockIdx.x], excl);
#pragma unroll
  for (int i = 0; i < BR_PER_THREAD; ++i) {
    const int64_t e = e0 + i;
    B = __dadd_rn(B, inc[i]);
    if (e < a.elems) {
      const int64_t boff = elem_offset(a, img, e);
      const uint32_t noise = u8_wrap(__dmul_rn(B, 255.0));
      const uint32_t sum = (uint32_t)a.src[boff] + noise;
      if (a.out_u8) a.out_u8[boff] = (uint8_t)(sum > 255u ? 255u : sum);
      if (a.out_f64) a.out_f64[(int64_t)img * a.elems + e] = B;  // the walk itself (debug/parity)
    }
  }
}

}  // namespace idn

extern "C" size_t idn_noise_add_workspace_size(int kind, int n, int h, int w, int c) {
  using namespace idn;
  if (kind != IDN_NOISE_BROWNIAN || n <= 0 || h <= 0 || w <= 0 || c <= 0) return 0;
  const int64_t elems = (int64_t)h * w * c;
  const int64_t nblk = (elems + BR_BLOCK - 1) / BR_BLOCK;
  return (size_t)(nblk * n) * sizeof(double);
}

namespace idn {
static int noise_add_impl(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n, int h,
                          int w, int c, int64_t row_stride, int kind, double p0, double p1,
                          uint64_t seed, uint64_t offset, const uint64_t* ids,
                          const double* replay, void* workspace, size_t ws_bytes, void* stream) {
  IDN_CHECK_ARG(src, "idn_noise_add_u8: null src");
  IDN_CHECK_ARG(out_u8 || out_f64, "idn_noise_add_u8: at least one of out_u8 / out_f64 is required");
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0 && c >= 1 && c <= 4, "idn_noise_add_u8: bad shape");
  IDN_CHECK_ARG(n <= 65535, "idn_noise_add_u8: at most 65535 images per call");
  IDN_CHECK_ARG(row_stride >= (int64_t)w * c, "idn_noise_add_u8: row_stride < w*c");
  IDN_CHECK_ARG(kind >= IDN_NOISE_UNIFORM && kind <= IDN_NOISE_BROWNIAN,
                "idn_noise_add_u8: unknown kind %d", kind);
  if (n == 0) return IDN_OK;
  hipStream_t st = as_stream(stream);
  AddArgs a;
  a.src = src;
  a.out_u8 = out_u8;
  a.out_f64 = out_f64;
  a.replay = replay;
  a.blk = nullptr;
  a.n = n;
  a.h = h;
  a.w = w;
  a.c = c;
  a.row_stride = row_stride;
  a.elems = (int64_t)h * w * c;
  a.p0 = p0;
  a.p1 = p1;
  a.key = seed ^ (ADD_TAG * (uint64_t)(kind + 1));
  a.offset = offset;
  a.ids = ids;
  a.nblk = 0;
  const unsigned gx = (unsigned)std::min<int64_t>((a.elems + 255) / 256, 65535);
  switch (kind) {
    case IDN_NOISE_UNIFORM:
      IDN_CHECK_ARG(p0 >= 0.0, "idn_noise_add_u8: uniform high must be >= 0");
      hipLaunchKernelGGL(noise_add_kernel<IDN_NOISE_UNIFORM>, dim3(gx, (unsigned)n), dim3(256), 0, st, a);
      break;
    case IDN_NOISE_GAMMA:
      IDN_CHECK_ARG(p0 > 0.0 && p1 >= 0.0, "idn_noise_add_u8: gamma shape must be > 0, scale >= 0");
      hipLaunchKernelGGL(noise_add_kernel<IDN_NOISE_GAMMA>, dim3(gx, (unsigned)n), dim3(256), 0, st, a);
      break;
    case IDN_NOISE_RAYLEIGH:
      IDN_CHECK_ARG(p0 >= 0.0, "idn_noise_add_u8: rayleigh scale must be >= 0");
      hipLaunchKernelGGL(noise_add_kernel<IDN_NOISE_RAYLEIGH>, dim3(gx, (unsigned)n), dim3(256), 0, st, a);
      break;
    default: {  // BROWNIAN
      IDN_CHECK_ARG(p0 >= 0.0, "idn_noise_add_u8: brownian dt must be >= 0");
      const size_t need = idn_noise_add_workspace_size(kind, n, h, w, c);
      IDN_CHECK_ARG(workspace && ws_bytes >= need,
                    "idn_noise_add_u8: brownian needs %zu workspace bytes (got %zu)", need, ws_bytes);
      a.blk = (double*)workspace;
      a.nblk = (int)((a.elems + BR_BLOCK - 1) / BR_BLOCK);
      const double sdt = sqrt(p0);  // np.sqrt(dt)
      hipLaunchKernelGGL(brownian_sums_kernel, dim3((unsigned)a.nblk, (unsigned)n), dim3(BR_THREADS), 0, st, a, sdt);
      hipLaunchKernelGGL(brownian_offsets_kernel, dim3((unsigned)n), dim3(BR_THREADS), 0, st, a);
      hipLaunchKernelGGL(brownian_apply_kernel, dim3((unsigned)a.nblk, (unsigned)n), dim3(BR_THREADS), 0, st, a, sdt);
      break;
    }
  }
  IDN_CHECK_LAUNCH("idn_noise_add_u8");
  return IDN_OK;
}
}  // namespace idn

extern "C" int idn_noise_add_u8(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n, int h,
                                int w, int c, int64_t row_stride, int kind, double p0, double p1,
                                uint64_t seed, uint64_t offset, const double* replay,
                                void* workspace, size_t ws_bytes, void* stream) {
  return idn::noise_add_impl(src, out_u8, out_f64, n, h, w, c, row_stride, kind, p0, p1, seed,
                             offset, nullptr, replay, workspace, ws_bytes, stream);
}

extern "C" int idn_noise_add_ids_u8(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n,
                                    int h, int w, int c, int64_t row_stride, int kind, double p0,
                                    double p1, uint64_t seed, const uint64_t* image_ids,
                                    void* workspace, size_t ws_bytes, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(image_ids || n == 0, "idn_noise_add_ids_u8: null image_ids");
  return noise_add_impl(src, out_u8, out_f64, n, h, w, c, row_stride, kind, p0, p1, seed, 0,
                        image_ids, nullptr, workspace, ws_bytes, stream);
}
