// Haar L = 3 on u8 images (BASELINE config 5's denoiser: skimage 0.14.2 denoise_wavelet(db1,
// wavelet_levels=3), lib/roi_data_layer/minibatch_before_curvelet.py:85-87), round 6: two reads of
// the image and one write.  Included by wavelet.hip inside namespace idn, after the shared helpers
// (stats layout, haar_int / ycc_w, the exact dd key, select_bin / radix_pass).
//
//   wl_h3_window  reads 1/8 of the level-1 rows of every image: per channel a histogram of the
//                 finest |T| (T = w_c . D_dd, the exact integer that the finest dd is a multiple
//                 of) and a window [lo, hi] of |T| that holds the median rank with a wide margin
//   wl_h3_stats   reads the image once: the exact fp64 YCbCr min / max (integer keys per lane,
//                 the fp64 chain only on the pixels holding a workgroup's extreme key), the integer
//                 second moments of every detail band (the BayesShrink sums), the count of nonzero
//                 finest T, the count below the window, the |T| inside the window (appended), and
//                 the positions where T = 0 but the reference's fp64 dd may be a rounding residue
//   wl_h3_sigma   per image and channel: the residues evaluated exactly (the nonzero count), the
//                 median rank selected among the window's |T| (sigma), the sums and thresholds;
//                 an image whose rank falls outside its window, or is a residue, takes an exact
//                 full-image selection in the same workgroup
//   wl_h3_synth   reads the image again: the three levels' coefficients from the integer
//                 combinations, soft thresholds, synthesis, clip, de-normalisation, YCbCr -> RGB
//                 and the U8 store, in fp32 (packed where two 2x2 groups run side by side)
//
// Sigma: the reference's finest dd is 0.5 T / (255000 range) within 2e-12 / range (the error
// analysis at wl_haar_stats), and distinct |T| differ by >= 1.96e-6 / range, so the ranks of the
// fp64 values are the ranks of |T| and T = 0 ranks below every T != 0.  The median is taken as
// 0.5 |T_k| / (255000 range) in fp64: relative 1e-6 / |T_k| from the reference's value (a few
// 1e-12 at the usual |T_k| ~ 1e5..1e7), far inside the 1e-5 output tolerance.  The nonzero
// count stays exact: every T = 0 position that is not an equal-triple pair (exact 0, x - x) is
// evaluated with the reference's fp64 chain.

// wl_h3_stats / wl_h3_synth grid: a workgroup of WLH_WG threads = WLH_WG / 4 quads = the 8x8 blocks
// of H3_COLS consecutive block columns (a column strip), walking a chunk of block rows
constexpr int H3_COLS = WLH_WG / 4;
__host__ __device__ inline int h3_strips(int w) { return ((w >> 3) + H3_COLS - 1) / H3_COLS; }
constexpr int H3_SEL = 66;   // stats doubles [66, 78): per channel 8 u32 (H3Sel)
constexpr int H3_CST = 112;  // stats doubles [112, 154): per channel 28 floats (H3Const)
struct H3Sel {
  uint32_t lo, hi;  // window of |T| (wl_h3_window)
  uint32_t n_t;     // nonzero finest T (wl_h3_stats)
  uint32_t n_lo;    // |T| < lo, zeros included
  uint32_t n_c;     // |T| appended from the window
  uint32_t n_r;     // residue positions appended (channel 0's slot counts for the image)
  uint32_t fb;      // diagnostics: 1 = full-image fallback taken (wl_h3_sigma)
  uint32_t pad;
};
struct H3Const {  // fp32 synthesis constants of one channel (wl_h3_consts)
  float w1[3], w2[3], w3[3];  // rgb2ycbcr row x 1000 x the level's coefficient scale
  float t1[3], t2[3], t3[3];  // soft thresholds in the same (folded) units
  float ka;                   // level-3 approximation offset
  float rng, mo;              // de-normalisation: v * rng + mo (mo = min - YCbCr offset)
  float mr[3], br[3];         // this channel's column of the output map (H3Rgb): 255 R[k][c] rng,
  float pad;                  // and its part of the offsets, 255 R[k][c] mo
};
static_assert(sizeof(H3Const) == 28 * sizeof(float), "28 floats per channel");
struct H3Rgb {     // out_k = sum_c m[k][c] v_c + b[k], v_c the clipped [0, 1] synthesis output of
  float m[3][3];  // channel c: skimage's ycbcr2rgb rows x 255 x range_c; the de-normalisation
  float b[3];     // offsets in b (minus 0.5: the U8 cast rounds to nearest, see wl_h3_synth)
};
__host__ __device__ inline H3Sel* h3_sel(double* st) { return reinterpret_cast<H3Sel*>(st + H3_SEL); }
__host__ __device__ inline const H3Const* h3_cst(const double* st) {
  return reinterpret_cast<const H3Const*>(st + H3_CST);
}

// skimage ycbcr2rgb (the inverse of rgb2ycbcr's matrix, per unit of Y - 16, Cb - 128, Cr - 128)
__host__ __device__ constexpr double h3_r(int k, int c) {
  constexpr double R[3][3] = {{0.004566210045662101, 1.1808799897950177e-09, 0.006258928969943937},
                              {0.004566210045662101, -0.0015363236860449021, -0.003188110949655707},
                              {0.004566210045662101, 0.007910716233554741, 1.1977497040511743e-08}};
  return R[k][c];
}
// The synthesis constants from the stats block (min / max, half thresholds thrh, flag).  With
// s1 = 0.5 / (255000 range) and k = 2 (offset - min) / range (wl_haar_synth_int), and the idwt's
// factors 1/2 folded into the coefficients (a power of two commutes with soft()):
//   level 1 detail  soft(T s1 / 2, thrh(0))          -> w1 = w s1 / 2,  t1 = thrh(0)
//   level 2 detail  soft(T s1 / 8, thrh(1) / 2)      -> w2 = w s1 / 8,  t2 = thrh(1) / 2
//   level 3         (w . S64) s1 / 32 + k / 2 +- soft(T s1 / 32, thrh(2) / 4)
// so each level's approximation enters the next butterfly unscaled.
__device__ void h3_consts(double* st, int c) {
  wreal mn, mx;
  wl_minmax64(st, c, mn, mx);
  const double inv = mx - mn, s1 = 0.5 / (255000.0 * inv);
  const double k = 2.0 * ((c == 0 ? 16.0 : 128.0) - mn) / inv;
  H3Const* q = const_cast<H3Const*>(h3_cst(st)) + c;
  for (int j = 0; j < 3; ++j) {
    const double wj = (double)ycc_w(c, j);
    q->w1[j] = (float)(wj * s1 * 0.5);
    q->w2[j] = (float)(wj * s1 * 0.125);
    q->w3[j] = (float)(wj * s1 * 0.03125);
    q->t1[j] = (float)st[WlStats::thrh(c, 0, j)];
    q->t2[j] = (float)(0.5 * st[WlStats::thrh(c, 1, j)]);
    q->t3[j] = (float)(0.25 * st[WlStats::thrh(c, 2, j)]);
  }
  q->ka = (float)(0.5 * k);
  q->rng = (float)inv;
  q->mo = (float)(mn - (c == 0 ? 16.0 : 128.0));
  for (int j = 0; j < 3; ++j) {
    q->mr[j] = (float)(255.0 * h3_r(j, c) * inv);
    q->br[j] = (float)(255.0 * h3_r(j, c) * (mn - (c == 0 ? 16.0 : 128.0)));
  }
}
__device__ __forceinline__ float uniform_f32(float v) {  // a wave-uniform float into an SGPR
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
// out_k = 255 sum_c R[k][c] (v_c rng_c + mo_c) - 0.5 from the three channels' columns (H3Const)
__device__ __forceinline__ H3Rgb h3_rgb(const H3Const* K) {
  H3Rgb o;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
#pragma unroll
    for (int c = 0; c < 3; ++c) o.m[k][c] = K[c].mr[k];
    o.b[k] = uniform_f32(((K[0].br[k] - 0.5f) + K[1].br[k]) + K[2].br[k]);
  }
  return o;
}
__global__ void wl_h3_consts(double* __restrict__ stats, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 3 * n) h3_consts(stats + (size_t)(i / 3) * WL_STATS, i % 3);
}


// ---- wl_h3_synth ---------------------------------------------------------------------------------
typedef float h3f2 __attribute__((ext_vector_type(2)));
typedef short h3s2 __attribute__((ext_vector_type(2)));
// lane value of quad member k (DPP quad_perm broadcast, one VALU op)
__device__ __forceinline__ int quad_get(int v, int k) {
  switch (k) {
    case 0: return __builtin_amdgcn_mov_dpp(v, 0x00, 0xF, 0xF, false);
    case 1: return __builtin_amdgcn_mov_dpp(v, 0x55, 0xF, 0xF, false);
    case 2: return __builtin_amdgcn_mov_dpp(v, 0xAA, 0xF, 0xF, false);
    default: return __builtin_amdgcn_mov_dpp(v, 0xFF, 0xF, 0xF, false);
  }
}
__device__ __forceinline__ float soft_f(float x, float t) {
  return x - __builtin_amdgcn_fmed3f(x, -t, t);
}
__device__ __forceinline__ h3f2 soft_f2(h3f2 x, float t) {
  const h3f2 c = {__builtin_amdgcn_fmed3f(x.x, -t, t), __builtin_amdgcn_fmed3f(x.y, -t, t)};
  return x - c;
}
__device__ __forceinline__ h3f2 fma2(h3f2 a, h3f2 b, h3f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ h3f2 splat2(float v) { return h3f2{v, v}; }
// a + b and a - b clamped to [0, 1] by the packed add's clamp bit (LLVM clamps each half with a
// v_max_f32 instead: one instruction per value)
__device__ __forceinline__ h3f2 pk_add_clamp(h3f2 a, h3f2 b) {
  h3f2 r;
  asm("v_pk_add_f32 %0, %1, %2 clamp" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ h3f2 pk_sub_clamp(h3f2 a, h3f2 b) {
  h3f2 r;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1] clamp" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
#ifndef IDN_H3S_Q3  // 1: level 3 of the synthesis split across the quad's lanes (A/B; 207 against
#define IDN_H3S_Q3 0    // 187 us with each lane forming all: the DPP round trips lengthen the chain)
#endif
#ifndef IDN_H3S_PK  // level 1 of the synthesis's analysis on 16-bit integer pairs
#define IDN_H3S_PK 1
#endif
#ifndef IDN_H3S_CLAMP  // 1: the inner clip as the clamp bit of the packed adds (A/B: 0 = v_max clamp)
#define IDN_H3S_CLAMP 1
#endif

// One thread per 4x4 sub-block; the four sub-blocks of an 8x8 block are consecutive lanes (a
// quad), which exchange their level-2 approximation sums by DPP for level 3.  Level 1 runs on two
// 2x2 groups side by side as fp32 pairs (v_pk_fma / add / mul).  Outputs within the 1e-5
// tolerance of the fp64 form (fp32 throughout: the synthesis is continuous in its inputs and no
// exact zero depends on it).  GEN = false: u8 output only, dword-aligned rows (the product's
// case); true: any of u8 (byte stores) / f32 output.
#ifndef IDN_H3S_IT  // block rows per synthesis thread (A/B builds set it)
#define IDN_H3S_IT 2
#endif
constexpr int H3S_IT = IDN_H3S_IT;
__host__ __device__ inline int h3s_chunks(int h) { return ((h >> 3) + H3S_IT - 1) / H3S_IT; }
#ifndef IDN_H3S_WPE
#define IDN_H3S_WPE 1
#endif
#ifndef IDN_H3S_XCD  // XCD-contiguous workgroup order: neighbouring strips share their edge lines
#define IDN_H3S_XCD 1    // in one L2 (FETCH 536 -> 461 MB per 256 images, 187.9 -> 185.7 us)
#endif
template <bool GEN>
__global__ __launch_bounds__(WLH_WG) __attribute__((amdgpu_waves_per_eu(IDN_H3S_WPE))) void wl_h3_synth(const uint8_t* __restrict__ src, int h, int w,
                                                      int64_t row_stride,
                                                      const double* __restrict__ stats,
                                                      uint8_t* __restrict__ out_u8,
                                                      float* __restrict__ out_f32) {
  // grid: (column strips of 32 blocks x chunks of H3S_IT block rows, images); IDN_H3S_XCD: in
  // XCD-contiguous order, as wl_h3_stats
  const int lin0 = (int)(blockIdx.y * gridDim.x + blockIdx.x);
  const int lin = IDN_H3S_XCD ? xcd_contiguous_block(lin0, (int)(gridDim.x * gridDim.y)) : lin0;
  const int img = lin / (int)gridDim.x, wg = lin - img * (int)gridDim.x;
  const int nbx = w >> 3, nby = h >> 3, strips = h3_strips(w);
  const int strip = wg % strips, chunk = wg / strips;
  const int sub = threadIdx.x & 3, bx = strip * H3_COLS + (threadIdx.x >> 2);
  const int by0 = chunk * H3S_IT, nit = min(H3S_IT, nby - by0);
  const bool act = bx < nbx;  // uniform over each quad
  const double* st = stats + (size_t)img * WL_STATS;
  const H3Const* K = h3_cst(st);
  const int x0 = bx * 8 + (sub & 1) * 4;
  const int64_t img_off = (int64_t)img * h * row_stride;
  const uint8_t* ib = src + img_off + (int64_t)(8 * by0 + (sub >> 1) * 4) * row_stride + (int64_t)x0 * 3;
  auto load_q = [&](int it, uint32_t (&qq)[4][3]) {
    if (!act || it >= nit) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t* p = reinterpret_cast<const uint32_t*>(ib + (int64_t)it * 8 * row_stride + r * row_stride);
#pragma unroll
      for (int k = 0; k < 3; ++k) qq[r][k] = p[k];
    }
  };
  // IDN_H3S_Q3: this lane's level-3 signs over x01, x10, x11 (haar_int's bands ad, da, dd for
  // sub = 0, 1, 2; the approximation for 3), chain start (ka for the approximation) and threshold
  const float q3s[3] = {sub == 1 || sub == 3 ? 1.f : -1.f, sub == 0 || sub == 3 ? 1.f : -1.f,
                        sub >= 2 ? 1.f : -1.f};
  float q3b[3], q3t[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    q3b[c] = sub == 3 ? K[c].ka : 0.f;
    q3t[c] = sub == 3 ? 0.f : (sub == 0 ? K[c].t3[0] : sub == 1 ? K[c].t3[1] : K[c].t3[2]);
  }
  uint32_t qn[4][3] = {};
  load_q(0, qn);
#pragma unroll 1
  for (int it = 0; it < nit; ++it) {
  const int y0 = 8 * (by0 + it) + (sub >> 1) * 4;
  uint32_t q[4][3];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int k = 0; k < 3; ++k) q[r][k] = qn[r][k];
  load_q(it + 1, qn);
  // the bytes as floats (v_cvt_f32_ubyte): every combination below is an exact small integer
  auto pxf = [&](int r, int k) { return (float)((q[r][k >> 2] >> (8 * (k & 3))) & 0xFFu); };
  // level 1 on the group pairs (gx = 0, 1 of row pair gy) as fp32 pairs: S1[gy][rgb] sums,
  // D1[gy][band][rgb] details
  h3f2 S1[2][3], D1[2][3][3];
  if (IDN_H3S_PK) {
    // as wl_h3_stats: the two groups side by side in 16-bit lanes (v_perm of the row dwords,
    // v_pk_add / sub_u16: exact), then each 16-bit result to float
    auto pk = [&](int r, int k) {  // bytes k (gx 0) and k + 6 (gx 1) of row r
      const int k1 = k + 6;
      const uint32_t sel = (uint32_t)(k & 3) | 0x0C00u | ((uint32_t)(4 + (k1 & 3)) << 16) | 0x0C000000u;
      return __builtin_bit_cast(h3s2, __builtin_amdgcn_perm(q[r][k1 >> 2], q[r][k >> 2], sel));
    };
    auto f2 = [](h3s2 v) { return h3f2{(float)v.x, (float)v.y}; };
#pragma unroll
    for (int gy = 0; gy < 2; ++gy)
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        const h3s2 x00 = pk(2 * gy, ch), x01 = pk(2 * gy, 3 + ch), x10 = pk(2 * gy + 1, ch),
                   x11 = pk(2 * gy + 1, 3 + ch);
        const h3s2 lo0 = x00 + x10, lo1 = x01 + x11, hi0 = x00 - x10, hi1 = x01 - x11;
        S1[gy][ch] = f2(lo0 + lo1);
        D1[gy][0][ch] = f2(lo0 - lo1);
        D1[gy][1][ch] = f2(hi0 + hi1);
        D1[gy][2][ch] = f2(hi0 - hi1);
      }
  } else
#pragma unroll
  for (int gy = 0; gy < 2; ++gy)
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const h3f2 x00 = {pxf(2 * gy, ch), pxf(2 * gy, 6 + ch)}, x01 = {pxf(2 * gy, 3 + ch), pxf(2 * gy, 9 + ch)};
      const h3f2 x10 = {pxf(2 * gy + 1, ch), pxf(2 * gy + 1, 6 + ch)},
                 x11 = {pxf(2 * gy + 1, 3 + ch), pxf(2 * gy + 1, 9 + ch)};
      const h3f2 lo0 = x00 + x10, lo1 = x01 + x11, hi0 = x00 - x10, hi1 = x01 - x11;
      S1[gy][ch] = lo0 + lo1;
      D1[gy][0][ch] = lo0 - lo1;
      D1[gy][1][ch] = hi0 + hi1;
      D1[gy][2][ch] = hi0 - hi1;
    }
  // level 2 on the four groups' sums (g0 g1 / g2 g3 = S1[0].x .y / S1[1].x .y)
  float S16[3], fd2[3][3];
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const h3f2 lo = S1[0][ch] + S1[1][ch], hi = S1[0][ch] - S1[1][ch];
    S16[ch] = lo.x + lo.y;
    fd2[0][ch] = lo.x - lo.y;
    fd2[1][ch] = hi.x + hi.y;
    fd2[2][ch] = hi.x - hi.y;
  }
  // level 3 across the quad
  float f64s[3], fd3[3][3], y3[3];
  if (IDN_H3S_Q3) {
    // quad lane `sub` forms one of the quad's level-3 sums: band sub (< 3) or the approximation
    // (3), exact small integers in any order
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const int b16 = __float_as_int(S16[ch]);
      const float x00 = __int_as_float(quad_get(b16, 0)), x01 = __int_as_float(quad_get(b16, 1));
      const float x10 = __int_as_float(quad_get(b16, 2)), x11 = __int_as_float(quad_get(b16, 3));
      y3[ch] = __fmaf_rn(q3s[2], x11, __fmaf_rn(q3s[1], x10, __fmaf_rn(q3s[0], x01, x00)));
    }
  } else
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const int b16 = __float_as_int(S16[ch]);
    const float x00 = __int_as_float(quad_get(b16, 0)), x01 = __int_as_float(quad_get(b16, 1));
    const float x10 = __int_as_float(quad_get(b16, 2)), x11 = __int_as_float(quad_get(b16, 3));
    const float lo0 = x00 + x10, lo1 = x01 + x11, hi0 = x00 - x10, hi1 = x01 - x11;
    f64s[ch] = lo0 + lo1;
    fd3[0][ch] = lo0 - lo1;
    fd3[1][ch] = hi0 + hi1;
    fd3[2][ch] = hi0 - hi1;
  }
  if (!act) continue;
  if (st[WlStats::FLAG] != 0.0) {  // image-uniform: zeros (0.14.2's NaN -> U8 0)
#pragma unroll 1
    for (int r = 0; r < 4; ++r)
#pragma unroll 1
      for (int k = 0; k < 12; ++k) {
        const int y = y0 + r, xx = x0 + k / 3, c = k % 3;
        if (out_u8) out_u8[img_off + (int64_t)y * row_stride + (int64_t)xx * 3 + c] = 0;
        if (out_f32) out_f32[(((int64_t)img * h + y) * w + xx) * 3 + c] = 0.0f;
      }
    continue;
  }
  // lane signs of this sub-block's output in the level-3 butterfly (r = sub >> 1, s = sub & 1)
  const float sad = (sub & 1) ? -1.f : 1.f, sda = (sub & 2) ? -1.f : 1.f, sdd = sad * sda;
  // per channel: level 3 -> a2, level 2 -> the four groups' level-1 approximations
  float A1[3][4];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const H3Const& k = K[c];
    auto dotw = [&](const float (&wv)[3], const float (&d)[3]) {
      return __fmaf_rn(wv[2], d[2], __fmaf_rn(wv[1], d[1], wv[0] * d[0]));
    };
    float a2;
    if (IDN_H3S_Q3) {
      // this lane's term: the soft-thresholded band (threshold 0 leaves the approximation term,
      // whose chain starts at ka), then the quad's four terms in the chain's order
      const float tq = soft_f(__fmaf_rn(k.w3[2], y3[2], __fmaf_rn(k.w3[1], y3[1], __fmaf_rn(k.w3[0], y3[0], q3b[c]))), q3t[c]);
      const int ti = __float_as_int(tq);
      a2 = __int_as_float(quad_get(ti, 3));
      a2 = __fmaf_rn(sad, __int_as_float(quad_get(ti, 0)), a2);
      a2 = __fmaf_rn(sda, __int_as_float(quad_get(ti, 1)), a2);
      a2 = __fmaf_rn(sdd, __int_as_float(quad_get(ti, 2)), a2);
    } else {
      a2 = __fmaf_rn(k.w3[2], f64s[2], __fmaf_rn(k.w3[1], f64s[1], __fmaf_rn(k.w3[0], f64s[0], k.ka)));
      a2 = __fmaf_rn(sad, soft_f(dotw(k.w3, fd3[0]), k.t3[0]), a2);
      a2 = __fmaf_rn(sda, soft_f(dotw(k.w3, fd3[1]), k.t3[1]), a2);
      a2 = __fmaf_rn(sdd, soft_f(dotw(k.w3, fd3[2]), k.t3[2]), a2);
    }
    const float ad = soft_f(dotw(k.w2, fd2[0]), k.t2[0]);
    const float da = soft_f(dotw(k.w2, fd2[1]), k.t2[1]);
    const float dd = soft_f(dotw(k.w2, fd2[2]), k.t2[2]);
    const float p = a2 + ad, m = a2 - ad, q0 = da + dd, q1 = da - dd;
    A1[c][0] = p + q0;
    A1[c][1] = m + q1;
    A1[c][2] = p - q0;
    A1[c][3] = m - q1;
  }
  // level 1: groups (0, 1) and (2, 3) side by side -> pixel values v[pair][pixel (r, s)][c]
  const H3Rgb M = h3_rgb(K);
  const bool dw = !GEN;
#pragma unroll
  for (int gp = 0; gp < 2; ++gp) {  // pair gp: groups 2 gp (x of the pair) and 2 gp + 1 (y)
    h3f2 v[4][3];                    // [pixel (r, s)][c]: .x group 2 gp, .y group 2 gp + 1
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const H3Const& k = K[c];
      h3f2 d[3];
#pragma unroll
      for (int b = 0; b < 3; ++b)
        d[b] = soft_f2(fma2(splat2(k.w1[2]), D1[gp][b][2],
                            fma2(splat2(k.w1[1]), D1[gp][b][1], splat2(k.w1[0]) * D1[gp][b][0])), k.t1[b]);
      const h3f2 A = {A1[c][2 * gp], A1[c][2 * gp + 1]};
      const h3f2 p = A + d[0], m = A - d[0], q0 = d[1] + d[2], q1 = d[1] - d[2];
      if (IDN_H3S_CLAMP) {  // v already clipped to [0, 1]
        v[0][c] = pk_add_clamp(p, q0);
        v[1][c] = pk_add_clamp(m, q1);
        v[2][c] = pk_sub_clamp(p, q0);
        v[3][c] = pk_sub_clamp(m, q1);
      } else {
        v[0][c] = p + q0;
        v[1][c] = m + q1;
        v[2][c] = p - q0;
        v[3][c] = m - q1;
      }
    }
    // inner clip [0, 1]; de-normalisation, YCbCr -> RGB x 255 and the offsets in one affine map
    // (H3Rgb, its bias minus 0.5); the cast: round to nearest with saturation
    uint32_t rowp[2][3] = {{0u, 0u, 0u}, {0u, 0u, 0u}};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = i >> 1, s = i & 1;
      h3f2 vc[3];
#pragma unroll
      for (int c = 0; c < 3; ++c)
        vc[c] = IDN_H3S_CLAMP ? v[i][c]
                              : h3f2{__builtin_amdgcn_fmed3f(v[i][c].x, 0.f, 1.f), __builtin_amdgcn_fmed3f(v[i][c].y, 0.f, 1.f)};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const h3f2 o = fma2(vc[2], splat2(M.m[c][2]),
                            fma2(vc[1], splat2(M.m[c][1]), fma2(vc[0], splat2(M.m[c][0]), splat2(M.b[c]))));
#pragma unroll
        for (int g2 = 0; g2 < 2; ++g2) {  // group 2 gp + g2: pixel column 2 g2 + s
          const float of = g2 ? o.y : o.x;  // out - 0.5
          const int xx = x0 + 2 * g2 + s, y = y0 + 2 * gp + r;
          if (dw) {
            const int bi = (2 * g2 + s) * 3 + c;
            rowp[r][bi >> 2] = __builtin_amdgcn_cvt_pk_u8_f32(of, bi & 3, rowp[r][bi >> 2]);
          } else if (out_u8) {
            out_u8[img_off + (int64_t)y * row_stride + (int64_t)xx * 3 + c] =
                (uint8_t)(__builtin_amdgcn_cvt_pk_u8_f32(of, 0, 0u) & 0xFFu);
          }
          if (GEN && out_f32)
            out_f32[(((int64_t)img * h + y) * w + xx) * 3 + c] =
                __builtin_amdgcn_fmed3f(of + 0.5f, 0.f, 255.f) * (1.f / 255.f);
        }
      }
    }
    if (dw) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        uint32_t* p = reinterpret_cast<uint32_t*>(out_u8 + img_off + (int64_t)(y0 + 2 * gp + r) * row_stride +
                                                  (int64_t)x0 * 3);
#pragma unroll
        for (int j = 0; j < 3; ++j) p[j] = rowp[r][j];
      }
    }
  }
  }  // it
}

// ---- wl_h3_window ---------------------------------------------------------------------------------
// |T| histogram bins: floor(log2 |T|) and the next H3_MB bits (monotone in |T|; |T| < 2^31)
#ifndef IDN_H3_MB  // mantissa bits of the window histogram (finer bins: a narrower window)
#define IDN_H3_MB 6
#endif
constexpr int H3_MB = IDN_H3_MB;
constexpr uint32_t H3_MM = (1u << H3_MB) - 1u;
constexpr int H3_HB = 32 << H3_MB;
constexpr int H3_WIN_WG = 1024;
constexpr int H3_SAMPLE = 16;  // every 16th level-1 row (rows 2i, 2i + 1 of the image)
__device__ __forceinline__ int h3_bin(uint32_t a) {  // a >= 1
  const int e = 31 - __clz((int)a);
  const uint32_t m = e >= H3_MB ? (a >> (e - H3_MB)) & H3_MM : (a << (H3_MB - e)) & H3_MM;
  return (e << H3_MB) + (int)m;
}
// the largest |T| whose bin is <= b (bins below 2^H3_MB hold few integers: found by search)
__device__ uint32_t h3_bin_hi(int b) {
  const int n = b + 1, e = n >> H3_MB;
  if (e >= 31) return 0xFFFFFFFFu;
  if (e >= H3_MB) return ((uint32_t)((1 << H3_MB) + (n & (int)H3_MM)) << (e - H3_MB)) - 1u;
  uint32_t hi = 0;
  for (uint32_t a = 1; a < (1u << H3_MB); ++a)
    if (h3_bin(a) <= b) hi = a;
  return hi;
}
__device__ __forceinline__ uint32_t h3_bin_lo(int b) {  // the smallest |T| of bin b, 1 below 2^H3_MB
  const int e = b >> H3_MB;
  return e >= H3_MB ? (uint32_t)((1 << H3_MB) + (b & (int)H3_MM)) << (e - H3_MB) : 1u;
}
// equal RGB triples along the rows or the columns of a 2x2 group: the reference's dd is x - x = 0
__device__ __forceinline__ bool h3_eqtrip(uint32_t t00, uint32_t t01, uint32_t t10, uint32_t t11) {
  return (t00 == t01 && t10 == t11) || (t00 == t10 && t01 == t11);
}

// The sample: level-1 rows i = 0, 16, 32, .. (the finest dd of row i reads image rows 2i, 2i + 1),
// every column.  Per channel the window of |T| ranks [n (0.5 - rho / 2 - m), n (0.5 + m)] of the
// sample's n nonzero T, rho the sample's share of residue candidates (T = 0, not an equal-triple
// pair: each may or may not be a nonzero fp64 residue, so the median's rank among the T != 0 lies
// up to rho / 2 lower) and m = 4 sample standard errors of the median rank (2 / sqrt(n)) + 0.3 %.
// A rank outside the window costs wl_h3_sigma its exact full-image path, not correctness.
__global__ __launch_bounds__(H3_WIN_WG) void wl_h3_window(const uint8_t* __restrict__ src, int h,
                                                          int w, int64_t row_stride,
                                                          double* __restrict__ stats,
                                                          int force_fb = 0) {
  const int img = blockIdx.x;
  __shared__ uint32_t hist[3][H3_HB];
  __shared__ uint32_t nres[3];
  {  // this image's statistics block as wl_init_stats leaves it (no colour keys): min keys ~0,
     // max keys 0, the rest 0.0 -- the first kernel of the path, so no separate launch
    double* st = stats + (size_t)img * WL_STATS;
    for (int k = threadIdx.x; k < WL_STATS; k += H3_WIN_WG)
      reinterpret_cast<unsigned long long*>(st)[k] =
          k >= WlStats::MN64 && k < WlStats::MN64 + 3 ? ~0ull : 0ull;
  }
  for (int k = threadIdx.x; k < 3 * H3_HB; k += H3_WIN_WG) (&hist[0][0])[k] = 0u;
  if (threadIdx.x < 3) nres[threadIdx.x] = 0u;
  __syncthreads();
  const int H1 = h >> 1, npair = w >> 2;  // position pairs (4 pixels, 3 dwords) per row
  const int nrows = (H1 + H3_SAMPLE - 1) / H3_SAMPLE, items = nrows * npair;
  const uint8_t* ib = src + (int64_t)img * h * row_stride;
  for (int it = threadIdx.x; it < items; it += H3_WIN_WG) {
    const int i = (it / npair) * H3_SAMPLE, jp = it - (it / npair) * npair;
    uint32_t q[2][3];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const uint32_t* p = reinterpret_cast<const uint32_t*>(ib + (int64_t)(2 * i + r) * row_stride +
                                                            (int64_t)jp * 12);
#pragma unroll
      for (int k = 0; k < 3; ++k) q[r][k] = p[k];
    }
    auto px = [&](int r, int k) { return (int)((q[r][k >> 2] >> (8 * (k & 3))) & 0xFFu); };
    auto trip = [&](int r, int pix) {
      return (uint32_t)(px(r, 3 * pix) | (px(r, 3 * pix + 1) << 8) | (px(r, 3 * pix + 2) << 16));
    };
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      int D[3];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch)
        D[ch] = px(0, 6 * s + ch) - px(0, 6 * s + 3 + ch) - px(1, 6 * s + ch) + px(1, 6 * s + 3 + ch);
      const bool eq = h3_eqtrip(trip(0, 2 * s), trip(0, 2 * s + 1), trip(1, 2 * s), trip(1, 2 * s + 1));
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int T = __mul24(ycc_w(c, 0), D[0]) + __mul24(ycc_w(c, 1), D[1]) + __mul24(ycc_w(c, 2), D[2]);
        if (T != 0) atomicAdd(&hist[c][h3_bin((uint32_t)(T < 0 ? -T : T))], 1u);
        else if (!eq) atomicAdd(&nres[c], 1u);
      }
    }
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave >= 3) return;
  const int c = wave;
  constexpr int PER = H3_HB / 64;
  uint32_t own = 0;
  for (int b = 0; b < PER; ++b) own += hist[c][lane * PER + b];
  uint32_t inc = own;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)inc, o);
    if (lane >= o) inc += t;
  }
  const uint32_t n = (uint32_t)__shfl((int)inc, 63);
  auto find = [&](uint32_t rank) -> int {  // bin holding sample rank `rank` (< n)
    const uint32_t excl = inc - own;
    int bin = H3_HB - 1;
    if (own && rank >= excl && rank < inc) {
      uint32_t acc = excl;
      int b = lane * PER;
      for (; b < lane * PER + PER - 1; ++b) {
        if (acc + hist[c][b] > rank) break;
        acc += hist[c][b];
      }
      bin = b;
    }
    const unsigned long long m = __ballot(own && rank >= excl && rank < inc);
    return __shfl(bin, m ? __ffsll((long long)m) - 1 : 0);
  };
  uint32_t lo = 1u, hi = 0xFFFFFFFFu;
  if (n >= 512) {
    const double rho = fmin((double)nres[c] / (double)n, 1.0);
    const double m = 2.0 / sqrt((double)n) + 0.003;
    const double qlo = 0.5 - 0.5 * rho - m, qhi = 0.5 + m;
    const int64_t klo = (int64_t)floor(qlo * (double)n), khi = (int64_t)ceil(qhi * (double)n);
    const int blo = klo > 0 ? find((uint32_t)klo) : -1;
    const int bhi = khi < (int64_t)n - 1 ? find((uint32_t)khi) : -1;
    if (blo >= 0) lo = h3_bin_lo(blo);
    if (bhi >= 0) hi = h3_bin_hi(bhi);
  }
  if (force_fb) lo = hi = 0xFFFFFFFFu;  // tests: an empty window, every channel takes the exact path
  if (lane == 0) {
    H3Sel* s = h3_sel(stats + (size_t)img * WL_STATS) + c;
    s->lo = lo;
    s->hi = hi;
  }
}

// ---- wl_h3_stats ----------------------------------------------------------------------------------
#ifndef IDN_H3_IT  // A/B builds set these
#define IDN_H3_IT 16
#endif
#ifndef IDN_H3_K
#define IDN_H3_K 8
#endif
#ifndef IDN_H3_WPE  // waves per EU the statistics kernel is scheduled for (~158 VGPRs either way:
#define IDN_H3_WPE 3    // without the hint LLVM's schedule of the branch-free body ran 352 us, with 3 308.5)
#endif
#ifndef IDN_H3_MOM  // level-1 moments: 0 v_dot2 on group pairs, 1 24-bit multiply-adds
#define IDN_H3_MOM 0
#endif
#ifndef IDN_H3_BRW  // 1: below-window count from the borrow of |T| - lo (A/B: 308.8 against 308.5)
#define IDN_H3_BRW 0
#endif
#ifndef IDN_H3_ZC  // 1: zero |T| counted on the residue branch (the nonzero count derived; A/B:
#define IDN_H3_ZC 0    // 331 against 308.5 us)
#endif
#ifndef IDN_H3_L3Q  // 1: level-3 moments by band across the quad's lanes; 0: the first lane all
#define IDN_H3_L3Q 1    // (308.5 against 340 us)
#endif
#ifndef IDN_H3_UNR  // unroll of the block-row loop
#define IDN_H3_UNR 1
#endif
#ifndef IDN_H3_PROBE  // timing probes only (wrong results): bit 0 no proxies, 1 no T / counts /
#define IDN_H3_PROBE 0  // appends, 2 no level-1 moments, 3 no levels 2-3, 5 flush without its
#endif                  // global atomic, 6 no flush
constexpr int H3_IT = IDN_H3_IT;  // block rows per workgroup (int32 moments: <= 16 steps, 1.07e9)
// Appends go to per-lane LDS slots (no atomics, no barriers): slot j of lane t of channel c at
// [c][j][t]; a wave moves its lanes' slots to the image's arrays (one scan, one global atomic per
// array) once some lane could overflow in the next iteration (4 appends per lane and array).
constexpr int H3_K = IDN_H3_K;
constexpr int H3_KR = 4;  // residue slots per lane (overflow: a global atomic each)
// a wave's per-lane runs buf[j][t] (j < n, the lane's count) to dst[base + exclusive prefix]
__device__ __forceinline__ void h3_wave_flush(const uint32_t* buf, uint32_t n, uint32_t* dst,
                                              uint32_t* gcount) {
  const int lane = threadIdx.x & 63;
  uint32_t inc = n;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)inc, o);
    if (lane >= o) inc += t;
  }
  const uint32_t tot = (uint32_t)__shfl((int)inc, 63);
  if (tot == 0 || (IDN_H3_PROBE & 64)) return;
  uint32_t base = 0;
  if (lane == 63 && !(IDN_H3_PROBE & 32)) base = atomicAdd(gcount, tot);
  base = (uint32_t)__shfl((int)base, 63) + inc - n;
  for (uint32_t j = 0; j < n; ++j) dst[base + j] = buf[j * WLH_WG + threadIdx.x];
}
#ifndef IDN_H3_MIN3  // one v_min3 / v_max3 per pixel pair in the proxies (309 -> 298 us)
#define IDN_H3_MIN3 1
#endif
#ifndef IDN_H3_MICRO  // running extremes by v_min3 / v_max3, level 2 from the packed sums, the
#define IDN_H3_MICRO 1   // residue test's ballot straight from the compare
#endif
#ifndef IDN_H3_PK  // level 1 of the statistics on 16-bit pairs (the two groups side by side)
#define IDN_H3_PK 1
#endif
__device__ __forceinline__ float h3_min3(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float h3_max3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// rgb2ycbcr coefficients as floats: the fp32 proxy of a pixel's YCbCr dot x 255 (|error| < 0.03
// for bytes: three roundings at magnitude < 2^16 plus the coefficients' own, < 1e-3 each)
__device__ __forceinline__ float h3_ycf(int c, int k) {
  constexpr float W[3][3] = {{65.481f, 128.553f, 24.966f}, {-37.797f, -74.203f, 112.0f},
                             {112.0f, -93.786f, -18.214f}};
  return W[c][k];
}
constexpr float H3_PTOL = 0.0625f;
// the RGB cube corner (bits: r g b = 255) where channel c's YCbCr dot is lowest / highest
__device__ __forceinline__ int h3_corner(int c, bool hi) {
  constexpr int C[3][2] = {{0b000, 0b111}, {0b110, 0b001}, {0b011, 0b100}};
  return C[c][hi ? 1 : 0];
}
__device__ __forceinline__ float h3_corner_proxy(int k, int c) {  // as the loop's proxy (x 255)
  const float R = (k & 4) ? 255.f : 0.f, G = (k & 2) ? 255.f : 0.f, B = (k & 1) ? 255.f : 0.f;
  return __fmaf_rn(h3_ycf(c, 2), B, __fmaf_rn(h3_ycf(c, 1), G, h3_ycf(c, 0) * R));
}
__device__ __forceinline__ void h3_corner_dots(int k, double (&d)[3]) {  // wl_color_minmax's chain
  const double v = 255.0 * (1.0 / 255.0);
  ycc_dots((k & 4) ? v : 0.0, (k & 2) ? v : 0.0, (k & 1) ? v : 0.0, d);
}
__device__ __forceinline__ int ykey(int c, int r, int g, int b) {  // exact YCbCr dot x 255000
  return __mul24(ycc_w(c, 0), r) + __mul24(ycc_w(c, 1), g) + __mul24(ycc_w(c, 2), b);
}

// Work split: a workgroup of 128 threads = 32 quads = the 8x8 blocks of 32 consecutive block
// columns; it walks H3_IT block rows down (one 4x4 sub-block per thread and step: the quad's four
// sub-blocks are consecutive lanes, as wl_haar_stats), so a thread's column and its level-1
// position advance by constants (no per-step index division).  Grid: (column strips x row
// chunks, images).  Workspace (the image's slot): |T| candidates [3][P] u32, residues [P] u32
// (level-1 position | channel mask << 28), P = (h / 2) (w / 2).
__host__ __device__ inline int h3_chunks(int h) { return ((h >> 3) + H3_IT - 1) / H3_IT; }
// the min / max form's block rows per workgroup: its workgroups are short and light, so more
// of them even out the last round of the grid
#ifndef IDN_H3_ITMM
#define IDN_H3_ITMM 8  // (A/B, bior1.5 u8: 4 132.2, 8 123.9, 16 128.4 us; the statistics at 8 instead of 16: 314 against 274)
#endif
constexpr int H3_IT_MM = IDN_H3_ITMM;
__host__ __device__ inline int h3_chunks_mm(int h) { return ((h >> 3) + H3_IT_MM - 1) / H3_IT_MM; }
// MM = true: the exact fp64 YCbCr min / max alone (the proxies, their rescans and the keys), for
// the other wavelets' u8 input in place of wl_color_minmax (ws / part unused)
template <bool MM>
__global__ __launch_bounds__(WLH_WG) __attribute__((amdgpu_waves_per_eu(IDN_H3_WPE))) void wl_h3_stats(const uint8_t* __restrict__ src, int h, int w,
                                                      int64_t row_stride, wreal* __restrict__ ws,
                                                      size_t img_floats, double* __restrict__ stats,
                                                      double* __restrict__ part, size_t part_per_img) {
  constexpr int L = 3;
  // XCD-contiguous order over (image, chunk, strip): a strip's neighbours share its edge lines
  const int lin = xcd_contiguous_block((int)(blockIdx.y * gridDim.x + blockIdx.x), (int)(gridDim.x * gridDim.y));
  const int img = lin / (int)gridDim.x, wg = lin - img * (int)gridDim.x;
  const int nbx = w >> 3, nby = h >> 3;
  const int strips = h3_strips(w);
  const int strip = wg % strips, chunk = wg / strips;
  const int sub = threadIdx.x & 3, bx = strip * H3_COLS + (threadIdx.x >> 2);
  constexpr int IT = MM ? H3_IT_MM : H3_IT;
  const int by0 = chunk * IT, nit = min(IT, nby - by0);  // block rows of this workgroup
  const bool colact = bx < nbx;
  const int x0 = bx * 8 + (sub & 1) * 4, sy = (sub >> 1) * 4;
  double* st = stats + (size_t)img * WL_STATS;
  H3Sel* sel = h3_sel(st);
  const uint32_t W1 = (uint32_t)(w >> 1), P = (uint32_t)(h >> 1) * W1;
  uint32_t* cand = reinterpret_cast<uint32_t*>(ws + img * img_floats);
  uint32_t* resl = cand + 3 * (size_t)P;
  __shared__ double red[3 * L * 3][WLH_WG / 64];
  __shared__ int ml2[3 * 6][WLH_WG];
  __shared__ int ml3[3 * 6][WLH_WG / 4];
  __shared__ uint32_t cb[3][H3_K * WLH_WG];  // [channel][slot][thread]
  __shared__ uint32_t rb[H3_KR * WLH_WG];     // residues [slot][thread]
  __shared__ uint32_t cnt_s[6];
  __shared__ float kred[6][WLH_WG / 64];
  __shared__ double dred[6][WLH_WG / 64];
  if constexpr (!MM) {
#pragma unroll
    for (int k = 0; k < 3 * 6; ++k) ml2[k][threadIdx.x] = 0;
    if (threadIdx.x < WLH_WG / 4)
#pragma unroll
      for (int k = 0; k < 3 * 6; ++k) ml3[k][threadIdx.x] = 0;
    if (threadIdx.x < 6) cnt_s[threadIdx.x] = 0u;
  }
  uint32_t lo[3] = {0u, 0u, 0u}, span[3] = {0u, 0u, 0u};
  if constexpr (!MM)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      lo[c] = (uint32_t)__builtin_amdgcn_readfirstlane((int)sel[c].lo);
      span[c] = (uint32_t)__builtin_amdgcn_readfirstlane((int)(sel[c].hi - sel[c].lo));
    }
  __syncthreads();
  int mom[3][6];
#pragma unroll
  for (int b = 0; b < 3; ++b)
#pragma unroll
    for (int k = 0; k < 6; ++k) mom[b][k] = 0;
  float pmn[3] = {INFINITY, INFINITY, INFINITY}, pmx[3] = {-INFINITY, -INFINITY, -INFINITY};
  uint32_t smn[3] = {0u, 0u, 0u}, smx[3] = {0u, 0u, 0u};  // steps near the lane's extremes
  uint32_t ct[3] = {0u, 0u, 0u}, cl[3] = {0u, 0u, 0u};  // per-lane counts: zero / below-window |T|
  uint32_t na[4] = {0u, 0u, 0u, 0u};                    // this lane's filled slots
  auto mom_lds = [&](int l, int b, int r, int g, int bl) {
    const int ld = l == 1 ? WLH_WG : WLH_WG / 4;
    int* m = l == 1 ? &ml2[b * 6][threadIdx.x] : &ml3[b * 6][threadIdx.x >> 2];
    atomicAdd(m + 0 * ld, __mul24(r, r));
    atomicAdd(m + 1 * ld, __mul24(g, g));
    atomicAdd(m + 2 * ld, __mul24(bl, bl));
    atomicAdd(m + 3 * ld, __mul24(r, g));
    atomicAdd(m + 4 * ld, __mul24(r, bl));
    atomicAdd(m + 5 * ld, __mul24(g, bl));
  };
  // this thread's sub-block at step it: rows y0 = 8 (by0 + it) + sy, columns x0 .. x0 + 3
  const uint8_t* ib = src + (int64_t)img * h * row_stride + (int64_t)(8 * by0 + sy) * row_stride +
                      (int64_t)x0 * 3;
  const int64_t step_bytes = 8 * row_stride;
  auto load_q = [&](int it, uint32_t (&qq)[4][3]) {
    if (!colact || it >= nit) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t* p = reinterpret_cast<const uint32_t*>(ib + it * step_bytes + r * row_stride);
#pragma unroll
      for (int k = 0; k < 3; ++k) qq[r][k] = p[k];
    }
  };
  auto flush = [&](int a) {  // wave-uniform
    h3_wave_flush(a < 3 ? cb[a] : rb, na[a], a < 3 ? cand + (size_t)a * P : resl,
                  a < 3 ? &sel[a].n_c : &sel[0].n_r);
    na[a] = 0u;
  };
  auto put_res = [&](bool cond, uint32_t v) {  // a lane's residue slots full: straight out
    if (cond) {
      if (na[3] < (uint32_t)H3_KR) {
        rb[na[3] * WLH_WG + threadIdx.x] = v;
        ++na[3];
      } else {
        resl[atomicAdd(&sel[0].n_r, 1u)] = v;
      }
    }
  };
  // level-1 position of group (0, 0) of this thread's sub-block at step 0; + 4 W1 per step
  const uint32_t pos00 = (uint32_t)(4 * by0 + sy / 2) * W1 + (uint32_t)(x0 / 2);
  // haar_int's band signs of x01, x10, x11 for band `sub` (ad: - + -, da: + - -, dd: - - +)
  const int s3b[3] = {sub == 1 ? 1 : -1, sub == 0 ? 1 : -1, sub == 2 ? 1 : -1};
  const uint64_t actmask = __builtin_amdgcn_ballot_w64(colact);  // lanes inside the image
  uint32_t qn[4][3] = {};
  load_q(0, qn);
  // Lanes past the image hold zero pixels throughout (load_q never fills them): their moments
  // add nothing, and their proxies, counts and masks are dropped after the loop, so the body runs
  // without per-lane branches (only the residue appends test `act`).
#pragma unroll IDN_H3_UNR
  for (int it = 0; it < nit; ++it) {
    const bool act = colact;  // (rows: it < nit, uniform)
    uint32_t q[4][3];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int k = 0; k < 3; ++k) q[r][k] = qn[r][k];
    load_q(it + 1, qn);
    auto px = [&](int r, int k) { return (int)((q[r][k >> 2] >> (8 * (k & 3))) & 0xFFu); };
    auto pxf = [&](int r, int k) { return (float)((q[r][k >> 2] >> (8 * (k & 3))) & 0xFFu); };
    // fp32 proxies of the YCbCr dots (x 255) of pixel pairs: per lane min / max (exact values
    // only where a lane is within H3_PTOL of the workgroup's extreme, after the loop)
    // Per extreme, a mask of the steps whose pixels come within H3_PTOL of the lane's running
    // extreme (reset when the extreme moves past it): at the end it holds every step with a pixel
    // within H3_PTOL of the lane's final extreme, the only steps a rescan reads.
    if (!(IDN_H3_PROBE & 1)) {
      float imn[3], imx[3];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const h3f2 R = {pxf(r, 6 * pp), pxf(r, 6 * pp + 3)}, G = {pxf(r, 6 * pp + 1), pxf(r, 6 * pp + 4)},
                     B = {pxf(r, 6 * pp + 2), pxf(r, 6 * pp + 5)};
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const h3f2 k2 = fma2(splat2(h3_ycf(c, 2)), B, fma2(splat2(h3_ycf(c, 1)), G, splat2(h3_ycf(c, 0)) * R));
            if (IDN_H3_MIN3) {  // one v_min3 / v_max3 per pair (LLVM: min + min3 + canonicalising max)
              imn[c] = r + pp == 0 ? h3_min3(k2.x, k2.x, k2.y) : h3_min3(imn[c], k2.x, k2.y);
              imx[c] = r + pp == 0 ? h3_max3(k2.x, k2.x, k2.y) : h3_max3(imx[c], k2.x, k2.y);
            } else {
              const float lo2 = __builtin_fminf(k2.x, k2.y), hi2 = __builtin_fmaxf(k2.x, k2.y);
              imn[c] = r + pp == 0 ? lo2 : __builtin_fminf(imn[c], lo2);
              imx[c] = r + pp == 0 ? hi2 : __builtin_fmaxf(imx[c], hi2);
            }
          }
        }
      const uint32_t bit = 1u << it;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        // branch-free: a new extreme past the tolerance restarts the mask; within it, adds the step
        smn[c] = (imn[c] < pmn[c] - H3_PTOL ? 0u : smn[c]) | (imn[c] <= pmn[c] + H3_PTOL ? bit : 0u);
        smx[c] = (imx[c] > pmx[c] + H3_PTOL ? 0u : smx[c]) | (imx[c] >= pmx[c] - H3_PTOL ? bit : 0u);
        pmn[c] = IDN_H3_MICRO ? h3_min3(pmn[c], imn[c], imn[c]) : __builtin_fminf(pmn[c], imn[c]);
        pmx[c] = IDN_H3_MICRO ? h3_max3(pmx[c], imx[c], imx[c]) : __builtin_fmaxf(pmx[c], imx[c]);
      }
    }
    if constexpr (MM) continue;  // (the min / max alone)
    int a1[4][3];
    h3s2 Apk[2][3];  // IDN_H3_PK: the level-1 sums of row pair gy as 16-bit pairs (gx = 0 low)
#pragma unroll
    for (int gy = 0; gy < 2; ++gy) {
      int D[2][3][3];  // [gx][band][rgb]
      h3s2 PD[3][3];   // IDN_H3_PK: [band][rgb] as 16-bit pairs (gx = 0 low, 1 high)
      if (IDN_H3_PK) {
        // the two groups side by side in 16-bit lanes: each pixel pair is one v_perm of the row
        // dwords (bytes k and k + 6, zero-extended), the butterflies are v_pk_add / v_pk_sub_u16
        // (|D| <= 510, sums <= 1020: no wrap), and the moments take the pairs as they are
        auto pk = [&](int r, int k) {  // bytes k (gx 0) and k + 6 (gx 1) of row r
          const int k1 = k + 6;
          const uint32_t sel = (uint32_t)(k & 3) | 0x0C00u | ((uint32_t)(4 + (k1 & 3)) << 16) | 0x0C000000u;
          return __builtin_bit_cast(h3s2, __builtin_amdgcn_perm(q[r][k1 >> 2], q[r][k >> 2], sel));
        };
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
          const h3s2 x00 = pk(2 * gy, ch), x01 = pk(2 * gy, 3 + ch), x10 = pk(2 * gy + 1, ch),
                     x11 = pk(2 * gy + 1, 3 + ch);
          const h3s2 lo0 = x00 + x10, lo1 = x01 + x11, hi0 = x00 - x10, hi1 = x01 - x11;
          const h3s2 A = lo0 + lo1;
          PD[0][ch] = lo0 - lo1;
          PD[1][ch] = hi0 + hi1;
          PD[2][ch] = hi0 - hi1;
          a1[gy * 2][ch] = A.x;
          a1[gy * 2 + 1][ch] = A.y;
          Apk[gy][ch] = A;
#pragma unroll
          for (int b = 0; b < 3; ++b) {
            D[0][b][ch] = PD[b][ch].x;
            D[1][b][ch] = PD[b][ch].y;
          }
        }
      } else {
#pragma unroll
        for (int gx = 0; gx < 2; ++gx)
#pragma unroll
          for (int ch = 0; ch < 3; ++ch)
            haar_int(px(2 * gy, 6 * gx + ch), px(2 * gy, 6 * gx + 3 + ch), px(2 * gy + 1, 6 * gx + ch),
                     px(2 * gy + 1, 6 * gx + 3 + ch), a1[gy * 2 + gx][ch], D[gx][0][ch], D[gx][1][ch],
                     D[gx][2][ch]);
      }
      // the two groups' moments as 16-bit pairs: one v_dot2 per moment and band (|D| <= 510)
      if (IDN_H3_MOM == 1 && !(IDN_H3_PROBE & 4))
#pragma unroll
        for (int gx = 0; gx < 2; ++gx)
#pragma unroll
          for (int b = 0; b < 3; ++b) mom_add(mom[b], D[gx][b][0], D[gx][b][1], D[gx][b][2]);
#pragma unroll
      for (int b = 0; b < ((IDN_H3_PROBE & 4) || IDN_H3_MOM == 1 ? 0 : 3); ++b) {
        h3s2 P[3];
#pragma unroll
        for (int ch = 0; ch < 3; ++ch)
          P[ch] = IDN_H3_PK ? PD[b][ch]
                            : __builtin_bit_cast(h3s2, __builtin_amdgcn_perm(D[1][b][ch], D[0][b][ch], 0x05040100u));
        mom[b][0] = __builtin_amdgcn_sdot2(P[0], P[0], mom[b][0], false);
        mom[b][1] = __builtin_amdgcn_sdot2(P[1], P[1], mom[b][1], false);
        mom[b][2] = __builtin_amdgcn_sdot2(P[2], P[2], mom[b][2], false);
        mom[b][3] = __builtin_amdgcn_sdot2(P[0], P[1], mom[b][3], false);
        mom[b][4] = __builtin_amdgcn_sdot2(P[0], P[2], mom[b][4], false);
        mom[b][5] = __builtin_amdgcn_sdot2(P[1], P[2], mom[b][5], false);
      }
#pragma unroll
      for (int gx = 0; gx < ((IDN_H3_PROBE & 2) ? 0 : 2); ++gx) {
        const uint32_t pos = pos00 + (uint32_t)(4 * it + gy) * W1 + (uint32_t)gx;
        int T[3];
        uint32_t aT[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          T[c] = ykey(c, D[gx][2][0], D[gx][2][1], D[gx][2][2]);
          aT[c] = (uint32_t)(T[c] < 0 ? -T[c] : T[c]);
          // branch-free: per-lane counts; the slot store is unconditional (a slot written
          // without the count moving is overwritten by the next append)
          // (IDN_H3_ZC: nonzero counts as the groups less the zeros, counted on the residue branch)
          if (!IDN_H3_ZC) ct[c] += aT[c] != 0u ? 1u : 0u;
          if (IDN_H3_BRW) {  // the subtraction's borrow as the below-window test
            uint32_t dl;
            cl[c] += __builtin_sub_overflow(aT[c], lo[c], &dl) ? 1u : 0u;
            cb[c][na[c] * WLH_WG + threadIdx.x] = aT[c];
            na[c] += dl <= span[c] ? 1u : 0u;
          } else {
            cl[c] += aT[c] < lo[c] ? 1u : 0u;
            cb[c][na[c] * WLH_WG + threadIdx.x] = aT[c];
            na[c] += aT[c] - lo[c] <= span[c] ? 1u : 0u;
          }
        }
        const bool z = act && min(min(aT[0], aT[1]), aT[2]) == 0u;
        if (IDN_H3_MICRO ? (__builtin_amdgcn_ballot_w64(min(min(aT[0], aT[1]), aT[2]) == 0u) & actmask) != 0ull
                         : __builtin_amdgcn_ballot_w64(z) != 0ull) {
          if (IDN_H3_ZC)
#pragma unroll
            for (int c = 0; c < 3; ++c) ct[c] += aT[c] == 0u ? 1u : 0u;  // zeros (past the image: dropped)
          auto trip = [&](int r, int k) { return (uint32_t)(px(r, k) | (px(r, k + 1) << 8) | (px(r, k + 2) << 16)); };
          const bool eq = h3_eqtrip(trip(2 * gy, 6 * gx), trip(2 * gy, 6 * gx + 3),
                                    trip(2 * gy + 1, 6 * gx), trip(2 * gy + 1, 6 * gx + 3));
          const uint32_t cm = (T[0] == 0 ? 1u : 0u) | (T[1] == 0 ? 2u : 0u) | (T[2] == 0 ? 4u : 0u);
          put_res(z && !eq, pos | (cm << 28));
        }
      }
    }
    if (MM || (IDN_H3_PROBE & 8)) continue;
    int a2[3], D2[3][3];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch)
      if (IDN_H3_PK && IDN_H3_MICRO) {  // level 2 from the packed level-1 sums of the two row pairs
        const h3s2 L = Apk[0][ch] + Apk[1][ch], H = Apk[0][ch] - Apk[1][ch];  // {lo0, lo1}, {hi0, hi1}
        a2[ch] = L.x + L.y;
        D2[0][ch] = L.x - L.y;
        D2[1][ch] = H.x + H.y;
        D2[2][ch] = H.x - H.y;
      } else {
        haar_int(a1[0][ch], a1[1][ch], a1[2][ch], a1[3][ch], a2[ch], D2[0][ch], D2[1][ch], D2[2][ch]);
      }
#pragma unroll
    for (int b = 0; b < 3; ++b) mom_lds(1, b, D2[b][0], D2[b][1], D2[b][2]);  // (zeros past the image)
    // level 3: quad lane `sub` < 3 takes band `sub` of the quad's group (haar_int's signs over
    // the quad's four level-2 sums), its moments into the quad's LDS column of that band
    if (IDN_H3_L3Q) {
      int D3[3];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch)
        D3[ch] = quad_get(a2[ch], 0) + __mul24(s3b[0], quad_get(a2[ch], 1)) +
                 __mul24(s3b[1], quad_get(a2[ch], 2)) + __mul24(s3b[2], quad_get(a2[ch], 3));
      if (sub < 3) mom_lds(2, sub, D3[0], D3[1], D3[2]);
    } else {  // the quad's first lane, all three bands
      int D3[3][3];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        int aa;
        haar_int(quad_get(a2[ch], 0), quad_get(a2[ch], 1), quad_get(a2[ch], 2), quad_get(a2[ch], 3), aa,
                 D3[0][ch], D3[1][ch], D3[2][ch]);
      }
      if (sub == 0)
#pragma unroll
        for (int b = 0; b < 3; ++b) mom_lds(2, b, D3[b][0], D3[b][1], D3[b][2]);
    }
    // a wave moves its slots out once a lane could overflow in the next step (4 appends each)
#pragma unroll
    for (int a = 0; a < 3; ++a)
      if (__builtin_amdgcn_ballot_w64(na[a] > (uint32_t)(H3_K - 4))) flush(a);
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if constexpr (!MM) {
#pragma unroll
  for (int a = 0; a < 4; ++a) flush(a);
  // counts (lanes past the image counted their zero groups: dropped)
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    uint32_t a = colact ? (IDN_H3_ZC ? 4u * (uint32_t)nit - ct[c] : ct[c]) : 0u;  // nonzero |T|
    uint32_t b = colact ? cl[c] : 0u;
    for (int o = 32; o > 0; o >>= 1) {
      a += (uint32_t)__shfl_xor((int)a, o);
      b += (uint32_t)__shfl_xor((int)b, o);
    }
    if (lane == 0) {
      atomicAdd(&cnt_s[c], a);
      atomicAdd(&cnt_s[3 + c], b);
    }
  }
  // unscaled sums of squares T^2 per (channel, level, band): w_c^T M w_c (wl_h3_sigma scales them)
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const double w0 = ycc_w(c, 0), w1 = ycc_w(c, 1), w2 = ycc_w(c, 2);
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        int m[6];
#pragma unroll
        for (int k = 0; k < 6; ++k)
          m[k] = l == 0 ? mom[b][k]
                 : l == 1 ? ml2[b * 6 + k][threadIdx.x]
                          : ((threadIdx.x & 3) == 0 ? ml3[b * 6 + k][threadIdx.x >> 2] : 0);
        double v = w0 * w0 * (double)m[0] + w1 * w1 * (double)m[1] + w2 * w2 * (double)m[2] +
                   2.0 * (w0 * w1 * (double)m[3] + w0 * w2 * (double)m[4] + w1 * w2 * (double)m[5]);
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) red[(c * L + l) * 3 + b][wave] = v;
      }
  }
  }  // !MM
  // the workgroup's extreme proxies (lanes past the image hold +-inf)
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float a = colact ? pmn[c] : INFINITY, b = colact ? pmx[c] : -INFINITY;  // (lanes past the image)
    for (int o = 32; o > 0; o >>= 1) {
      a = __builtin_fminf(a, __shfl_xor(a, o));
      b = __builtin_fmaxf(b, __shfl_xor(b, o));
    }
    if (lane == 0) {
      kred[c][wave] = a;
      kred[3 + c][wave] = b;
    }
  }
  __syncthreads();
  if (!MM && threadIdx.x < 3 * L * 3) {
    const int k = threadIdx.x, b = k % 3, l = (k / 3) % L, c = k / (3 * L);
    double t = red[k][0];
#pragma unroll
    for (int wv = 1; wv < WLH_WG / 64; ++wv) t += red[k][wv];
    part[img * part_per_img + (size_t)(c * 3 + b) * (part_per_img / 9) + (size_t)l * gridDim.x +
         (size_t)wg] = t;
  }
  if (!MM && threadIdx.x < 3) {
    atomicAdd(&sel[threadIdx.x].n_t, cnt_s[threadIdx.x]);
    atomicAdd(&sel[threadIdx.x].n_lo, cnt_s[3 + threadIdx.x]);
  }
  float gmn[3], gmx[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    gmn[c] = kred[c][0];
    gmx[c] = kred[3 + c][0];
#pragma unroll
    for (int wv = 1; wv < WLH_WG / 64; ++wv) {
      gmn[c] = __builtin_fminf(gmn[c], kred[c][wv]);
      gmx[c] = __builtin_fmaxf(gmx[c], kred[3 + c][wv]);
    }
  }
  // the fp64 chain only where a lane's proxy is within H3_PTOL of the workgroup's extreme: every
  // pixel there whose proxy is (exact ties differ in the last fp64 bits; the proxy's error is
  // below 0.03, distinct exact values 0.001 apart, so the extreme is among them)
  double dmn[3] = {INFINITY, INFINITY, INFINITY}, dmx[3] = {-INFINITY, -INFINITY, -INFINITY};
  // An extreme at the RGB cube's own (a corner: 0 / 255 channels, as saturated noise reaches) is
  // that corner's value exactly: each corner is the only triple with its exact key and the next
  // triple lies >= 18 proxy units away.  No rescan for those.
  uint32_t steps = 0u;  // the steps that may hold a workgroup extreme
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int cmn = h3_corner(c, false), cmx = h3_corner(c, true);
    const bool at_mn = gmn[c] <= h3_corner_proxy(cmn, c) + H3_PTOL;
    const bool at_mx = gmx[c] >= h3_corner_proxy(cmx, c) - H3_PTOL;
    double d[3];
    if (at_mn) {
      h3_corner_dots(cmn, d);
      dmn[c] = d[c];
    } else if (pmn[c] <= gmn[c] + H3_PTOL) {
      steps |= smn[c];
    }
    if (at_mx) {
      h3_corner_dots(cmx, d);
      dmx[c] = d[c];
    } else if (pmx[c] >= gmx[c] - H3_PTOL) {
      steps |= smx[c];
    }
  }
  if (colact && steps && !(IDN_H3_PROBE & 16)) {
#pragma unroll 1
    for (; steps; steps &= steps - 1u) {
      const int it = __builtin_ctz(steps);
      uint32_t q[4][3];
      load_q(it, q);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int r = k >> 2, p = k & 3;
        auto px = [&](int kk) { return (int)((q[r][kk >> 2] >> (8 * (kk & 3))) & 0xFFu); };
        const int R = px(3 * p), G = px(3 * p + 1), B = px(3 * p + 2);
        bool hit = false;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float pk = __fmaf_rn(h3_ycf(c, 2), (float)B, __fmaf_rn(h3_ycf(c, 1), (float)G, h3_ycf(c, 0) * (float)R));
          hit |= pk <= gmn[c] + H3_PTOL || pk >= gmx[c] - H3_PTOL;
        }
        if (!hit) continue;
        double d[3];
        ycc_dots((double)R * (1.0 / 255.0), (double)G * (1.0 / 255.0), (double)B * (1.0 / 255.0), d);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          dmn[c] = fmin(dmn[c], d[c]);
          dmx[c] = fmax(dmx[c], d[c]);
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double a = dmn[c], b = dmx[c];
    for (int o = 32; o > 0; o >>= 1) {
      a = fmin(a, __shfl_xor(a, o));
      b = fmax(b, __shfl_xor(b, o));
    }
    if (lane == 0) {
      dred[c][wave] = a;
      dred[3 + c][wave] = b;
    }
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int c = threadIdx.x;
    double a = dred[c][0], b = dred[3 + c][0];
#pragma unroll
    for (int wv = 1; wv < WLH_WG / 64; ++wv) {
      a = fmin(a, dred[c][wv]);
      b = fmax(b, dred[3 + c][wv]);
    }
    if (a <= b) {  // rounded offsets after the reduction, as wl_color_minmax
      atomicMinD(st + WlStats::MN64 + c, __dadd_rn(a, ycc_offset(c)));
      atomicMaxD(st + WlStats::MX64 + c, __dadd_rn(b, ycc_offset(c)));
    }
  }
}

// ---- wl_h3_sigma ----------------------------------------------------------------------------------
// rank `rank` of v[0..n) (u32, all in [lo, lo + span]), block-wide: radix passes of up to 11 bits
// over v - lo, as many as span needs (a 5 % window spans ~2^19: two passes), into H3_NH
// histogram copies by lane (the values crowd into few bins; one copy serialises the LDS atomics)
constexpr int H3_NH = 4;
__device__ uint32_t h3_select_u32(const uint32_t* __restrict__ v, uint32_t n, uint32_t rank,
                                  uint32_t lo, uint32_t span, uint32_t* hist) {
  const int nbits = max(32 - __clz((int)span), 1);  // bits of the largest offset
  uint32_t prefix = 0u, pmask = 0u;
#pragma unroll 1
  for (int top = nbits; top > 0; top -= 11) {
    const int wd = min(top, 11), sh = top - wd, nb = 1 << wd;
    for (int k = threadIdx.x; k < H3_NH * nb; k += blockDim.x) hist[k] = 0u;
    __syncthreads();
    uint32_t* hc = hist + (threadIdx.x & (H3_NH - 1)) * nb;
    for (uint32_t i0 = threadIdx.x; i0 < n; i0 += 4 * blockDim.x) {
      uint32_t x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t i = i0 + (uint32_t)u * blockDim.x;
        x[u] = i < n ? v[i] - lo : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i0 + (uint32_t)u * blockDim.x < n && (x[u] & pmask) == prefix)
          atomicAdd(&hc[(x[u] >> sh) & (uint32_t)(nb - 1)], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
      uint32_t t = 0;
#pragma unroll
      for (int cp = 0; cp < H3_NH; ++cp) t += hist[cp * nb + b];
      hist[b] = t;
    }
    __syncthreads();
    const BinSel bs = select_bin(hist, nb, rank, nullptr, false);
    prefix |= bs.bin << sh;
    pmask |= (uint32_t)(nb - 1) << sh;
    rank = bs.rank;
  }
  return prefix + lo;
}

// per (image, channel) workgroup of WLM_WG threads
__global__ __launch_bounds__(WLM_WG) void wl_h3_sigma(const uint8_t* __restrict__ src,
                                                      int64_t row_stride, wreal* __restrict__ ws,
                                                      size_t img_floats, double* __restrict__ stats,
                                                      WlLayout Lt, const double* __restrict__ part,
                                                      int nwg) {
  const int img = blockIdx.x / 3, c = blockIdx.x % 3;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double* st = stats + (size_t)img * WL_STATS;
  H3Sel* sel = h3_sel(st);
  const uint32_t W1 = (uint32_t)Lt.W[1], P = (uint32_t)Lt.H[1] * W1;
  const uint32_t* cand = reinterpret_cast<const uint32_t*>(ws + img * img_floats) + (size_t)c * P;
  const uint32_t* resl = reinterpret_cast<const uint32_t*>(ws + img * img_floats) + 3 * (size_t)P;
  double* kd = ws + img * img_floats + 2 * (size_t)P + (size_t)c * P;  // fallback keys
  wreal mn, mx;
  wl_minmax64(st, c, mn, mx);
  const wreal inv = mx - mn, rcp = 1.0 / inv;
  const double sc = 0.5 / (255000.0 * inv);
  __shared__ uint32_t hist[WLM_NH * WL_FBINS];
  __shared__ uint32_t red_u[WLM_WG / 64], le_s, gt_s;
  __shared__ unsigned long long gtk_s;
  __shared__ uint32_t lek_s;
  // 1. the residues of this channel: exact fp64 dd (nonzero ones count)
  const uint32_t nr = sel[0].n_r;
  uint32_t nz = 0;
  constexpr int BQ = 6;
  for (uint32_t t0 = threadIdx.x; t0 < nr; t0 += BQ * WLM_WG) {
    uint32_t e[BQ];
    Dd1Raw q[BQ];
#pragma unroll
    for (int u = 0; u < BQ; ++u) {
      e[u] = resl[min(t0 + (uint32_t)u * WLM_WG, nr - 1)];
      q[u] = wl_dd1_load(src, img, Lt.h, row_stride, e[u] & 0x0FFFFFFFu, (int)W1);
    }
#pragma unroll
    for (int u = 0; u < BQ; ++u)
      if (t0 + (uint32_t)u * WLM_WG < nr && ((e[u] >> (28 + c)) & 1u))
        nz += wl_dd1_eval<true>(q[u], c, mn, inv, rcp) != 0ull ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) nz += (uint32_t)__shfl_xor((int)nz, o);
  if (lane == 0) red_u[wave] = nz;
  if (threadIdx.x == 0) {
    le_s = 0u;
    gt_s = 0xFFFFFFFFu;
    gtk_s = ~0ull;
    lek_s = 0u;
  }
  __syncthreads();
  uint32_t nrnz = 0;
#pragma unroll
  for (int k = 0; k < WLM_WG / 64; ++k) nrnz += red_u[k];
  // 2. the median ranks among the nonzero finest dd (residues rank below every T != 0)
  const uint32_t n_t = sel[c].n_t, n_c = sel[c].n_c;
  const uint32_t below = sel[c].n_lo - (P - n_t);  // 0 < |T| < lo
  const uint32_t N = n_t + nrnz;
  double med = NAN;
  uint32_t total = N;
  bool fb = false;
  if (N) {
    const uint32_t klo = (N - 1) / 2, khi = N / 2;
    const uint32_t base = nrnz + below;  // rank of the window's first |T|
    if (klo >= base && khi < base + n_c) {
      const uint32_t rlo = klo - base, rhi = khi - base;
      const uint32_t wlo = sel[c].lo, wspan = sel[c].hi - sel[c].lo;
      const uint32_t tlo = h3_select_u32(cand, n_c, rlo, wlo, wspan, hist);
      uint32_t thi = tlo;
      if (rhi != rlo) {  // the upper middle: the same value while enough |T| are <= it
        uint32_t le = 0, gt = 0xFFFFFFFFu;
        for (uint32_t i = threadIdx.x; i < n_c; i += WLM_WG) {
          const uint32_t x = cand[i];
          if (x <= tlo) ++le;
          else gt = min(gt, x);
        }
        for (int o = 32; o > 0; o >>= 1) {
          le += (uint32_t)__shfl_xor((int)le, o);
          gt = min(gt, (uint32_t)__shfl_xor((int)gt, o));
        }
        if (lane == 0) {
          atomicAdd(&le_s, le);
          atomicMin(&gt_s, gt);
        }
        __syncthreads();
        if (le_s <= rhi) thi = gt_s;
      }
      med = ((double)tlo * sc + (double)thi * sc) / 2.0;
    } else {
      fb = true;
    }
  }
  if (fb) {
    // exact full-image selection: the reference's fp64 |dd| of every position (wl_dd1_key), then
    // the radix passes of wl_haar_median over them
    for (uint32_t p0 = threadIdx.x; p0 < P; p0 += BQ * WLM_WG) {
      Dd1Raw q[BQ];
#pragma unroll
      for (int u = 0; u < BQ; ++u)
        q[u] = wl_dd1_load(src, img, Lt.h, row_stride, min(p0 + (uint32_t)u * WLM_WG, P - 1), (int)W1);
#pragma unroll
      for (int u = 0; u < BQ; ++u)
        if (p0 + (uint32_t)u * WLM_WG < P)
          kd[p0 + (uint32_t)u * WLM_WG] =
              __longlong_as_double((long long)wl_dd1_eval<true>(q[u], c, mn, inv, rcp));
    }
    __syncthreads();
    RadixState rsx{0ull, 0ull, 0u};
    radix_pass(kd, P, 52, 11, rsx, hist, &total);
    if (total) {
      radix_pass(kd, P, 41, 11, rsx, hist, nullptr);
      radix_pass(kd, P, 30, 11, rsx, hist, nullptr);
      radix_pass(kd, P, 19, 11, rsx, hist, nullptr);
      radix_pass(kd, P, 8, 11, rsx, hist, nullptr);
      radix_pass(kd, P, 0, 8, rsx, hist, nullptr);
      const unsigned long long lo_key = rsx.prefix;
      const double vlo = __longlong_as_double((long long)lo_key);
      double vhi = vlo;
      if ((total - 1) / 2 != total / 2) {
        uint32_t le = 0;
        unsigned long long gt = ~0ull;
        for (uint32_t k = threadIdx.x; k < P; k += WLM_WG) {
          const unsigned long long key = absbits(kd[k]);
          if (key == 0ull) continue;
          if (key <= lo_key) ++le;
          else gt = key < gt ? key : gt;
        }
        for (int o = 32; o > 0; o >>= 1) {
          le += (uint32_t)__shfl_xor((int)le, o);
          const unsigned long long og = (unsigned long long)__shfl_xor((long long)gt, o);
          gt = og < gt ? og : gt;
        }
        if (lane == 0) {
          atomicAdd(&lek_s, le);
          atomicMin(&gtk_s, gt);
        }
        __syncthreads();
        if (lek_s <= total / 2) vhi = __longlong_as_double((long long)gtk_s);
      }
      med = (vlo + vhi) / 2.0;
    } else {
      med = NAN;
    }
  }
  // 3. sums of squares (wl_h3_stats' unscaled partials, in workgroup order) and thresholds
  __shared__ double sums[9];
  for (int k = wave; k < 9; k += WLM_WG / 64) {
    const int l = k / 3, b = k - 3 * l;
    const double* p = part + img * Lt.part_per_img + (size_t)(c * 3 + b) * (Lt.part_per_img / 9) +
                      (size_t)l * nwg;
    double s = 0.0;
    for (int t = lane; t < nwg; t += 64) s += p[t];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) {
      const double sl = ldexp(sc, -l);  // level l + 1's coefficient scale
      sums[k] = s * (sl * sl);
    }
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  constexpr int L = 3;
  st[WlStats::median(c, L)] = med;
  st[WlStats::DIAG + c] = (double)total;
  sel[c].fb = fb ? 1u : 0u;
  const double sigma = med / 0.6744897501960817;
  const bool bad = !(mx > mn) || !(sigma == sigma);
  const double var = sigma * sigma;
  for (int l = 0; l < L; ++l)
    for (int b = 0; b < 3; ++b) {
      const double sq = sums[3 * l + b];
      st[WlStats::sumsq(c, l, b, L)] = sq;
      const double cnt = (double)Lt.H[l + 1] * Lt.W[l + 1];
      const double t = var / sqrt(fmax(sq / cnt - var, 2.220446049250313e-16));
      st[WlStats::thr(c, l, b, L)] = t;
      st[WlStats::thrh(c, l, b)] = 0.5 * t;
    }
  if (bad) st[WlStats::FLAG] = 1.0;
  h3_consts(st, c);
}
