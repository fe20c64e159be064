// cv2.bilateralFilter(u8, d, sigma_color, sigma_space, borderType=BORDER_CONSTANT) for C = 3 / 1.
// Reference call sites: lib/model/test.py:272-278 (d=9, sigmaColor=20, sigmaSpace=100),
// lib/roi_data_layer/minibatch.py:172,1658-1663; BASELINE config 4 uses sigma 75/75.
//
// OpenCV 3.4.2 bilateralFilter_8u semantics (restated in oracle/filters.c): radius = d/2, taps
// {(i,j): sqrt(i^2+j^2) <= radius}, space weight float(exp(r^2 * -0.5/ss^2)), colour weight of
// the L1 distance |db|+|dg|+|dr|, float sums, out = cvRound(sum * (1.f / wsum)), border pixels 0.
//
// gfx950 design: a 256-thread workgroup owns a 64 x 16 output tile; the (64+2r) x (16+2r) input
// tile (BGR0-packed u32 per pixel, zero outside the image) is staged once in LDS, next to
// OpenCV's colour-weight table color_weight[i] = float(exp(i^2 * -0.5/sc^2)), i = 0..765, which
// each workgroup builds in LDS.  Each thread walks 4 output rows of one column.  Per tap: v_sad_u8
// on the packed pixels gives the L1 colour distance in one instruction, the weight is OpenCV's
// space_weight[k] * color_weight[dist] (space weights are compile-time taps in SGPRs), and
// (b, g) / (r, wsum) accumulate as packed fp32 pairs.  The weights are then exactly OpenCV's;
// only the fp32 summation order differs (<= 1 LSB after cvRound).
#include "idn_common.hpp"

#include <math.h>
#include <string.h>

namespace idn {

typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int BL_TW = 64;   // tile width (outputs)
constexpr int BL_TH = 16;   // tile height (outputs)
constexpr int BL_RPT = 4;   // output rows per thread
constexpr int BL_MAXR = 8;  // max radius supported (d <= 17)

struct BilateralTaps {
  double gcc;                                       // -0.5 / sigma_color^2
  float sw[(2 * BL_MAXR + 1) * (2 * BL_MAXR + 1)];  // space weight at (i+R)*(2R+1)+(j+R)
  float swq[BL_MAXR * BL_MAXR + 1];                 // space weight by r^2 = i^2 + j^2
  float kc;                                         // gcc * log2(e) (computed colour weights)
  float ksq[BL_MAXR * BL_MAXR + 1];                 // log2(space weight) by r^2
};
// computed weights (A/B, bilateral_u8_pre2_kernel): bit k set = the taps of the k-th distinct r^2
// take exp2(dist^2 * kc + log2(space weight)) on v_exp_f32 instead of the LDS table read
#ifndef IDN_BL_CW
#define IDN_BL_CW 0
#endif
#ifndef IDN_BL2_WGD  // resident workgroups per CU of the two-column kernel
#define IDN_BL2_WGD 2
#endif
constexpr int BL_LUT = 3 * 255 + 1;

template <int C>
__device__ __forceinline__ uint32_t load_px(const uint8_t* __restrict__ s, int64_t row_stride,
                                            int h, int w, int y, int x) {
  if (y < 0 || y >= h || x < 0 || x >= w) return 0u;  // BORDER_CONSTANT (0)
  const uint8_t* p = s + (int64_t)y * row_stride + (int64_t)x * C;
  if constexpr (C == 3) return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
  else return (uint32_t)p[0];
}

template <int C, int R>
__global__ __launch_bounds__(256) void bilateral_u8_kernel(const uint8_t* __restrict__ src,
                                                           uint8_t* __restrict__ dst, int h, int w,
                                                           int64_t row_stride, int tiles_x,
                                                           int tiles_y, BilateralTaps taps) {
  constexpr int LW = BL_TW + 2 * R;
  constexpr int LH = BL_TH + 2 * R;
  __shared__ uint32_t tile[LH * LW];
  __shared__ float cw[BL_LUT];

  const int t = blockIdx.x;
  const int tx = t % tiles_x;
  const int ty = (t / tiles_x) % tiles_y;
  const int img = t / (tiles_x * tiles_y);
  const uint8_t* s = src + (int64_t)img * h * row_stride;
  uint8_t* d = dst + (int64_t)img * h * row_stride;
  const int x0 = tx * BL_TW, y0 = ty * BL_TH;

  for (int i = threadIdx.x; i < LH * LW; i += 256) {
    const int ly = i / LW, lx = i % LW;
    tile[i] = load_px<C>(s, row_stride, h, w, y0 + ly - R, x0 + lx - R);
  }
  for (int i = threadIdx.x; i < BL_LUT; i += 256) cw[i] = (float)exp((double)(i * i) * taps.gcc);
  __syncthreads();

  const int col = threadIdx.x & 63;
  const int rgrp = threadIdx.x >> 6;  // 4 groups of BL_RPT rows
  const int x = x0 + col;
  if (x >= w) return;
#pragma unroll 1
  for (int rr = 0; rr < BL_RPT; ++rr) {
    const int ly = rgrp * BL_RPT + rr;
    const int y = y0 + ly;
    if (y >= h) break;
    const uint32_t p0 = tile[(ly + R) * LW + col + R];
    // (b, g) and (r, wsum) accumulate as packed pairs: one v_pk_fma_f32 each per tap
    f32x2 acc_bg = {0.f, 0.f}, acc_rw = {0.f, 0.f};
#pragma unroll
    for (int i = -R; i <= R; ++i) {
#pragma unroll
      for (int j = -R; j <= R; ++j) {
        if (i * i + j * j > R * R) continue;  // sqrt(i^2+j^2) > radius: not a tap
        const uint32_t p = tile[(ly + R + i) * LW + col + R + j];
        const uint32_t dist = __builtin_amdgcn_sad_u8(p, p0, 0u);
        const float wt = taps.sw[(i + R) * (2 * R + 1) + (j + R)] * cw[dist];
        const f32x2 w2 = {wt, wt};
        if constexpr (C == 3) {
          const f32x2 bg = {(float)(p & 0xFFu), (float)((p >> 8) & 0xFFu)};
          const f32x2 r1 = {(float)((p >> 16) & 0xFFu), 1.f};
          acc_bg = __builtin_elementwise_fma(bg, w2, acc_bg);
          acc_rw = __builtin_elementwise_fma(r1, w2, acc_rw);
        } else {
          const f32x2 b1 = {(float)(p & 0xFFu), 1.f};
          acc_rw = __builtin_elementwise_fma(b1, w2, acc_rw);
        }
      }
    }
    const float sb = (C == 3) ? acc_bg.x : acc_rw.x, sg = acc_bg.y, sr = acc_rw.x;
    const float ws = acc_rw.y;
    const float inv = 1.f / ws;
    uint8_t* o = d + (int64_t)y * row_stride + (int64_t)x * C;
    // cvRound = round half to even (v_rndne), saturate to u8
    auto cvt = [](float v) -> uint8_t {
      const float r = __builtin_rintf(v);
      return (uint8_t)(r < 0.f ? 0.f : (r > 255.f ? 255.f : r));
    };
    o[0] = cvt(sb * inv);
    if constexpr (C == 3) {
      o[1] = cvt(sg * inv);
      o[2] = cvt(sr * inv);
    }
  }
}

// ---- C = 3, radius <= 5: pre-multiplied per-radius weight tables ---------------------------------
// OpenCV's weight is float(space_weight[k] * color_weight[dist]); the space weight depends only on
// r^2 = i^2 + j^2, so the workgroup stores one table per distinct r^2 with the products already
// formed (the same float multiply, so the same bits): a tap is v_sad_u8 + one shift + one LDS read
// + two packed FMAs.  Each thread owns 4 output rows of one column and walks the (4 + 2R) x (2R+1)
// input pixels of their union once: every pixel is read from LDS and converted to float once and
// feeds each of the (up to 4) outputs it is a tap of.  512-thread workgroups (32-row tiles): the
// 34 KB of tables per workgroup then allow 6 waves per SIMD (256 threads: 3).
template <int R>
struct Rsq {  // the distinct r^2 <= R^2 that are taps: table slot of each r^2, r^2 of each slot
  int n = 0;
  int slot[R * R + 1] = {};
  int q[R * R + 1] = {};
  constexpr Rsq() {
    for (int v = 0; v <= R * R; ++v) slot[v] = -1;
    for (int v = 0; v <= R * R; ++v)
      for (int i = 0; i <= R; ++i)
        for (int j = 0; j <= R; ++j)
          if (i * i + j * j == v && slot[v] < 0) {
            q[n] = v;
            slot[v] = n++;
          }
  }
};

constexpr int BLP_NW = 8;  // waves per workgroup of the pre-multiplied kernel
template <int R, int RPT>
__global__ __launch_bounds__(64 * BLP_NW) void bilateral_u8_pre_kernel(const uint8_t* __restrict__ src,
                                                               uint8_t* __restrict__ dst, int h,
                                                               int w, int64_t row_stride,
                                                               int tiles_x, int tiles_y,
                                                               int ntiles, BilateralTaps taps) {
  constexpr int LW = BL_TW + 2 * R;
  constexpr int NT = 64 * BLP_NW;
  constexpr int TH = BLP_NW * RPT;  // tile height: one wave per RPT rows
  constexpr int LH = TH + 2 * R;
  constexpr Rsq<R> RS;
  __shared__ uint32_t tile[LH * LW];
  __shared__ float cw[BL_LUT];
  __shared__ float wt[RS.n * BL_LUT];

  // the weight tables, once per (persistent) workgroup
  for (int i = threadIdx.x; i < BL_LUT; i += NT) cw[i] = (float)exp((double)(i * i) * taps.gcc);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < RS.n; ++k) {
    const float sw = taps.swq[RS.q[k]];
    for (int i = threadIdx.x; i < BL_LUT; i += NT)
      wt[k * BL_LUT + i] = sw * cw[i];  // OpenCV: space_weight[k] * color_weight[dist]
  }

  const int col = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ly0 = wave * RPT;  // first of the thread's RPT output rows
  const uint32_t img_bytes = (uint32_t)((int64_t)h * row_stride);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int tx = t % tiles_x;
    const int ty = (t / tiles_x) % tiles_y;
    const int img = t / (tiles_x * tiles_y);
    const uint8_t* s = src + (int64_t)img * h * row_stride;
    uint8_t* d = dst + (int64_t)img * h * row_stride;
    const int x0 = tx * BL_TW, y0 = ty * TH;
    // staging: wave wv stages tile rows wv, wv + NW, ..., lane the columns lane and 64 + lane; one
    // unaligned dword load per pixel, bytes 3x-1 .. 3x+2 (0 .. 3 at x = 0; the launcher requires
    // w >= 2), so no load reaches past the image.  Rows / columns outside the image read 0
    // (BORDER_CONSTANT) through the buffer's range check (offsets >= 2^30; the launcher requires
    // images < 2^30 bytes).
    const rsrc_t rs = make_rsrc(s, img_bytes);
    uint32_t xo[2], sh[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int x = x0 + 64 * k + col - R;
      const bool in = x >= 0 && x < w;
      xo[k] = !in ? 0x40000000u : (x > 0 ? 3u * (uint32_t)x - 1u : 0u);
      sh[k] = x > 0 ? 8u : 0u;
    }
    __syncthreads();  // the previous tile is consumed (and the tables are built)
    for (int ly = wave; ly < LH; ly += BLP_NW) {
      const int y = y0 + ly - R;  // wave-uniform
      const uint32_t so = (y >= 0 && y < h) ? (uint32_t)y * (uint32_t)row_stride : 0x40000000u;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (64 * k + col < LW) {
          const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rs, xo[k], so, 0);
          tile[ly * LW + 64 * k + col] = (v >> sh[k]) & 0xFFFFFFu;
        }
      }
    }
    __syncthreads();

    const int x = x0 + col;
    if (x >= w) continue;
    uint32_t p0[RPT];
#pragma unroll
    for (int o = 0; o < RPT; ++o) p0[o] = tile[(ly0 + o + R) * LW + col + R];
    f32x2 acc_bg[RPT], acc_rw[RPT];
#pragma unroll
    for (int o = 0; o < RPT; ++o) acc_bg[o] = acc_rw[o] = f32x2{0.f, 0.f};
#pragma unroll
    for (int dy = -R; dy < RPT + R; ++dy) {
#pragma unroll
      for (int j = -R; j <= R; ++j) {
        const uint32_t p = tile[(ly0 + R + dy) * LW + col + R + j];
        const f32x2 bg = {(float)(p & 0xFFu), (float)((p >> 8) & 0xFFu)};  // v_cvt_f32_ubyte0/1
        const f32x2 r1 = {(float)((p >> 16) & 0xFFu), 1.f};
#pragma unroll
        for (int o = 0; o < RPT; ++o) {
          const int i = dy - o;
          if (i < -R || i > R || i * i + j * j > R * R) continue;  // not a tap of output o
          const uint32_t dist = __builtin_amdgcn_sad_u8(p, p0[o], 0u);
          const float wv = wt[RS.slot[i * i + j * j] * BL_LUT + dist];
          const f32x2 w2 = {wv, wv};
          acc_bg[o] = __builtin_elementwise_fma(bg, w2, acc_bg[o]);
          acc_rw[o] = __builtin_elementwise_fma(r1, w2, acc_rw[o]);
        }
      }
      // pin the accumulators at every input row: without it LLVM sinks all the FMA pairs below
      // the walk and keeps every weight and converted pixel live (VGPRs exhausted)
#pragma unroll
      for (int o = 0; o < RPT; ++o) asm volatile("" : "+v"(acc_bg[o]), "+v"(acc_rw[o]));
    }
    auto cvt = [](float v) -> uint8_t {  // cvRound (half to even) + saturate
      const float r = __builtin_rintf(v);
      return (uint8_t)(r < 0.f ? 0.f : (r > 255.f ? 255.f : r));
    };
#pragma unroll
    for (int o = 0; o < RPT; ++o) {
      const int y = y0 + ly0 + o;
      if (y >= h) break;
      const float inv = 1.f / acc_rw[o].y;
      uint8_t* op = d + (int64_t)y * row_stride + (int64_t)x * 3;
      op[0] = cvt(acc_bg[o].x * inv);
      op[1] = cvt(acc_bg[o].y * inv);
      op[2] = cvt(acc_rw[o].x * inv);
    }
  }
}

// ---- two adjacent columns x 4 rows per thread ---------------------------------------------------
// A pixel is a tap of up to 8 of the thread's outputs, so it is read from LDS and converted to
// float once per 8 outputs instead of once per 4 (~12.5 instead of 19 reads + 3 conversions per
// output).  Lane l owns columns 2l, 2l+1 of a 128-wide tile; the staged rows keep even and odd
// columns in separate halves (column x at (x & 1) * HW + x / 2), so for every tap the 64 lanes
// read consecutive dwords (the plain layout would make every pixel read a 2-way bank conflict,
// which is what sank the first two-column attempt).  The colour table is built straight into the
// per-r^2 products (color_weight is never stored): 30 KB of tables per workgroup.
constexpr int BL2_TW = 128;
// 1/x for x in [1, 128) (the kernel's weight sums: the centre weight is exactly 1, at most 81
// taps of weight <= 1): v_rcp_f32 and one Newton step, equal to the IEEE quotient 1.f / x for
// every float of the range (all 7 * 2^23 checked on the device: idn_internal_bl_recip_check,
// tests/test_filters_gpu.py) -- 3 instructions instead of the ~10 of the general division.
__device__ __forceinline__ float bl_recip(float x) {
  const float r = __builtin_amdgcn_rcpf(x);
  return __fmaf_rn(__fmaf_rn(-x, r, 1.f), r, r);
}
__global__ __launch_bounds__(256) void bl_recip_check_kernel(unsigned int* __restrict__ bad) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;  // floats [1, 128): 7 binades
  if (i >= 7u << 23) return;
  const float x = __uint_as_float(0x3F800000u + i);
  if (__float_as_uint(bl_recip(x)) != __float_as_uint(__fdiv_rn(1.f, x))) atomicAdd(bad, 1u);
}
template <int R, bool SYM = true>
__global__ __launch_bounds__(64 * BLP_NW) void bilateral_u8_pre2_kernel(
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int h, int w, int64_t row_stride,
    int tiles_x, int tiles_y, int ntiles, BilateralTaps taps) {
  constexpr int RPT = 4;
  constexpr int LWX = BL2_TW + 2 * R;  // staged columns
  constexpr int HW = (LWX + 1) / 2;    // columns per parity half
  constexpr int LW = 2 * HW;           // LDS row pitch (dwords)
  constexpr int NT = 64 * BLP_NW;
  constexpr int TH = BLP_NW * RPT;
  constexpr int LH = TH + 2 * R;
  constexpr Rsq<R> RS;
  constexpr uint32_t ALL = (1u << RS.n) - 1u;
  constexpr bool TABLE = (IDN_BL_CW & ALL) != ALL;  // some taps still read the table
  __shared__ uint32_t tile[LH * LW];
  __shared__ float wt[TABLE ? RS.n * BL_LUT : 1];

  // wt[k][i] = space_weight(r^2 = q_k) * color_weight[i], OpenCV's float product
  if (TABLE)
    for (int i = threadIdx.x; i < BL_LUT; i += NT) {
      const float cwv = (float)exp((double)(i * i) * taps.gcc);
#pragma unroll
      for (int k = 0; k < RS.n; ++k) wt[k * BL_LUT + i] = taps.swq[RS.q[k]] * cwv;
    }

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ly0 = wave * RPT;
  const uint32_t img_bytes = (uint32_t)((int64_t)h * row_stride);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int tx = t % tiles_x;
    const int ty = (t / tiles_x) % tiles_y;
    const int img = t / (tiles_x * tiles_y);
    const uint8_t* s = src + (int64_t)img * h * row_stride;
    uint8_t* d = dst + (int64_t)img * h * row_stride;
    const int x0 = tx * BL2_TW, y0 = ty * TH;
    // staging as bilateral_u8_pre_kernel (one unaligned dword per pixel, zero outside the image),
    // staged column sx = lane + 64 k at (sx & 1) * HW + sx / 2
    const rsrc_t rs = make_rsrc(s, img_bytes);
    constexpr int NK = (LWX + 63) / 64;
    uint32_t xo[NK], sh[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int x = x0 + 64 * k + lane - R;
      const bool in = x >= 0 && x < w;
      xo[k] = !in ? 0x40000000u : (x > 0 ? 3u * (uint32_t)x - 1u : 0u);
      sh[k] = x > 0 ? 8u : 0u;
    }
    __syncthreads();  // the previous tile is consumed (and the tables are built)
    for (int ly = wave; ly < LH; ly += BLP_NW) {
      const int y = y0 + ly - R;
      const uint32_t so = (y >= 0 && y < h) ? (uint32_t)y * (uint32_t)row_stride : 0x40000000u;
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        const int sx = 64 * k + lane;
        if (sx < LWX) {
          const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rs, xo[k], so, 0);
          tile[ly * LW + (sx & 1) * HW + (sx >> 1)] = (v >> sh[k]) & 0xFFFFFFu;
        }
      }
    }
    __syncthreads();

    // staged column of output column 2 lane + cc, offset j: 2 lane + cc + R + j
    auto at = [&](int row, int rel) -> uint32_t {  // rel = cc + R + j (compile time)
      return tile[row * LW + (rel & 1) * HW + lane + (rel >> 1)];
    };
    uint32_t p0[RPT][2];
#pragma unroll
    for (int o = 0; o < RPT; ++o)
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) p0[o][cc] = at(ly0 + o + R, cc + R);
    f32x2 acc_bg[RPT][2], acc_rw[RPT][2];
#pragma unroll
    for (int o = 0; o < RPT; ++o)
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) acc_bg[o][cc] = acc_rw[o][cc] = f32x2{0.f, 0.f};
    // weights shared by two of the thread's own outputs (w(A, B) = w(B, A): same r^2, same SAD),
    // looked up at the first of the two visits in the walk order and kept in a register for the
    // second; the centre tap's weight is the constant wt[slot(0)][0].  Each output's sum keeps
    // its order, so the results are unchanged bit for bit.
    const float w00 = TABLE ? wt[RS.slot[0] * BL_LUT] : 1.f;  // float(exp(0)) * float(exp(0))
    float wsh[RPT * 2][RPT * 2];
#pragma unroll
    for (int dy = -R; dy < RPT + R; ++dy) {
#pragma unroll
      for (int rel = 0; rel <= 2 * R + 1; ++rel) {  // staged columns 2 lane .. 2 lane + 2R + 1
        bool any = false;
#pragma unroll
        for (int o = 0; o < RPT; ++o)
#pragma unroll
          for (int cc = 0; cc < 2; ++cc) {
            const int i = dy - o, j = rel - cc - R;
            any |= (i >= -R && i <= R && j >= -R && j <= R && i * i + j * j <= R * R);
          }
        if (!any) continue;
        const uint32_t p = at(ly0 + R + dy, rel);
        const f32x2 bg = {(float)(p & 0xFFu), (float)((p >> 8) & 0xFFu)};
        const f32x2 r1 = {(float)((p >> 16) & 0xFFu), 1.f};
#pragma unroll
        for (int o = 0; o < RPT; ++o)
#pragma unroll
          for (int cc = 0; cc < 2; ++cc) {
            const int i = dy - o, j = rel - cc - R;
            if (i < -R || i > R || j < -R || j > R || i * i + j * j > R * R) continue;
            // walk positions of the tap (meaningful when it is one of the thread's own outputs)
            // and of the output
            const bool own = dy >= 0 && dy < RPT && rel - R >= 0 && rel - R < 2;
            const int kx = dy * 2 + (rel - R), ky = o * 2 + cc;
            float wv;
            if (SYM && own && kx == ky) {
              wv = w00;
            } else if (SYM && own && kx > ky) {
              wv = wsh[ky][kx];  // looked up when the walk passed the output's own position
            } else {
              const uint32_t dist = __builtin_amdgcn_sad_u8(p, p0[o][cc], 0u);
              if ((IDN_BL_CW >> RS.slot[i * i + j * j]) & 1) {
                const float df = (float)dist;
                wv = __builtin_amdgcn_exp2f(__fmaf_rn(df * df, taps.kc, taps.ksq[i * i + j * j]));
              } else {
                wv = wt[RS.slot[i * i + j * j] * BL_LUT + dist];
              }
              if (SYM && own) wsh[kx][ky] = wv;
            }
            const f32x2 w2 = {wv, wv};
            acc_bg[o][cc] = __builtin_elementwise_fma(bg, w2, acc_bg[o][cc]);
            acc_rw[o][cc] = __builtin_elementwise_fma(r1, w2, acc_rw[o][cc]);
          }
      }
#pragma unroll
      for (int o = 0; o < RPT; ++o)
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) asm volatile("" : "+v"(acc_bg[o][cc]), "+v"(acc_rw[o][cc]));
    }
    auto cvt = [](float v) -> uint32_t {  // cvRound (half to even) + saturate (finite v)
      return (uint32_t)__builtin_amdgcn_fmed3f(__builtin_rintf(v), 0.f, 255.f);
    };
    const int x = x0 + 2 * lane;
    if (x >= w) continue;
#pragma unroll
    for (int o = 0; o < RPT; ++o) {
      const int y = y0 + ly0 + o;
      if (y >= h) break;
      uint32_t b[6];
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const float inv = SYM ? bl_recip(acc_rw[o][cc].y) : 1.f / acc_rw[o][cc].y;
        b[3 * cc + 0] = cvt(acc_bg[o][cc].x * inv);
        b[3 * cc + 1] = cvt(acc_bg[o][cc].y * inv);
        b[3 * cc + 2] = cvt(acc_rw[o][cc].x * inv);
      }
      uint8_t* op = d + (int64_t)y * row_stride + (int64_t)x * 3;
      if (x + 1 < w && (((uintptr_t)op) & 1) == 0) {  // 6 bytes as three u16 stores
        uint16_t* o16 = reinterpret_cast<uint16_t*>(op);
        o16[0] = (uint16_t)(b[0] | b[1] << 8);
        o16[1] = (uint16_t)(b[2] | b[3] << 8);
        o16[2] = (uint16_t)(b[4] | b[5] << 8);
      } else {
#pragma unroll
        for (int k = 0; k < 6; ++k)
          if (k < 3 || x + 1 < w) op[k] = (uint8_t)b[k];
      }
    }
  }
}

template <int R>
static void launch_bl_pre2(const uint8_t* src, uint8_t* dst, int n, int h, int w, int64_t rs,
                           const BilateralTaps& taps, hipStream_t st) {
  const int tiles_x = (w + BL2_TW - 1) / BL2_TW;
  const int tiles_y = (h + BLP_NW * 4 - 1) / (BLP_NW * 4);
  const int64_t ntiles = (int64_t)n * tiles_x * tiles_y;
  const int64_t res = (int64_t)cu_count() * knob("IDN_BL2_WG", IDN_BL2_WGD);  // resident workgroups per CU
  const int64_t grid = ntiles < res ? ntiles : res;
  if (knob("IDN_BL2_SYM", 1))
    hipLaunchKernelGGL((bilateral_u8_pre2_kernel<R, true>), dim3((unsigned)grid), dim3(64 * BLP_NW),
                       0, st, src, dst, h, w, rs, tiles_x, tiles_y, (int)ntiles, taps);
  else
    hipLaunchKernelGGL((bilateral_u8_pre2_kernel<R, false>), dim3((unsigned)grid), dim3(64 * BLP_NW),
                       0, st, src, dst, h, w, rs, tiles_x, tiles_y, (int)ntiles, taps);
}

template <int R, int RPT>
static void launch_bl_pre_rpt(const uint8_t* src, uint8_t* dst, int n, int h, int w, int64_t rs,
                              const BilateralTaps& taps, hipStream_t st) {
  const int tiles_x = (w + BL_TW - 1) / BL_TW;
  const int tiles_y = (h + BLP_NW * RPT - 1) / (BLP_NW * RPT);
  const int64_t ntiles = (int64_t)n * tiles_x * tiles_y;
  // persistent workgroups, as many as are resident (3 per CU: LDS): the weight tables are built
  // once per workgroup
  const int64_t res = (int64_t)cu_count() * 3;
  const int64_t grid = ntiles < res ? ntiles : res;
  hipLaunchKernelGGL((bilateral_u8_pre_kernel<R, RPT>), dim3((unsigned)grid), dim3(64 * BLP_NW), 0, st, src,
                     dst, h, w, rs, tiles_x, tiles_y, (int)ntiles, taps);
}

// RPT output rows per thread: each converted pixel feeds up to RPT outputs (RPT = 5 / 6 measured
// 1.87 / 2.27 ms against 1.71 in steady state, though 5 % / 8 % fewer VALU per output; RPT = 8
// worse: the compiler spills the 16 accumulators around the pins; 2 columns x 4 rows per thread,
// 15 instead of 27 conversions per output, measured 2.18 / 1.95 ms at 3 / 2 workgroups per CU
// against 1.74)
template <int R>
static void launch_bl_pre(const uint8_t* src, uint8_t* dst, int n, int h, int w, int64_t rs,
                          const BilateralTaps& taps, hipStream_t st) {
  if (knob("IDN_BL2", 1)) launch_bl_pre2<R>(src, dst, n, h, w, rs, taps, st);
  else launch_bl_pre_rpt<R, 4>(src, dst, n, h, w, rs, taps, st);
}

template <int C, int R>
static void launch_bl(const uint8_t* src, uint8_t* dst, int n, int h, int w, int64_t rs,
                      const BilateralTaps& taps, hipStream_t st) {
  const int tiles_x = (w + BL_TW - 1) / BL_TW, tiles_y = (h + BL_TH - 1) / BL_TH;
  const int64_t blocks = (int64_t)n * tiles_x * tiles_y;
  hipLaunchKernelGGL((bilateral_u8_kernel<C, R>), dim3((unsigned)blocks), dim3(256), 0, st, src,
                     dst, h, w, rs, tiles_x, tiles_y, taps);
}

}  // namespace idn

// test hook (not part of include/idn.h): number of floats x in [1, 128) whose bl_recip(x)
// differs from the IEEE 1.f / x; -1 on a launch error
extern "C" int idn_internal_bl_recip_check(void* stream) {
  using namespace idn;
  hipStream_t st = as_stream(stream);
  unsigned int* bad = nullptr;
  if (hipMalloc(&bad, sizeof(unsigned int)) != hipSuccess) return -1;
  unsigned int h_bad = 0;
  int rc = -1;
  if (hipMemsetAsync(bad, 0, sizeof(unsigned int), st) == hipSuccess) {
    hipLaunchKernelGGL(bl_recip_check_kernel, dim3((7u << 23) / 256u), dim3(256), 0, st, bad);
    if (hipGetLastError() == hipSuccess &&
        hipMemcpyAsync(&h_bad, bad, sizeof(unsigned int), hipMemcpyDeviceToHost, st) == hipSuccess &&
        hipStreamSynchronize(st) == hipSuccess)
      rc = (int)h_bad;
  }
  (void)hipFree(bad);
  return rc;
}

extern "C" int idn_bilateral_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                                int64_t row_stride, int d, double sigma_color, double sigma_space,
                                void* stream) {
  using namespace idn;
  if (int e = check_filter_args(src, dst, n, h, w, c, row_stride, "idn_bilateral_u8")) return e;
  IDN_CHECK_ARG(c == 1 || c == 3, "idn_bilateral_u8: channels must be 1 or 3 (got %d)", c);
  if (n == 0) return IDN_OK;
  if (sigma_color <= 0) sigma_color = 1;
  if (sigma_space <= 0) sigma_space = 1;
  int radius = d <= 0 ? (int)lrint(sigma_space * 1.5) : d / 2;
  if (radius < 1) radius = 1;
  if (radius > BL_MAXR)
    return set_error(IDN_EUNSUPPORTED, "idn_bilateral_u8: radius %d > %d", radius, BL_MAXR);
  const int64_t blocks = (int64_t)n * ((w + BL_TW - 1) / BL_TW) * ((h + BL_TH - 1) / BL_TH);
  IDN_CHECK_ARG(blocks < 0x7FFFFFFF, "idn_bilateral_u8: batch too large");

  BilateralTaps taps;
  memset(&taps, 0, sizeof(taps));
  const double gcc = -0.5 / (sigma_color * sigma_color);
  const double gsc = -0.5 / (sigma_space * sigma_space);
  taps.gcc = gcc;
  for (int i = -radius; i <= radius; ++i)
    for (int j = -radius; j <= radius; ++j) {
      const double r = sqrt((double)i * i + (double)j * j);
      if (r > radius) continue;
      taps.sw[(i + radius) * (2 * radius + 1) + (j + radius)] = (float)exp(r * r * gsc);  // OpenCV's
      taps.swq[i * i + j * j] = (float)exp(r * r * gsc);
      taps.ksq[i * i + j * j] = (float)log2((double)taps.swq[i * i + j * j]);
    }
  taps.kc = (float)(gcc * 1.4426950408889634);
  hipStream_t st = as_stream(stream);
#define IDN_BL(CC)                                                          \
  switch (radius) {                                                         \
    case 1: launch_bl<CC, 1>(src, dst, n, h, w, row_stride, taps, st); break; \
    case 2: launch_bl<CC, 2>(src, dst, n, h, w, row_stride, taps, st); break; \
    case 3: launch_bl<CC, 3>(src, dst, n, h, w, row_stride, taps, st); break; \
    case 4: launch_bl<CC, 4>(src, dst, n, h, w, row_stride, taps, st); break; \
    case 5: launch_bl<CC, 5>(src, dst, n, h, w, row_stride, taps, st); break; \
    case 6: launch_bl<CC, 6>(src, dst, n, h, w, row_stride, taps, st); break; \
    case 7: launch_bl<CC, 7>(src, dst, n, h, w, row_stride, taps, st); break; \
    default: launch_bl<CC, 8>(src, dst, n, h, w, row_stride, taps, st); break; \
  }
  if (c == 3 && radius <= 5 && w >= 2 && (int64_t)h * row_stride < 0x3FFFFFFF) {
    switch (radius) {
      case 1: launch_bl_pre<1>(src, dst, n, h, w, row_stride, taps, st); break;
      case 2: launch_bl_pre<2>(src, dst, n, h, w, row_stride, taps, st); break;
      case 3: launch_bl_pre<3>(src, dst, n, h, w, row_stride, taps, st); break;
      case 4: launch_bl_pre<4>(src, dst, n, h, w, row_stride, taps, st); break;
      default: launch_bl_pre<5>(src, dst, n, h, w, row_stride, taps, st); break;
    }
  } else if (c == 3) {
    IDN_BL(3)
  } else {
    IDN_BL(1)
  }
#undef IDN_BL
  IDN_CHECK_LAUNCH("idn_bilateral_u8");
  return IDN_OK;
}
