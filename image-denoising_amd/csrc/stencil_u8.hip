// Separable 8-bit stencils on interleaved HxWxC images for gfx950:
//   cv2.GaussianBlur(u8, (3,3)|(5,5), 0)   and   cv2.blur(u8, (3,3)),  BORDER_REFLECT_101.
//
// Reference call sites: lib/model/test.py:224,241,1767; lib/roi_data_layer/minibatch.py:119,136,
// 1636-1643.  OpenCV 3.4.2 semantics restated in oracle/filters.c.
//
// Fast path design (one wave = one independent work item, no LDS, no barriers):
//   * A row of RB = W*C bytes is cut into segments of <= 1008 output bytes.  A wave owns one
//     segment of one horizontal band of rows of one image and slides down the band.
//   * Lane l holds the 16-byte chunk [seg_start - 8 + 16 l, +16) of the current row, loaded with
//     one range-checked buffer_load_dwordx4.  The 2C-byte horizontal halo comes from the two
//     neighbouring lanes through DPP wave shifts (wave_shr:1 / wave_shl:1), so every byte of HBM
//     is loaded once per row.  Row/segment edges rebuild the reflected bytes in registers.
//   * Horizontal taps are formed with v_alignbyte_b32 and summed SWAR: even and odd bytes are
//     split into two u16 lanes per VGPR (x & 0x00FF00FF, (x >> 8) & 0x00FF00FF), so one 32-bit
//     add works on two pixels' channels.  Vertical taps come from a K-deep register ring of the
//     horizontal sums; the Gaussian weights are scaled so the rounded result lands in the high
//     byte of each u16 lane and one v_perm_b32 packs 4 output bytes.
//   * Loads are issued PF rows ahead (register queue), stores are whole dwordx4 per lane.
// Generic path (any C, any alignment): one thread per pixel, same arithmetic, used for shapes
// the fast path does not accept.
#include "stripe.hpp"

namespace idn {

enum StencilOp { OP_GAUSS3 = 0, OP_GAUSS5 = 1, OP_BOX3 = 2 };

template <int OP> struct Stencil;
template <> struct Stencil<OP_GAUSS3> { static constexpr int K = 3; };
template <> struct Stencil<OP_GAUSS5> { static constexpr int K = 5; };
template <> struct Stencil<OP_BOX3> { static constexpr int K = 3; };

// Horizontal pass: H[2k] / H[2k+1] = even / odd u16 lanes of output dword k (bytes 4k..4k+3).
template <int C, int OP>
__device__ __forceinline__ void hpass(const uint32_t (&W)[8], uint32_t (&H)[8]) {
  Lanes16 V;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    V.SE[j] = even_u16(W[j]);
    V.SO[j] = __builtin_amdgcn_perm(0u, W[j], 0x0C030C01u);  // (x >> 8) & 0x00FF00FF
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int P = 4 * k + 8 + e;  // window byte of output byte 4k+e
      uint32_t acc;
      if constexpr (OP == OP_GAUSS5) {
        // [1 4 6 4 1]: max 16*255 = 4080 per u16 lane
        const uint32_t c0 = V.at(P);
        acc = V.at(P - 2 * C) + V.at(P + 2 * C) + 4u * (V.at(P - C) + V.at(P + C)) +
              (c0 << 2) + (c0 << 1);
      } else if constexpr (OP == OP_GAUSS3) {
        // 4*[1 2 1]: max 4080
        acc = 4u * (V.at(P - C) + V.at(P + C)) + (V.at(P) << 3);
      } else {
        acc = V.at(P - C) + V.at(P) + V.at(P + C);  // max 765
      }
      H[2 * k + e] = acc;
    }
  }
}

// Vertical pass over the ring rows r0..r(K-1) -> 4 output dwords.
template <int OP>
__device__ __forceinline__ v4u vpass(const uint32_t* h0, const uint32_t* h1, const uint32_t* h2,
                                     const uint32_t* h3, const uint32_t* h4) {
  uint32_t o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t v[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int j = 2 * k + e;
      if constexpr (OP == OP_GAUSS5) {
        // sum of [1 4 6 4 1]^2 weights = 256; +128 rounds half up; result = high byte of lane
        const uint32_t a = h0[j] + h4[j] + 0x00800080u;
        const uint32_t b = h1[j] + h2[j] + h3[j];
        v[e] = (b << 2) + a + (h2[j] << 1);
      } else if constexpr (OP == OP_GAUSS3) {
        // 16 * ([1 2 1]^2 sum) -> (S + 8) >> 4 == (16 S + 128) >> 8
        v[e] = ((h0[j] + h2[j]) << 2) + (h1[j] << 3) + 0x00800080u;
      } else {
        // round(S / 9) == (S*455 + 2075) >> 12 for S in [0, 2295] (exhaustively checked)
        const uint32_t s = h0[j] + h1[j] + h2[j];
        const uint32_t lo = ((s & 0xFFFFu) * 455u + 2075u) >> 12;
        const uint32_t hi = ((s >> 16) * 455u + 2075u) >> 12;
        v[e] = lo | (hi << 16);
      }
    }
    if constexpr (OP == OP_BOX3) {
      o[k] = v[0] | (v[1] << 8);
    } else {
      o[k] = __builtin_amdgcn_perm(v[1], v[0], 0x07030501u);
    }
  }
  v4u r = {o[0], o[1], o[2], o[3]};
  return r;
}

template <int C, int OP, int PF, int NT>
__global__ __launch_bounds__(256) void stencil_u8_fast(const uint8_t* __restrict__ src,
                                                       uint8_t* __restrict__ dst, int h, int rb,
                                                       uint32_t row_stride, int nseg, int seg_len,
                                                       int bands, int band_rows, int total_items) {
  constexpr int K = Stencil<OP>::K;
  constexpr int R = K / 2;
  constexpr int U = (K == 5) ? 5 : 6;  // unroll = lcm(K, PF)
  static_assert(U % K == 0 && U % PF == 0, "unroll must cover ring and queue");
  static_assert(R * C <= 8, "one-side halo must fit in two neighbour dwords");

  const int lane = threadIdx.x & 63;
  const int item = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (item >= total_items) return;
  const StripeGeom g = stripe_geom(item, lane, rb, nseg, seg_len, bands);

  const uint32_t img_bytes = (uint32_t)h * row_stride;
  const rsrc_t rs = make_rsrc(src + (size_t)g.img * img_bytes, img_bytes);
  const rsrc_t rd = make_rsrc(dst + (size_t)g.img * img_bytes, img_bytes);
  const uint32_t ld_off = g.lead ? 0u : (uint32_t)g.q;

  const int y0 = g.band * band_rows;
  const int y1 = min(y0 + band_rows, h);
  if (y0 >= y1) return;
  const int nin = (y1 - y0) + 2 * R;  // input rows of the band incl. halo

  // Rows are processed in groups of U (static ring / queue slots).  The group count is rounded
  // up and out-of-band rows are clamped to the band's last input row, so every group runs the
  // same straight-line code (no phi copies of the ring); only the store is predicated.
  const int ngroups = (nin + U - 1) / U;
  auto load_row = [&](int r) -> v4u {
    const int y = reflect101(y0 - R + min(r, nin - 1), h);
    return __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)y * row_stride + ld_off, 0,
                                                  (NT & 1) ? 2 : 0);
  };

  v4u Lq[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) Lq[i] = load_row(i);

  uint32_t Hr[K][8];

  for (int gi = 0; gi < ngroups; ++gi) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = gi * U + u;
      const v4u Lv = Lq[u % PF];
      Lq[u % PF] = load_row(r + PF);
      uint32_t W[8];
      build_window<C, BORDER_REFLECT101>(Lv, g.lead, g.fix_t0, g.fix_t8, W);
      hpass<C, OP>(W, Hr[u % K]);
      const int y = y0 + r - 2 * R;
      if (r >= 2 * R && y < y1) {
        v4u o;
        if constexpr (K == 5) {
          o = vpass<OP>(Hr[(u + 1) % K], Hr[(u + 2) % K], Hr[(u + 3) % K], Hr[(u + 4) % K],
                        Hr[u % K]);
        } else {
          o = vpass<OP>(Hr[(u + 1) % K], Hr[(u + 2) % K], Hr[u % K], nullptr, nullptr);
        }
        stripe_store<NT>(o, rd, (uint32_t)y * row_stride + (uint32_t)g.q, g.kind);
      }
    }
  }
}

// ---- generic path ------------------------------------------------------------------------
template <int OP>
__global__ __launch_bounds__(256) void stencil_u8_generic(const uint8_t* __restrict__ src,
                                                          uint8_t* __restrict__ dst, int n, int h,
                                                          int w, int c, int64_t row_stride) {
  constexpr int K = Stencil<OP>::K;
  constexpr int R = K / 2;
  const int64_t npix = (int64_t)n * h * w;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npix;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(p % w);
    const int64_t t = p / w;
    const int y = (int)(t % h);
    const int img = (int)(t / h);
    const uint8_t* s = src + (int64_t)img * h * row_stride;
    uint8_t* d = dst + (int64_t)img * h * row_stride + (int64_t)y * row_stride + (int64_t)x * c;
    for (int ch = 0; ch < c; ++ch) {
      uint32_t S = 0;
#pragma unroll
      for (int i = -R; i <= R; ++i) {
        const uint8_t* sr = s + (int64_t)reflect101(y + i, h) * row_stride;
#pragma unroll
        for (int j = -R; j <= R; ++j) {
          uint32_t v = sr[(int64_t)reflect101(x + j, w) * c + ch];
          uint32_t wgt;
          if constexpr (OP == OP_GAUSS5) {
            constexpr uint32_t a[5] = {1, 4, 6, 4, 1};
            wgt = a[i + R] * a[j + R];
          } else if constexpr (OP == OP_GAUSS3) {
            constexpr uint32_t a[3] = {1, 2, 1};
            wgt = a[i + R] * a[j + R];
          } else {
            wgt = 1;
          }
          S += wgt * v;
        }
      }
      uint32_t out;
      if constexpr (OP == OP_GAUSS5) out = (S + 128) >> 8;
      else if constexpr (OP == OP_GAUSS3) out = (S + 8) >> 4;
      else out = (2 * S + 9) / 18;
      d[ch] = (uint8_t)out;
    }
  }
}

// ---- float64 path (the reference's quirk branches filter the float64 output of random_noise) ----
// cv2.GaussianBlur / cv2.blur on CV_64F: separable double filter, BORDER_REFLECT_101, no rounding.
template <int OP>
__device__ __forceinline__ double f64_tap(int i) {
  if constexpr (OP == OP_GAUSS5) {
    constexpr double a[5] = {0.0625, 0.25, 0.375, 0.25, 0.0625};
    return a[i];
  } else if constexpr (OP == OP_GAUSS3) {
    constexpr double a[3] = {0.25, 0.5, 0.25};
    return a[i];
  } else {
    return 1.0;
  }
}

// Summation order follows OpenCV's 64F engines so results agree to the last ulp for the Gaussian:
// RowFilter<double> sums taps left to right; SymmColumnFilter<double> forms
// ky0*c + ky1*(r+1 + r-1) + ky2*(r+2 + r-2).  cv2.blur's 64F path uses running row/column sums
// (RowSum/ColumnSum), which this direct 3x3 sum matches only to a few ulp.
template <int OP>
__global__ __launch_bounds__(256) void stencil_f64(const double* __restrict__ src,
                                                   double* __restrict__ dst, int n, int h, int w,
                                                   int c) {
  constexpr int K = Stencil<OP>::K;
  constexpr int R = K / 2;
  const int64_t total = (int64_t)n * h * w * c;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int ch = (int)(e % c);
    int64_t t = e / c;
    const int x = (int)(t % w);
    t /= w;
    const int y = (int)(t % h);
    const int img = (int)(t / h);
    const double* s = src + (int64_t)img * h * w * c;
    double rs[K];
#pragma unroll
    for (int i = -R; i <= R; ++i) {
      const double* row = s + (int64_t)reflect101(y + i, h) * w * c;
      double racc = f64_tap<OP>(0) * row[(int64_t)reflect101(x - R, w) * c + ch];
#pragma unroll
      for (int j = -R + 1; j <= R; ++j)
        racc = __dadd_rn(racc, __dmul_rn(f64_tap<OP>(j + R), row[(int64_t)reflect101(x + j, w) * c + ch]));
      rs[i + R] = racc;
    }
    double acc;
    if constexpr (OP == OP_BOX3) {
      acc = __dadd_rn(__dadd_rn(rs[0], rs[1]), rs[2]) * (1.0 / 9.0);
    } else {
      acc = __dmul_rn(f64_tap<OP>(R), rs[R]);
#pragma unroll
      for (int k = 1; k <= R; ++k)
        acc = __dadd_rn(acc, __dmul_rn(f64_tap<OP>(R + k), __dadd_rn(rs[R + k], rs[R - k])));
    }
    dst[e] = acc;
  }
}

template <int OP>
static int launch_f64(const double* src, double* dst, int n, int h, int w, int c, hipStream_t st,
                      const char* name) {
  const int64_t total = (int64_t)n * h * w * c;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL((stencil_f64<OP>), dim3((unsigned)blocks), dim3(256), 0, st, src, dst, n, h, w, c);
  IDN_CHECK_LAUNCH(name);
  return IDN_OK;
}

// ---- host launchers --------------------------------------------------------------------------
template <int OP>
static int launch_stencil(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                          int64_t row_stride, hipStream_t st, const char* name) {
  const int64_t rb = (int64_t)w * c;
  if (stripe_ok(c, rb, row_stride, h, src, dst)) {
    constexpr int K = Stencil<OP>::K;
    constexpr int U = (K == 5) ? 5 : 6;
    constexpr int PF = (K == 5) ? 5 : 6;
    // one resident round: 5 waves/SIMD x 1024 SIMDs at <= 96 VGPRs
    const StripePlan p = plan_stripe(n, h, rb, K, U, 5120);
    IDN_CHECK_ARG(p.total < (int64_t)0x7FFFFFFF, "%s: batch too large", name);
    const dim3 grid((unsigned)((p.total + 3) / 4)), block(256);
    const int nt = env_int("IDN_STENCIL_NT", 0) & 3;
#define IDN_LAUNCH_FAST(NTV)                                                                     \
  hipLaunchKernelGGL((stencil_u8_fast<3, OP, PF, NTV>), grid, block, 0, st, src, dst, h, (int)rb, \
                     (uint32_t)row_stride, p.nseg, p.seg_len, p.bands, p.band_rows, (int)p.total)
    switch (nt) {
      case 1: IDN_LAUNCH_FAST(1); break;
      case 2: IDN_LAUNCH_FAST(2); break;
      case 3: IDN_LAUNCH_FAST(3); break;
      default: IDN_LAUNCH_FAST(0); break;
    }
#undef IDN_LAUNCH_FAST
  } else {
    const int64_t npix = (int64_t)n * h * w;
    int64_t blocks = (npix + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL((stencil_u8_generic<OP>), dim3((unsigned)blocks), dim3(256), 0, st, src,
                       dst, n, h, w, c, row_stride);
  }
  IDN_CHECK_LAUNCH(name);
  return IDN_OK;
}

int check_filter_args(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                        int64_t row_stride, const char* name) {
  IDN_CHECK_ARG(src && dst, "%s: null pointer", name);
  IDN_CHECK_ARG(src != dst, "%s: in-place filtering is not supported (src == dst)", name);
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0, "%s: bad shape n=%d h=%d w=%d", name, n, h, w);
  IDN_CHECK_ARG(c >= 1 && c <= 4, "%s: channels must be 1..4 (got %d)", name, c);
  IDN_CHECK_ARG(row_stride >= (int64_t)w * c, "%s: row_stride %lld < w*c", name,
                (long long)row_stride);
  return IDN_OK;
}

}  // namespace idn

extern "C" int idn_gaussian_blur_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                                    int64_t row_stride, int ksize, void* stream) {
  using namespace idn;
  if (int e = check_filter_args(src, dst, n, h, w, c, row_stride, "idn_gaussian_blur_u8")) return e;
  if (n == 0) return IDN_OK;
  if (ksize == 3)
    return launch_stencil<OP_GAUSS3>(src, dst, n, h, w, c, row_stride, as_stream(stream),
                                     "idn_gaussian_blur_u8");
  if (ksize == 5)
    return launch_stencil<OP_GAUSS5>(src, dst, n, h, w, c, row_stride, as_stream(stream),
                                     "idn_gaussian_blur_u8");
  return set_error(IDN_EUNSUPPORTED, "idn_gaussian_blur_u8: ksize %d not supported (3 or 5)",
                   ksize);
}

extern "C" int idn_box_blur_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                               int64_t row_stride, int ksize, void* stream) {
  using namespace idn;
  if (int e = check_filter_args(src, dst, n, h, w, c, row_stride, "idn_box_blur_u8")) return e;
  if (n == 0) return IDN_OK;
  if (ksize == 3)
    return launch_stencil<OP_BOX3>(src, dst, n, h, w, c, row_stride, as_stream(stream),
                                   "idn_box_blur_u8");
  return set_error(IDN_EUNSUPPORTED, "idn_box_blur_u8: ksize %d not supported (3)", ksize);
}

extern "C" int idn_gaussian_blur_f64(const double* src, double* dst, int n, int h, int w, int c,
                                     int ksize, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(src && dst && src != dst, "idn_gaussian_blur_f64: bad pointers");
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0 && c >= 1 && c <= 4, "idn_gaussian_blur_f64: bad shape");
  if (n == 0) return IDN_OK;
  if (ksize == 3) return launch_f64<OP_GAUSS3>(src, dst, n, h, w, c, as_stream(stream), "idn_gaussian_blur_f64");
  if (ksize == 5) return launch_f64<OP_GAUSS5>(src, dst, n, h, w, c, as_stream(stream), "idn_gaussian_blur_f64");
  return set_error(IDN_EUNSUPPORTED, "idn_gaussian_blur_f64: ksize %d not supported", ksize);
}

extern "C" int idn_box_blur_f64(const double* src, double* dst, int n, int h, int w, int c,
                                int ksize, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(src && dst && src != dst, "idn_box_blur_f64: bad pointers");
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0 && c >= 1 && c <= 4, "idn_box_blur_f64: bad shape");
  if (n == 0) return IDN_OK;
  if (ksize == 3) return launch_f64<OP_BOX3>(src, dst, n, h, w, c, as_stream(stream), "idn_box_blur_f64");
  return set_error(IDN_EUNSUPPORTED, "idn_box_blur_f64: ksize %d not supported", ksize);
}
