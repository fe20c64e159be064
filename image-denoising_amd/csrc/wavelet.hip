// Wavelet denoiser: skimage 0.14.2 denoise_wavelet(img, method='BayesShrink', mode='soft',
// wavelet=db1|bior1.5, multichannel=True, convert2ycbcr=True, wavelet_levels=L) followed by the
// caller's (255 * out).astype(np.uint8).
// Reference call sites: lib/model/test.py:197-201,1807-1810, lib/roi_data_layer/minibatch.py:
// 1653-1656, minibatch_before_curvelet.py:85-87.  Restated in numpy in oracle/wavelet.py (pinned
// against pywt 1.1.1 / skimage 0.18.3 fixtures).
//
// Pipeline per image (all images of the batch in every launch; grid.z = image x channel):
//   1 wl_color_minmax  per-channel fp64 min / max of the YCbCr image (BGR data treated as RGB,
//                   as the reference does); the YCbCr planes are never stored
//   2 wl_dwt  x L   one separable 2-D analysis level per launch: a 256-thread workgroup stages a
//                   (2T+F-2)^2 input tile in LDS (pywt 'symmetric' extension), filters rows, then
//                   columns, and writes the aa / ad / da / dd bands plus the tile's sums of squares
//                   of the three detail bands.  Level 1 stages straight from the u8 (or f64) image:
//                   YCbCr channel + (x - min) / (max - min) normalisation on the fly.
//   3 wl_sumsq      per detail band: add the tile partials in tile order (deterministic)
//   4 wl_median     sigma = median(|finest dd| != 0) / 0.6744897501960817: exact radix select on
//                   the float bits (two 11-bit passes over the band, compaction of the selected
//                   prefix into the consumed input plane, four passes over that), + one pass for
//                   the upper middle rank
//   5 wl_thresh     BayesShrink t = var / sqrt(max(mean(d^2) - var, eps)) per band
//   6 wl_idwt x L-1 synthesis levels L..2 (stage-2 valid convolution of pywt's
//                   upsampling_convolution_valid_sf) with the soft threshold d*max(1-t/|d|, 0)
//                   applied to every detail read; output cropped to the next level's size
//   7 wl_idwt_final level 1 for all three channels of a pixel at once, fused with clip [0,1],
//                   de-normalisation, YCbCr -> RGB, clip [0,1] and the U8 cast
// Storage and arithmetic are fp64 (`wreal`): the BayesShrink threshold var/sqrt(mean(d^2) - var)
// is ill-conditioned when a band is noise dominated, so fp32 bands moved outputs by up to 5e-5.
// The analysis filters multiply then add (no FMA), as pywt's C loop does: a detail coefficient of
// two equal samples is then exactly 0 (-S*x + S*x), which the "nonzero" median relies on.
#include "idn_common.hpp"

#include <cmath>
#include <mutex>
#include <type_traits>

#include <math.h>

#include <algorithm>

#include "ycc.hpp"

namespace idn {

using wreal = double;  // workspace / arithmetic type of the transform
constexpr wreal S2 = 0.7071067811865476;
constexpr wreal B1 = 0.016572815184059706;
constexpr wreal B2 = 0.12153397801643785;

// fused multiply-add in the arithmetic type T (the build has -ffp-contract=off: no implicit fma)
template <typename T>
__device__ __forceinline__ T fma_t(T a, T b, T c) {
  if constexpr (sizeof(T) == 4) return __fmaf_rn(a, b, c);
  else return __fma_rn(a, b, c);
}

template <int WV> struct Wav;
template <> struct Wav<IDN_WAVELET_DB1> {
  static constexpr int F = 2;
  static constexpr wreal dlo[2] = {S2, S2};
  static constexpr wreal dhi[2] = {-S2, S2};
  static constexpr wreal rlo[2] = {S2, S2};
  static constexpr wreal rhi[2] = {S2, -S2};
};
template <> struct Wav<IDN_WAVELET_BIOR15> {
  static constexpr int F = 10;
  static constexpr wreal dlo[10] = {B1, -B1, -B2, B2, S2, S2, B2, -B2, -B1, B1};
  static constexpr wreal dhi[10] = {0, 0, 0, 0, -S2, S2, 0, 0, 0, 0};
  static constexpr wreal rlo[10] = {0, 0, 0, 0, S2, S2, 0, 0, 0, 0};
  static constexpr wreal rhi[10] = {B1, B1, -B2, -B2, S2, -S2, B2, B2, -B1, -B1};
};

inline int wl_filter_len(int wv) { return wv == IDN_WAVELET_DB1 ? 2 : 10; }

// pywt dwt_max_level: floor(log2(n / (F - 1))) with integer division, 0 if n < F - 1
inline int wl_max_level(int n, int F) {
  if (F <= 1 || n < F - 1) return 0;
  int q = n / (F - 1), l = 0;
  while (q > 1) {
    q >>= 1;
    ++l;
  }
  return l;
}

constexpr int WL_MAXL = 12;
constexpr int RB_TY = 8, RB_TX = 32, RB_R = 4;  // analysis tile (wl_dwt_rb)
constexpr int WL_STATS = 256;  // doubles of per-image stats
constexpr int WL_N32U = 156;   // stats [156, 159): u32 counts of the N32 analysis' uncertain codes

struct WlLayout {
  int n, h, w, F, L;
  int H[WL_MAXL + 1], W[WL_MAXL + 1];  // H[0] = h; H[l] = band height of level l
  size_t off_band[WL_MAXL + 1];        // element offset of level l's 3x4 bands inside an image
  size_t img_floats;                   // wreal elements per image (planes + bands)
  size_t stats_off;                    // byte offset of the stats region (after all images)
  int tiles_x[WL_MAXL + 1], tiles[WL_MAXL + 1];  // DWT tiles per level (partial-sum slots)
  int bands[WL_MAXL + 1];              // bior1.5 streaming analysis: row bands per strip
  double sq_grid[WL_MAXL + 1];         // ... and the grid its sum-of-squares partials round to
  size_t part_tile0[WL_MAXL + 1];      // first tile index of level l in the partials array
  size_t part_per_img;                 // partial sums per image: 3 channels x 3 bands x tiles
  size_t part_off;                     // byte offset of the partial sums region
  size_t bytes;
};

// stats region per image (doubles): [0..6) min/max as u32 pairs, [8..) sumsq[3][L][3],
// [8+9L..) median[3], thr as double[3][L][3] after that, [255] degenerate flag
struct WlStats {
  __host__ __device__ static int sumsq(int c, int l, int b, int L) { return 8 + (c * L + l) * 3 + b; }
  __host__ __device__ static int median(int c, int L) { return 8 + 9 * L + c; }
  __host__ __device__ static int thr(int c, int l, int b, int L) { return 8 + 9 * L + 3 + (c * L + l) * 3 + b; }
  // half thresholds for the integer Haar synthesis (written for L <= 3 only: [170, 197))
  __host__ __device__ static int thrh(int c, int l, int b) { return 170 + (c * 3 + l) * 3 + b; }
  static constexpr int FLAG = 255;
  static constexpr int DIAG = 248;  // [248..251) nonzero count of the finest dd per channel
  static constexpr int MN64 = 200;  // [200..203) fp64 channel min (u64 bits), [203..206) max
  static constexpr int MX64 = 203;
};
constexpr int WL_EBINS = 64;  // exponent bins of |dd|: bin = clamp(exponent - (1023 - 61), 0, 63)
__device__ __forceinline__ int wl_ebin(unsigned long long key) {
  const int e = (int)(key >> 52) - (1023 - 61);
  return e < 0 ? 0 : (e > WL_EBINS - 1 ? WL_EBINS - 1 : e);
}

// fine bins of |dd| keys: exponent (clamped as wl_ebin) and the top 4 mantissa bits, monotone in
// the key; the clamped exponent bins keep one sub-bin
constexpr int WL_FBINS = WL_EBINS * 16;
__device__ __forceinline__ unsigned long long absbits(double v) {
  return (unsigned long long)__double_as_longlong(v) & 0x7FFFFFFFFFFFFFFFull;
}
__device__ __forceinline__ int wl_fbin(unsigned long long key) {
  const int e = (int)(key >> 52) - (1023 - 61);
  if (e < 0) return 0;
  if (e > WL_EBINS - 1) return WL_FBINS - 1;
  return e * 16 + (int)((key >> 48) & 15u);
}

inline int ws_strips(int Wo);
inline int ws_sw(int Wo);
inline int ws_bands(int n, int Ho, int Wo, int strips, int level);
// rows per sum-of-squares group of the streaming analysis: 5, the step loop's unroll, so a group
// ends at the same static position of every unrolled iteration (no per-row test or branch)
constexpr int WS_G = 5;
// Row bands per strip so that the grid fills whole rounds of resident workgroups: for each
// candidate band count b the time is ~ rounds(b) x (rows per band + warm-up rows), rounds(b) =
// ceil(units * b / resident).  (A grid of 2.5 rounds leaves the chip half idle for the last one.)
inline int best_bands(int64_t units, int M, int warm, int64_t resident, int min_rows) {
  const int bmax = std::max(1, std::min(64, M / std::max(min_rows, 1)));
  int best = 1;
  double bestc = 1e300;
  for (int b = 1; b <= bmax; ++b) {
    const double rounds = std::ceil((double)(units * b) / (double)std::max<int64_t>(resident, 1));
    const double c = rounds * ((M + b - 1) / b + warm);
    if (c < bestc * 0.999) {
      bestc = c;
      best = b;
    }
  }
  return best;
}
// resident workgroups per CU of a kernel at a block size (cached; 1 if the query fails)
inline int occ_wgs(const void* kernel, int block) {
  static std::mutex mu;
  static const void* keys[32];
  static int blocks[32], vals[32], nk = 0;
  std::lock_guard<std::mutex> g(mu);
  for (int i = 0; i < nk; ++i)
    if (keys[i] == kernel && blocks[i] == block) return vals[i];
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, block, 0) != hipSuccess || nb < 1)
    nb = 1;
  if (nk < 32) {
    keys[nk] = kernel;
    blocks[nk] = block;
    vals[nk++] = nb;
  }
  return nb;
}
inline WlLayout wl_layout(int n, int h, int w, int wv, int levels) {
  WlLayout Lt;
  Lt.n = n;
  Lt.h = h;
  Lt.w = w;
  Lt.F = wl_filter_len(wv);
  if (levels <= 0) {
    const int ml = std::min(wl_max_level(h, Lt.F), wl_max_level(w, Lt.F));
    levels = std::max(ml - 3, 1);
  }
  Lt.L = levels;
  Lt.H[0] = h;
  Lt.W[0] = w;
  size_t off = (size_t)3 * h * w;
  for (int l = 1; l <= Lt.L && l <= WL_MAXL; ++l) {
    Lt.H[l] = (Lt.H[l - 1] + Lt.F - 1) / 2;
    Lt.W[l] = (Lt.W[l - 1] + Lt.F - 1) / 2;
    Lt.off_band[l] = off;
    off += (size_t)12 * Lt.H[l] * Lt.W[l];
  }
  Lt.img_floats = (off + 63) / 64 * 64;
  Lt.stats_off = (size_t)n * Lt.img_floats * sizeof(wreal);
  size_t tiles_tot = 0;
  for (int l = 1; l <= Lt.L && l <= WL_MAXL; ++l) {
    if (wv == IDN_WAVELET_BIOR15) {
      // wl_dwt_stream: strips x row bands of whole WS_G-row groups (the bands' sums are exact,
      // see the kernel).  sq_grid: 2^-F with the band's total below 2^(52 - F) for any input.
      // With the filters' L1 norms Llo = 4 B1 + 4 B2 + 2 S2 (~1.967) and Lhi = 2 S2 (~1.414),
      // level-l data of a [0, 1] image lie within Llo^(2(l-1)) (the 'aa' chain) and a detail
      // coefficient within Llo * Lhi times that, so a square <= (Llo Lhi)^2 Llo^(4(l-1))
      const int groups = (Lt.H[l] + WS_G - 1) / WS_G;
      Lt.tiles_x[l] = ws_strips(Lt.W[l]);
      Lt.bands[l] = std::min(ws_bands(n, Lt.H[l], Lt.W[l], Lt.tiles_x[l], l), groups);
      // tuning: a fixed band count per level (bit field: level l's count in bits 8(l-1)..)
      if (const int fb = (knob("IDN_WAVELET_BANDS", 0) >> (8 * (l - 1))) & 0xFF)
        Lt.bands[l] = std::min(fb, groups);
      Lt.tiles[l] = Lt.tiles_x[l] * Lt.bands[l];
      const double llo = 4.0 * B1 + 4.0 * B2 + 2.0 * S2, lhi = 2.0 * S2;
      const double bound = (llo * lhi) * (llo * lhi) * std::pow(llo, 4.0 * (l - 1)) *
                           (double)Lt.H[l] * (double)Lt.W[l];
      Lt.sq_grid[l] = std::ldexp(1.0, (int)std::ceil(std::log2(bound)) - 52);
    } else {
      Lt.bands[l] = 0;
      Lt.tiles_x[l] = (Lt.W[l] + RB_TX - 1) / RB_TX;  // wl_dwt_rb tiles
      Lt.tiles[l] = Lt.tiles_x[l] * ((Lt.H[l] + RB_TY - 1) / RB_TY);
    }
    Lt.part_tile0[l] = tiles_tot;
    tiles_tot += (size_t)Lt.tiles[l];
  }
  if (wv == IDN_WAVELET_DB1 && Lt.L <= 3 && h % (1 << Lt.L) == 0 && w % (1 << Lt.L) == 0) {
    // the fused Haar path's partials: one per workgroup of 128 threads and level
    const size_t ns = Lt.L == 3 ? 4 : 1;
    const size_t nwg = ((size_t)(h >> Lt.L) * (size_t)(w >> Lt.L) * ns + 127) / 128;
    tiles_tot = std::max(tiles_tot, (size_t)Lt.L * nwg);
  }
  Lt.part_per_img = 9 * tiles_tot;  // [c][b][tile]
  Lt.part_off = Lt.stats_off + (size_t)n * WL_STATS * sizeof(double);
  Lt.bytes = Lt.part_off + (size_t)n * Lt.part_per_img * sizeof(double);
  return Lt;
}

__device__ __forceinline__ int sym_idx(int i, int n) {  // pywt 'symmetric' (half-sample)
  if ((unsigned)i < (unsigned)n) return i;  // interior: no division
  const int period = 2 * n;
  i %= period;
  if (i < 0) i += period;
  return i < n ? i : period - 1 - i;
}

// ---- 1: colour transform + min / max -----------------------------------------------------------
// ycc_keys (nullable): the colour range already reduced by the float64 noise kernel that wrote the
// input (idn_noise_ycc_u8), per image min keys of Y Cb Cr then max keys -- copied in, and
// wl_color_minmax does not run
__global__ void wl_init_stats(double* stats, int n, const unsigned long long* ycc_keys = nullptr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * WL_STATS) return;
  const int k = i % WL_STATS, img = i / WL_STATS;
  if (k >= WlStats::MN64 && k < WlStats::MN64 + 3) {
    reinterpret_cast<unsigned long long*>(stats)[i] =
        ycc_keys ? ycc_keys[6 * img + (k - WlStats::MN64)] : ~0ull;  // min key
  } else if (k >= WlStats::MX64 && k < WlStats::MX64 + 3) {
    reinterpret_cast<unsigned long long*>(stats)[i] =
        ycc_keys ? ycc_keys[6 * img + 3 + (k - WlStats::MX64)] : 0ull;  // max key
  } else {
    stats[i] = 0.0;
  }
}

__device__ __forceinline__ void ycbcr64(double x0, double x1, double x2, double (&o)[3]) {
  o[0] = __dadd_rn(dot3(x0, x1, x2, 65.481, 128.553, 24.966), 16.0);
  o[1] = __dadd_rn(dot3(x0, x1, x2, -37.797, -74.203, 112.0), 128.0);
  o[2] = __dadd_rn(dot3(x0, x1, x2, 112.0, -93.786, -18.214), 128.0);
}

__device__ __forceinline__ void load_rgb64(const uint8_t* __restrict__ src,
                                           const double* __restrict__ in64, int img, int h, int w,
                                           int64_t row_stride, int y, int x, double (&v)[3]) {
  if (in64) {
    const double* s = in64 + (((int64_t)img * h + y) * w + x) * 3;
    v[0] = s[0];
    v[1] = s[1];
    v[2] = s[2];
  } else {
    const uint8_t* s = src + (int64_t)img * h * row_stride + (int64_t)y * row_stride + (int64_t)x * 3;
    v[0] = (double)s[0] * (1.0 / 255.0);
    v[1] = (double)s[1] * (1.0 / 255.0);
    v[2] = (double)s[2] * (1.0 / 255.0);
  }
}

__device__ __forceinline__ void wl_minmax64(const double* st, int c, double& mn, double& mx) {
  const unsigned long long* u64 = reinterpret_cast<const unsigned long long*>(st);
  mn = dkey_inv(u64[WlStats::MN64 + c]);
  mx = dkey_inv(u64[WlStats::MX64 + c]);
}

// per-channel min / max of the YCbCr image (fp64 exact); the planes themselves are never
// stored: the analysis recomputes Y/Cb/Cr while staging.  Compact u8 rows (row_stride == 3w,
// dword-aligned) take 4 pixels per thread with three dword loads and no index division.
__global__ __launch_bounds__(256) void wl_color_minmax(const uint8_t* __restrict__ src,
                                                       const double* __restrict__ in64, int h, int w,
                                                       int64_t row_stride, double* __restrict__ stats) {
  const int img = blockIdx.y;
  const int64_t np = (int64_t)h * w;
  // the dot products only: x -> round(x + k) is monotone, so the min / max of ycbcr64's rounded
  // sums is the rounded sum of the dot products' min / max -- the offsets are added once per
  // wave after the reduction (bit-identical, three fp64 adds per pixel fewer)
  double dmn[3] = {INFINITY, INFINITY, INFINITY}, dmx[3] = {-INFINITY, -INFINITY, -INFINITY};
  auto acc = [&](double v0, double v1, double v2) {
    const double yc[3] = {dot3(v0, v1, v2, 65.481, 128.553, 24.966),
                          dot3(v0, v1, v2, -37.797, -74.203, 112.0),
                          dot3(v0, v1, v2, 112.0, -93.786, -18.214)};
#pragma unroll
    for (int c = 0; c < 3; ++c) {  // inputs are finite: fmin / fmax are plain selects
      dmn[c] = fmin(dmn[c], yc[c]);
      dmx[c] = fmax(dmx[c], yc[c]);
    }
  };
  const bool flat = !in64 && row_stride == (int64_t)w * 3 && (np & 3) == 0 &&
                    (((uintptr_t)src & 3) == 0);
  if (flat) {
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src + (int64_t)img * h * row_stride);
    const int nq = (int)(np >> 2);  // groups of 4 pixels = 3 dwords
    const int stride = gridDim.x * blockDim.x;
    for (int q0 = blockIdx.x * blockDim.x + threadIdx.x; q0 < nq; q0 += 4 * stride) {
      uint32_t d[4][3];  // 4 groups in flight per thread
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = q0 + u * stride;
#pragma unroll
        for (int j = 0; j < 3; ++j) d[u][j] = q < nq ? s4[3 * q + j] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (q0 + u * stride >= nq) break;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          double v[3];
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const int k = 3 * p + c;
            v[c] = (double)((d[u][k >> 2] >> (8 * (k & 3))) & 0xFFu) * (1.0 / 255.0);
          }
          acc(v[0], v[1], v[2]);
        }
      }
    }
  } else {
    // pixel p = y * w + x with 32-bit index math (p < 2^31 per image: checked on the host)
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < (int)np; p += gridDim.x * blockDim.x) {
      const int y = p / w, x = p - y * w;
      double v[3];
      load_rgb64(src, in64, img, h, w, row_stride, y, x, v);
      acc(v[0], v[1], v[2]);
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double da = dmn[c], db = dmx[c];
    for (int o = 32; o > 0; o >>= 1) {
      da = fmin(da, __shfl_xor(da, o));
      db = fmax(db, __shfl_xor(db, o));
    }
    if ((threadIdx.x & 63) == 0 && da <= db) {
      const double off = c == 0 ? 16.0 : 128.0;  // ycbcr64's offsets
      atomicMinD(stats + (size_t)img * WL_STATS + WlStats::MN64 + c, __dadd_rn(da, off));
      atomicMaxD(stats + (size_t)img * WL_STATS + WlStats::MX64 + c, __dadd_rn(db, off));
    }
  }
}

// ---- 2: one analysis level ----------------------------------------------------------------------

// channel c of skimage rgb2ycbcr for one pixel (same fma chain as ycbcr64)
__device__ __forceinline__ double ycbcr_c(const double (&v)[3], int c) {
  if (c == 0) return __dadd_rn(dot3(v[0], v[1], v[2], 65.481, 128.553, 24.966), 16.0);
  if (c == 1) return __dadd_rn(dot3(v[0], v[1], v[2], -37.797, -74.203, 112.0), 128.0);
  return __dadd_rn(dot3(v[0], v[1], v[2], 112.0, -93.786, -18.214), 128.0);
}

// Register-blocked analysis tile: RB_TY x RB_TX output coefficients per band, all three channels
// in one 256-thread workgroup.
//   axis 0: thread (c, q) owns staged input column q of channel c (3 x NX threads); it loads the
//           NY input samples of its column (u8 / f64 pixels normalised on the fly, or the level
//           above's 'aa' plane), all loads in flight at once, and runs the F-tap lowpass and
//           highpass down the column in registers into S.vl / S.vh.
//   axis 1: thread (c, ii, group) computes R consecutive output columns of all four bands from
//           2R + F - 2 staged values of S.vl and S.vh (wave w = channel w).
//   the four bands go out through LDS (reusing vl / vh) as whole rows, so each wave's stores are
//   contiguous (register-blocked lanes stored 8-byte pieces at a 32-byte stride: 4x the L2 write
//   requests).
// LDS traffic is ~10 accesses per input pixel (round 1's per-output gathers: ~42).
template <int WV>
struct DwtRB {
  static constexpr int F = Wav<WV>::F;
  static constexpr int NX = 2 * RB_TX + F - 2;  // staged input columns
  static constexpr int NY = 2 * RB_TY + F - 2;  // input rows per column
  // row stride: odd (the 8 rows of a 32-lane read fall on distinct banks) and large enough for
  // vl + vh to hold the band staging buffer
  static constexpr int NXP = (NX + 1 > 2 * (RB_TX + 1) ? NX + 1 : 2 * (RB_TX + 1)) | 1;
  wreal vl[3][RB_TY][NXP], vh[3][RB_TY][NXP];
};
static_assert(3 * RB_TY * (RB_TX / RB_R) == 192, "axis-1 items: one per thread of waves 0-2");
constexpr int RB_OBS = RB_TX + 1;  // band staging row stride (doubles): conflict-free b64 stores


// fp32 band storage (IDN_WAVELET_FDET, default on): bands that only the synthesis (or the next
// analysis) reads round-trip through HBM as fp32 (relative 6e-8; the thresholds come from the fp64
// sums of squares taken before the store).  Band mask fmask: bit b (0 aa, 1 ad, 2 da, 3 dd) = band
// b of the level is fp32, bit 4 = the analysis's input 'aa' (level above) is fp32.
//   level 1: ad, da (dd stays fp64 for the sigma median's exact keys), aa when L > 1;
//   levels >= 2: ad, da, dd, aa when l < L (the coarsest 'aa' and the synthesis's reconstructions
//   in the 'aa' slots stay fp64)
constexpr int WL_FB_AIN = 16;
__host__ __device__ __forceinline__ bool wl_fband(int fmask, int b) { return (fmask >> b) & 1; }

// SRC: 0 = u8 image, 1 = f64 image (level 1, normalised per channel), 2 = the 'aa' planes of the
// level above (levels >= 2; wl_dwt_stream: 2 fp64, 3 fp32).  Grid (tiles, 1, n).
template <int WV, int SRC>
__global__ __launch_bounds__(256) void wl_dwt_rb(wreal* __restrict__ ws, size_t img_floats,
                                                 const double* __restrict__ stats, size_t in_off,
                                                 int Hin, int Win, size_t out_off, int Ho, int Wo,
                                                 int tiles_x, const uint8_t* __restrict__ src,
                                                 const double* __restrict__ in64,
                                                 int64_t row_stride, double* __restrict__ part,
                                                 size_t part_per_img, size_t part_tile0,
                                                 int emit_codes, int fmask, int coop) {
  using Wv = Wav<WV>;
  constexpr int F = Wv::F, NX = DwtRB<WV>::NX, NY = DwtRB<WV>::NY;
  __shared__ DwtRB<WV> S;
  const int img = blockIdx.z;
  wreal* base = ws + img * img_floats;
  const int ti = blockIdx.x / tiles_x, tj = blockIdx.x - ti * tiles_x;
  const int i0 = ti * RB_TY, j0 = tj * RB_TX;
  const int r0 = 2 * i0 + 2 - F, q0 = 2 * j0 + 2 - F;  // input coordinate of staged [0][0]
  const int t = threadIdx.x;
  wreal x[NY];
  // u8 input, cooperative form (IDN_WAVELET_COOP, default on): every staged pixel is loaded and
  // normalised once for its three channels by one of the 256 threads, through LDS in two halves
  // of rows (aliasing vl / vh), instead of once per channel by the three (channel, column)
  // threads -- the same fp64 operations per sample, a third of the u8 -> fp64 conversions
  const bool coop_u8 = SRC == 0 && coop;
  if (coop_u8) {
    constexpr int HR = NY / 2;  // NY = 2 RB_TY + F - 2 is even
    constexpr int IT = (HR * NX + 255) / 256;
    static_assert(sizeof(S) >= sizeof(wreal) * 3 * HR * NX, "normalised half fits in vl + vh");
    wreal(*nz)[HR][NX] = reinterpret_cast<wreal(*)[HR][NX]>(&S.vl[0][0][0]);
    const double* st = stats + (size_t)img * WL_STATS;
    wreal mn[3], inv[3], rcp[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      wreal mx;
      wl_minmax64(st, c, mn[c], mx);
      inv[c] = mx - mn[c];
      rcp[c] = 1.0 / inv[c];
    }
    const uint8_t* im = src + (int64_t)img * Hin * row_stride;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      uint32_t raw[IT];
#pragma unroll
      for (int it = 0; it < IT; ++it) {  // all loads in flight before any use
        const int k = t + 256 * it, rr = k / NX, q = k - rr * NX;
        raw[it] = 0;
        if (k < HR * NX) {
          const uint8_t* p = im + (int64_t)sym_idx(r0 + hf * HR + rr, Hin) * row_stride +
                             (int64_t)sym_idx(q0 + q, Win) * 3;
          raw[it] = (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16;
        }
      }
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int k = t + 256 * it, rr = k / NX, q = k - rr * NX;
        if (k < HR * NX) {
          double px[3];
#pragma unroll
          for (int kk = 0; kk < 3; ++kk)
            px[kk] = (double)((raw[it] >> (8 * kk)) & 0xFFu) * (1.0 / 255.0);
#pragma unroll
          for (int c = 0; c < 3; ++c) {  // as the per-channel form below, op for op
            const wreal a = ycbcr_c(px, c) - mn[c];
            const wreal qq = a * rcp[c];
            nz[c][rr][q] = __fma_rn(__fma_rn(-qq, inv[c], a), rcp[c], qq);
          }
        }
      }
      __syncthreads();
      if (t < 3 * NX) {
        const int c = t / NX, q = t - c * NX;
#pragma unroll
        for (int rr = 0; rr < HR; ++rr) x[hf * HR + rr] = nz[c][rr][q];
      }
      __syncthreads();  // nz is rewritten by the next half / becomes vl / vh
    }
  }
  if (t < 3 * NX) {
    const int c = t / NX, q = t - c * NX;
    const int xx = sym_idx(q0 + q, Win);
    if (coop_u8) {
      // x holds the column already
    } else if (SRC == 2) {
      if (fmask & WL_FB_AIN) {  // the level above stored its 'aa' as fp32
        const float* X = reinterpret_cast<const float*>(base + in_off + (size_t)c * 4 * Hin * Win) + xx;
#pragma unroll
        for (int r = 0; r < NY; ++r) x[r] = (wreal)X[(size_t)sym_idx(r0 + r, Hin) * Win];
      } else {
        const wreal* X = base + in_off + (size_t)c * 4 * Hin * Win + xx;
#pragma unroll
        for (int r = 0; r < NY; ++r) x[r] = X[(size_t)sym_idx(r0 + r, Hin) * Win];
      }
    } else {
      const double* st = stats + (size_t)img * WL_STATS;
      wreal mn, mx;
      wl_minmax64(st, c, mn, mx);
      const wreal inv = mx - mn, rcp = 1.0 / inv;
      if (SRC == 0) {
        const uint8_t* col = src + (int64_t)img * Hin * row_stride + (int64_t)xx * 3;
        uint32_t raw[NY];
#pragma unroll
        for (int r = 0; r < NY; ++r) {  // all loads in flight before any use
          const uint8_t* p = col + (int64_t)sym_idx(r0 + r, Hin) * row_stride;
          raw[r] = (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16;
        }
#pragma unroll
        for (int r = 0; r < NY; ++r) {
          double px[3];
#pragma unroll
          for (int k = 0; k < 3; ++k) px[k] = (double)((raw[r] >> (8 * k)) & 0xFFu) * (1.0 / 255.0);
          // skimage: channel = out - min; channel /= max - min, as the IEEE quotient (reciprocal
          // multiply + one Markstein correction, exact over every u8 triple: tools/check_div.c)
          const wreal a = ycbcr_c(px, c) - mn;
          const wreal qq = a * rcp;
          x[r] = __fma_rn(__fma_rn(-qq, inv, a), rcp, qq);
        }
      } else {
        double px[NY][3];
#pragma unroll
        for (int r = 0; r < NY; ++r)
          load_rgb64(src, in64, img, Hin, Win, row_stride, sym_idx(r0 + r, Hin), xx, px[r]);
#pragma unroll
        for (int r = 0; r < NY; ++r) x[r] = (ycbcr_c(px[r], c) - mn) / inv;
      }
    }
    // axis 0 first (pywt dwtn order): output row ii uses staged rows 2ii + F-1-p
#pragma unroll
    for (int ii = 0; ii < RB_TY; ++ii) {
      wreal lo = 0, hi = 0;
#pragma unroll
      for (int p = 0; p < F; ++p) {
        const wreal v = x[2 * ii + F - 1 - p];
        // the highpass keeps pywt's mul-then-add (dd's exact zeros feed the sigma median); the
        // lowpass only reaches aa / ad / da, whose rounding the thresholds and the synthesis
        // absorb (1e-16 relative), so it takes fmas
        if (Wv::dlo[p] != 0) lo = __fma_rn(Wv::dlo[p], v, lo);
        if (Wv::dhi[p] != 0) hi = __dadd_rn(hi, __dmul_rn(Wv::dhi[p], v));  // pywt: mul, then add
      }
      S.vl[c][ii][q] = lo;
      S.vh[c][ii][q] = hi;
    }
  }
  __syncthreads();
  // wave = channel (waves 0-2); lane bits [5] g / 4, [4:2] ii, [1:0] g % 4: a 32-lane half reads
  // 8 rows x 4 column groups, whose ds_read_b64 addresses (row stride NX + 1, 8 doubles per
  // group) fall on distinct bank pairs (lanes g / g + 4 of one row were 2-way conflicts)
  const int c = t >> 6, ii = (t >> 2) & 7, g = ((t >> 5) & 1) * 4 + (t & 3);
  const int i = i0 + ii, jl = g * RB_R;
  constexpr int NC = 2 * RB_R + F - 2;  // staged columns one thread reads
  wreal l[NC], h[NC];
  if (t < 192) {
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      l[k] = S.vl[c][ii][2 * jl + k];
      h[k] = S.vh[c][ii][2 * jl + k];
    }
  }
  __syncthreads();  // vl / vh become the output staging buffer
  // rows padded to RB_OBS = RB_TX + 1 doubles: the 16 lanes of a ds_write_b64 group (4 rows x 4
  // column groups) hit distinct bank pairs (an unpadded stride made them 4-way conflicts)
  static_assert(sizeof(S) >= sizeof(wreal) * 3 * 4 * RB_TY * RB_OBS, "band staging fits");
  wreal(*ob)[4][RB_TY][RB_OBS] = reinterpret_cast<wreal(*)[4][RB_TY][RB_OBS]>(&S.vl[0][0][0]);
  double sq[3] = {0.0, 0.0, 0.0};
  if (t < 192) {
#pragma unroll
  for (int r = 0; r < RB_R; ++r) {
    wreal aa = 0, ad = 0, da = 0, dd = 0;
#pragma unroll
    for (int qq = 0; qq < F; ++qq) {  // then axis 1: output column j uses staged cols 2j + F-1-q
      const wreal lv = l[2 * r + F - 1 - qq], hv = h[2 * r + F - 1 - qq];
      if (Wv::dlo[qq] != 0) {
        aa = __fma_rn(Wv::dlo[qq], lv, aa);  // key 'aa': axis 0 low, axis 1 low
        da = __fma_rn(Wv::dlo[qq], hv, da);  // key 'da': axis 0 high, axis 1 low
      }
      if (Wv::dhi[qq] != 0) {
        ad = __fma_rn(Wv::dhi[qq], lv, ad);                 // key 'ad': axis 0 low, axis 1 high
        dd = __dadd_rn(dd, __dmul_rn(Wv::dhi[qq], hv));  // pywt's order: exact zeros
      }
    }
    // level 1: the fine-bin code of |dd| (0: exact zero) for the sigma median
    // (wl_haar_median<BAND>), in this channel's unused input-plane slot
    if (emit_codes && i < Ho && j0 + jl + r < Wo) {
      const unsigned long long key = absbits(dd);
      reinterpret_cast<uint16_t*>(base + (size_t)c * Hin * Win)[(size_t)i * Wo + j0 + jl + r] =
          (uint16_t)(key ? wl_fbin(key) + 1 : 0);
    }
    ob[c][0][ii][jl + r] = aa;
    ob[c][1][ii][jl + r] = ad;
    ob[c][2][ii][jl + r] = da;
    ob[c][3][ii][jl + r] = dd;
    if (i < Ho && j0 + jl + r < Wo) {
      sq[0] += ad * ad;
      sq[1] += da * da;
      sq[2] += dd * dd;
    }
  }
  // per-tile sums of squares of the three detail bands of this wave's channel, fixed order
  // (wl_sumsq adds the tiles)
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    double v = sq[b];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((t & 63) == 0)
      part[img * part_per_img + (size_t)(c * 3 + b) * (part_per_img / 9) + part_tile0 +
           blockIdx.x] = v;
  }
  }
  __syncthreads();
  // coalesced band stores: rows of RB_TX coefficients, 16 lanes x 16 bytes per row; fp32 bands
  // (fmask) in the first half of their slot
  const size_t bsz = (size_t)Ho * Wo;
  constexpr int PR = RB_TX / 2;  // coefficient pairs per row
  for (int k = t; k < 3 * 4 * RB_TY * PR; k += 256) {
    const int row = k / PR, pr = k - row * PR;  // row = (c * 4 + band) * RB_TY + ii
    const int cb = row / RB_TY, iy = row - cb * RB_TY;  // wave-uniform (4 rows of one band)
    const int oi = i0 + iy, oj = j0 + 2 * pr;
    if (oi >= Ho || oj >= Wo) continue;
    const wreal* sv = &ob[0][0][0][0] + (size_t)row * RB_OBS + 2 * pr;
    if (wl_fband(fmask, cb & 3)) {
      float* dst = reinterpret_cast<float*>(base + out_off + (size_t)cb * bsz) + (size_t)oi * Wo + oj;
      dst[0] = (float)sv[0];
      if (oj + 1 < Wo) dst[1] = (float)sv[1];
    } else {
      wreal* dst = base + out_off + (size_t)cb * bsz + (size_t)oi * Wo + oj;
      dst[0] = sv[0];
      if (oj + 1 < Wo) dst[1] = sv[1];
    }
  }
}

// ---- 2b: bior1.5 analysis, streaming form ------------------------------------------------------
// pywt's bior1.5 decomposition pair in terms of input pairs: with s_k = x[2k] + x[2k+1] and
// e_k = x[2k+1] - x[2k] over the symmetrically extended input (output i uses x[2i-8 .. 2i+1]),
//   lo[i] = S2 s_{i-2} + B1 (e_i - e_{i-4}) + B2 (e_{i-3} - e_{i-1})     (10 taps -> 5 operations;
//           rounding within a few ulps of pywt's sum: aa / ad / da only feed the thresholds and
//           the synthesis, both checked within 1e-5)
//   hi[i] = (-S2 x[2i-3]) + S2 x[2i-4]                                  (pywt's order, exact:
//           the finest dd's exact zeros select the sigma median's population)
// One workgroup per (image, strip of SW output columns, band of output rows) walks down the rows,
// one input row pair per step.
//   column phase: thread u = staged input column 2 j0 - 8 + u (all three channels) normalises its
//     two new samples -- every sample once per strip (halo: 8 of 2 SW + 8 columns; the tiled
//     wl_dwt_rb normalised each sample ~1.7 times) -- and adds the pair to five running lowpass
//     accumulators (pair k contributes B1 e_k, -B2 e_k, S2 s_k, B2 e_k, -B1 e_k to outputs
//     k .. k+4); output row i's column lowpass / highpass go to LDS (double-buffered: one barrier
//     per step).  The raw samples of the next PF steps are in flight in a register ring.
//   row phase: thread (c, jj) runs the pair form along the row for the two adjacent outputs jj,
//     jj + 1: aa / da (lowpass of the column low / high), ad = S2 (v[2j-4] - v[2j-3]), dd in
//     pywt's exact order; band stores (fp32 bands per fmask), level-1 dd codes, sums of squares
// Row bands start four pairs early to fill the accumulators (4 / band height extra work).
#ifndef IDN_WS_MAXT  // A/B builds set it
#define IDN_WS_MAXT 512
#endif
constexpr int WS_MAXT = IDN_WS_MAXT;         // threads = staged columns per workgroup (max)
// output columns per strip (max): (threads - 8) / 2; tuning: IDN_WAVELET_WST threads (64..256)
inline int ws_maxsw() {
  const int t = std::min(std::max(knob("IDN_WAVELET_WST", WS_MAXT), 64), WS_MAXT) / 64 * 64;
  return (t - 8) / 2;
}
inline int ws_strips(int Wo) { return (Wo + ws_maxsw() - 1) / ws_maxsw(); }
inline int ws_sw(int Wo) {
  const int st = ws_strips(Wo);
  return ((Wo + st - 1) / st + 1) & ~1;
}
int ws_resident(int level, int block);  // resident analysis workgroups (defined below)
// bands of whole WS_G-row groups, >= 16 output rows each: as best_bands, costed by the rows of
// the longest band
inline int ws_bands(int n, int Ho, int Wo, int strips, int level) {
  const int groups = (Ho + WS_G - 1) / WS_G;
  // resident workgroups as a 512-thread launch would have them.  (The deeper 600x1000 levels
  // launch 320 threads; counting those -- twice the workgroups per CU -- picked more, shorter bands
  // and measured 20 % slower at levels 2-3: the analysis is throughput-bound there, and extra bands
  // only add warm-up rows, profiles/r04/wavelet/.)
  (void)Wo;
  const int block = WS_MAXT;
  const int64_t units = (int64_t)n * strips, resident = std::max<int64_t>(ws_resident(level, block), 1);
  const int bmax = std::max(1, std::min({64, Ho / 16, groups}));
  int best = 1;
  double bestc = 1e300;
  for (int b = 1; b <= bmax; ++b) {
    const double rounds = std::ceil((double)(units * b) / (double)resident);
    const double c = rounds * ((groups + b - 1) / b * WS_G + 4);
    if (c < bestc * 0.999) {
      bestc = c;
      best = b;
    }
  }
  return best;
}

template <int SRC>
struct WsRaw;  // the raw input of one step (two rows) for one staged column
template <> struct WsRaw<0> {  // u8 pixels: the raw dword holding each row's 3 bytes (see load)
  uint32_t p[2];
};
template <> struct WsRaw<1> {  // f64 pixels
  double p[2][3];
};
template <> struct WsRaw<2> {  // the level above's 'aa', three channels, fp64
  double p[2][3];
};
template <> struct WsRaw<3> {  // the level above's 'aa', three channels, fp32 (WL_FB_AIN)
  float p[2][3];
};
// prefetch depth (steps; divides 5): the u8 and fp32 rings are small, the fp64 ones are not.
// (Round 3 measured the fp32 'aa' ring at depth 5 1 % slower than depth 1 -- when no ring load was
// in flight past its own step, see the ring comments in wl_dwt_stream; with working prefetch
// depth 5 is the faster.)
#ifndef IDN_WS_PF0  // A/B builds set these
#define IDN_WS_PF0 5
#endif
#ifndef IDN_WS_WPE
#define IDN_WS_WPE 1
#endif
#ifndef IDN_S3_WPE
#define IDN_S3_WPE 1
#endif
#ifndef IDN_S3_PAD
#define IDN_S3_PAD 0
#endif
#ifndef IDN_WS_PF3  // the fp32 'aa' input of levels >= 2: a 5-step ring measured 2.773 -> 2.752 ms on
#define IDN_WS_PF3 5  // the op against 1 (levels 2 / 3: 283 -> 264 / 92 -> 88 us, profiles/r04/wavelet/)
#endif
#ifndef IDN_WS_PF1  // the live path's fp64 pixels (A/B builds set it)
#define IDN_WS_PF1 1
#endif
template <int SRC> constexpr int ws_pf() {
  return SRC == 0 ? IDN_WS_PF0 : SRC == 3 ? IDN_WS_PF3 : SRC == 1 ? IDN_WS_PF1 : 1;
}


__device__ __forceinline__ double uniform_f64(double v) {  // a wave-uniform double into SGPRs
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readfirstlane((int)b);
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo));
}
__device__ __forceinline__ int ycc_w(int c, int k) {  // rgb2ycbcr coefficients x 1000
  constexpr int W[3][3] = {{65481, 128553, 24966}, {-37797, -74203, 112000}, {112000, -93786, -18214}};
  return W[c][k];
}
// bior1.5: the level-1 highpass has two taps, so a finest dd is the 2x2 combination of the
// normalised samples at rows 2i-4, 2i-3 and columns 2j-4, 2j-3 (pywt 'symmetric' indices), in
// wl_dwt_stream's op order: the column highpass (two products, then their sum) of both columns,
// then the row highpass.  The sigma median recomputes the few exact values it needs from the input
// (wl_haar_median<1, true, true>), so the analysis keeps the level-1 dd band in fp32 only -- all
// that the synthesis reads of it.
__device__ __forceinline__ double bior_dd2x2(double x00, double x01, double x10, double x11) {
  const double h0 = (-S2) * x10 + S2 * x00, h1 = (-S2) * x11 + S2 * x01;  // x[row][column]
  return (-S2) * h1 + S2 * h0;
}
struct BiorDdRaw {  // u8: the dword holding each sample's 3 bytes, and the bit offset of the pixel
  uint32_t v[2][2];
  uint32_t sh[2];
};
__device__ __forceinline__ BiorDdRaw wl_bior_dd1_load(rsrc_t rs, int h, int w, int64_t row_stride,
                                                      uint32_t pos, int W1) {
  const int i = (int)(pos / (uint32_t)W1), j = (int)(pos - (uint32_t)i * (uint32_t)W1);
  const int y[2] = {sym_idx(2 * i - 4, h), sym_idx(2 * i - 3, h)};
  const int x[2] = {sym_idx(2 * j - 4, w), sym_idx(2 * j - 3, w)};
  BiorDdRaw q;
#pragma unroll
  for (int cc = 0; cc < 2; ++cc) q.sh[cc] = x[cc] > 0 ? 8u : 0u;
  // bytes 3x - 1 .. 3x + 2 (0 .. 3 at x = 0): never past the end.  The whole offset goes in the
  // per-lane operand (a per-lane row offset in the scalar one becomes a loop over the lanes)
#pragma unroll
  for (int rr = 0; rr < 2; ++rr)
#pragma unroll
    for (int cc = 0; cc < 2; ++cc)
      q.v[rr][cc] = __builtin_amdgcn_raw_buffer_load_b32(
          rs, (uint32_t)((int64_t)y[rr] * row_stride) + (x[cc] > 0 ? 3u * (uint32_t)x[cc] - 1u : 0u),
          0u, 0);
  return q;
}
__device__ __forceinline__ unsigned long long wl_bior_dd1_eval(const BiorDdRaw& q, int c, wreal mn,
                                                               wreal inv, wreal rcp) {
  double r[2][2];
#pragma unroll
  for (int rr = 0; rr < 2; ++rr)
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      double px[3];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch)
        px[ch] = (double)((q.v[rr][cc] >> (q.sh[cc] + 8 * ch)) & 0xFFu) * (1.0 / 255.0);
      const wreal a = ycbcr_c(px, c) - mn;  // wl_dwt_stream's norm (u8: reciprocal + Markstein)
      const wreal q0 = a * rcp;
      r[rr][cc] = __fma_rn(__fma_rn(-q0, inv, a), rcp, q0);
    }
  return absbits(bior_dd2x2(r[0][0], r[0][1], r[1][0], r[1][1]));
}
// TL / TH: arithmetic of the lowpass / highpass paths.  fp64 throughout is pywt's precision; the
// product runs the lowpass outputs (aa, ad, da: continuous inputs of the thresholds' fp64 sums of
// squares and of the synthesis) in fp32, and at level 1 keeps the normalisation, the column
// highpass and dd in fp64 with pywt's op order (the finest dd's exact zeros select the sigma
// median's population); deeper levels (no median) run both paths in fp32.
// FM >= 0: the band storage mask (wl_fband) and CODES the level-1 code emission as compile-time
// constants (the product's masks: no per-band branches); FM = -1 takes both from the arguments.
// NT: threads per workgroup the LDS arrays are sized for (the product launches 512; instances
// sized for 64- and 256-thread strips measured slower at every band count: level 1 1.39 / 1.04
// ms vs 0.93, profiles/r04/wavelet/strips_sweep.txt)
template <int SRC, typename TL = wreal, typename TH = wreal, int FM = -1, int CODES = -1,
          int NT = WS_MAXT>
__global__ __launch_bounds__(NT, IDN_WS_WPE) void wl_dwt_stream(
    wreal* __restrict__ ws, size_t img_floats, const double* __restrict__ stats, size_t in_off,
    int Hin, int Win, size_t out_off, int Ho, int Wo, int SW, int strips, int bands, int groups,
    const uint8_t* __restrict__ src, const double* __restrict__ in64, int64_t row_stride,
    double* __restrict__ part, size_t part_per_img, size_t part_tile0, int emit_codes_arg,
    int fmask_arg, double sq_grid) {
  const int fmask = FM >= 0 ? FM : fmask_arg;
  const int emit_codes = CODES >= 0 ? CODES : emit_codes_arg;
  constexpr int PF = ws_pf<SRC>();
  // VL / VF: the column lowpass / highpass in the lowpass type (TL) at staged column u; VH: the
  // column highpass in TH for dd, even and odd columns in separate halves (column u at
  // (u & 1) * WS_MAXT / 2 + u / 2) so that the row threads' 16-byte reads (lane stride 4 columns)
  // fill whole bank rows -- interleaved fp64 columns put two lanes on every 16-byte slot
  constexpr bool SEPF = !std::is_same<TL, TH>::value;  // a separate TL copy of the highpass
  // N32 (round 6; u8 level 1 with an fp32 highpass): the normalisation is one fp32 affine map of
  // the bytes per channel, and the finest dd's codes come from the exact integer T = K00 - K10 -
  // K01 + K11 of the pixels' YCbCr keys K = w . rgb (the dd is 0.5 T / (255000 range) within
  // 2e-12 / range, as for the fused Haar: wl_haar_stats' certainty rule, the exact fp64 key where
  // it is not certain) -- sigma stays bit-identical while every coefficient runs in fp32
  constexpr bool N32 = SRC == 0 && std::is_same<TH, float>::value && CODES != 0;
  __shared__ TL VL[2][3][NT];
  __shared__ TL VF[SEPF ? 2 : 1][SEPF ? 3 : 1][SEPF ? NT : 1];
  __shared__ TH VH[2][3][NT];
  __shared__ int VK[N32 ? 2 : 1][N32 ? 3 : 1][N32 ? NT : 1];  // key column highpass, VH's layout
  __shared__ double RED[3][NT];
  const int img = blockIdx.z;
  const int strip = (int)blockIdx.x % strips, band = (int)blockIdx.x / strips;
  const int j0 = strip * SW;
  // the band: whole WS_G-row groups [ga, gb) (the last group of the image may be short)
  const int ga = (int)((int64_t)band * groups / bands), gb = (int)((int64_t)(band + 1) * groups / bands);
  const int ia = ga * WS_G, ib = min(gb * WS_G, Ho);
  const int t = threadIdx.x;
  wreal* base = ws + img * img_floats;
  // ---- column role
  const int NXs = 2 * SW + 8;
  const bool colt = t < NXs;
  const int qc = sym_idx(2 * j0 - 8 + t, Win);  // this thread's input column
  // u8 source: one unaligned dword per row, bytes 3 qc - 1 .. 3 qc + 2 (bytes 0..3 for column 0),
  // so it never reaches past the image's last byte; the pixel is at bit qsh of it.  The bytes are
  // extracted where the step is consumed (norm), PF steps later: packing three byte loads at load
  // time made every load wait for its data at once, and the ring prefetched nothing.
  const uint32_t qvo = qc > 0 ? 3u * (uint32_t)qc - 1u : 0u, qsh = qc > 0 ? 8u : 0u;
  wreal mn[3] = {0, 0, 0}, inv[3] = {1, 1, 1}, rcp[3] = {1, 1, 1};
  if (SRC < 2) {
    const double* st = stats + (size_t)img * WL_STATS;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      wreal mx;
      wl_minmax64(st, c, mn[c], mx);
      inv[c] = mx - mn[c];
      rcp[c] = 1.0 / inv[c];
    }
  }
  // N32: x_c = sum_k A[c][k] b_k + Bc[c] (b the bytes) = ((w_c . b) / 255000 + off_c - min_c) / range_c
  float A32c[3][3] = {}, B32c[3] = {};
  double sc1[3] = {0.0, 0.0, 0.0};  // the finest dd per unit of T: 0.5 / (255000 range)
  if constexpr (N32) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      sc1[c] = uniform_f64(0.5 / (255000.0 * inv[c]));
#pragma unroll
      for (int k = 0; k < 3; ++k) A32c[c][k] = (float)((double)ycc_w(c, k) / (255000.0 * inv[c]));
      B32c[c] = (float)(((c == 0 ? 16.0 : 128.0) - mn[c]) / inv[c]);
    }
  }
  rsrc_t rs;
  if (SRC == 0)
    rs = make_rsrc(src + (int64_t)img * Hin * row_stride, (uint32_t)((int64_t)Hin * row_stride));
  else if (SRC == 1)
    rs = make_rsrc(in64 + (int64_t)img * Hin * Win * 3, (uint32_t)((int64_t)Hin * Win * 24));
  auto load = [&](int k, WsRaw<SRC>& R) {
    const int rows[2] = {sym_idx(2 * k, Hin), sym_idx(2 * k + 1, Hin)};
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      if constexpr (SRC == 0) {
        const uint32_t so = (uint32_t)((int64_t)rows[h2] * row_stride);
        R.p[h2] = __builtin_amdgcn_raw_buffer_load_b32(rs, qvo, so, 0);
      } else if constexpr (SRC == 1) {
        const uint32_t so = (uint32_t)rows[h2] * (uint32_t)Win * 24u;
#pragma unroll
        for (int k3 = 0; k3 < 3; ++k3)
          R.p[h2][k3] = __longlong_as_double((long long)__builtin_amdgcn_raw_buffer_load_b64(
              rs, (uint32_t)qc * 24u + 8u * k3, so, 0));
      } else {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const wreal* X = base + in_off + (size_t)c * 4 * Hin * Win;
          const size_t e = (size_t)rows[h2] * Win + qc;
          if constexpr (SRC == 3) R.p[h2][c] = reinterpret_cast<const float*>(X)[e];
          else R.p[h2][c] = X[e];
        }
      }
    }
  };
  // channel c of row h2 of the raw step: normalised (SRC 0 / 1) or the aa sample (SRC 2)
  auto norm = [&](const WsRaw<SRC>& R, int h2, int c) -> wreal {
    if constexpr (SRC >= 2) {
      return (wreal)R.p[h2][c];
    } else {
      double px[3];
#pragma unroll
      for (int k3 = 0; k3 < 3; ++k3) {
        if constexpr (SRC == 0) px[k3] = (double)((R.p[h2] >> (qsh + 8 * k3)) & 0xFFu) * (1.0 / 255.0);
        else px[k3] = R.p[h2][k3];
      }
      const wreal a = ycbcr_c(px, c) - mn[c];
      if constexpr (SRC == 1) {
        return a / inv[c];
      } else {
        // skimage's (Y - min) / (max - min) as the IEEE quotient: reciprocal multiply + one
        // Markstein correction, exact over every u8 triple (tools/check_div.c)
        const wreal qq = a * rcp[c];
        return __fma_rn(__fma_rn(-qq, inv[c], a), rcp[c], qq);
      }
    }
  };
  TL acc[3][5];              // running column lowpass of outputs k .. k+4 (slot = output % 5)
  TH hd0[3], hd1[3];         // column highpass of pairs k-1, k-2 (hi[i] is pair i-2's)
  int kd0[3], kd1[3];        // N32: the key highpass K(row 2k) - K(row 2k+1) of the same pairs
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    kd0[c] = kd1[c] = 0;
    hd0[c] = hd1[c] = (TH)0;
#pragma unroll
    for (int r = 0; r < 5; ++r) acc[c][r] = (TL)0;
  }
  // ---- row role
  const int half = SW / 2;
  // task u = (channel rc, column pair jj): at level 1 spread over every wave of the workgroup in
  // contiguous runs, so that no wave sits at the step's barrier without row work (934 vs 962 us);
  // deeper levels keep u = t (spread measured 273 vs 262 us at level 2: profiles/r04/wavelet/)
  const int nwv = (int)(blockDim.x >> 6);  // waves of the launch (NT is only the maximum)
  const int rw = SRC < 2 ? (3 * half + nwv - 1) / nwv : 64;  // tasks per wave
  const int u = SRC < 2 ? (t >> 6) * rw + (t & 63) : t;
  const bool rowt = (t & 63) < rw && u < 3 * half;
  const int rc = rowt ? u / half : 0, jj = rowt ? 2 * (u - rc * half) : 0;
  const int oj = j0 + jj;
  const bool ok0 = rowt && oj < Wo, ok1 = rowt && oj + 1 < Wo;
  const size_t bsz = (size_t)Ho * Wo;
  // Sums of squares, independent of the band split (batch size, device): each row thread sums
  // its two outputs of a WS_G-row group's rows in row order (sq), and at the group's last row rounds
  // that partial to a multiple of sq_grid (a power of two) into sqa.  Sums of multiples of
  // sq_grid below 2^53 sq_grid are exact in fp64, and the layout sizes sq_grid so that the whole
  // band's sum stays below that (wl_layout): every later addition -- this thread's groups, the
  // workgroup's threads, wl_sumsq's tiles -- is exact, hence order-free.  (Rounding error per
  // partial <= sq_grid / 2, ~1e-10 of a typical band total.)
  double sq[3] = {0.0, 0.0, 0.0}, sqa[3] = {0.0, 0.0, 0.0};
  const double sq_inv = 1.0 / sq_grid;  // exact: a power of two

  const int k0 = ia - 4, M = ib - ia + 4;  // steps m = 0 .. M-1 cover pairs k = k0 + m
  WsRaw<SRC> rq[PF];                        // raw samples of steps m .. m + PF - 1 (slot m % PF)
  // the ring's loads are unconditional (rows past the band mirror into the image, sym_idx, and are
  // never used): a load under a branch leaves a phi whose copy waits for the data at once
#pragma unroll
  for (int f = 0; f < PF; ++f) load(k0 + f, rq[f]);
  for (int m0 = 0; m0 < M; m0 += 5) {
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const int m = m0 + r;
      const int k = k0 + m;
      const int buf = m & 1;
      if (colt) {
        const int slot = r % PF;  // PF divides 5 (compile-time after unrolling)
        const WsRaw<SRC>& cur = rq[slot];
        float bf[2][3];   // N32: the pixel bytes as floats
        int bi[2][3];     //      and as integers
        if constexpr (N32) {
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
            for (int k3 = 0; k3 < 3; ++k3) {
              bi[h2][k3] = (int)((cur.p[h2] >> (qsh + 8 * k3)) & 0xFFu);
              bf[h2][k3] = (float)bi[h2][k3];
            }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          TH h0, h1;
          TL l0, l1;
          if constexpr (N32) {
            const float y0 = __fmaf_rn(A32c[c][2], bf[0][2], __fmaf_rn(A32c[c][1], bf[0][1], __fmaf_rn(A32c[c][0], bf[0][0], B32c[c])));
            const float y1 = __fmaf_rn(A32c[c][2], bf[1][2], __fmaf_rn(A32c[c][1], bf[1][1], __fmaf_rn(A32c[c][0], bf[1][0], B32c[c])));
            l0 = (TL)y0;
            l1 = (TL)y1;
            h0 = (TH)y0;
            h1 = (TH)y1;
          } else {
            const auto x0 = norm(cur, 0, c), x1 = norm(cur, 1, c);
            l0 = (TL)x0;
            l1 = (TL)x1;
            h0 = (TH)x0;
            h1 = (TH)x1;
          }
          const TL sk = l0 + l1, ek = l1 - l0;
          const TH hk = (TH)(-S2) * h1 + (TH)S2 * h0;  // pywt: mul, add (no contraction)
          // pair k's contributions; slot (k + j) % 5 == (r + j) % 5 for the unrolled r
          acc[c][(r + 4) % 5] = (TL)(-B1) * ek;
          acc[c][(r + 3) % 5] = fma_t<TL>((TL)B2, ek, acc[c][(r + 3) % 5]);
          acc[c][(r + 2) % 5] = fma_t<TL>((TL)S2, sk, acc[c][(r + 2) % 5]);
          acc[c][(r + 1) % 5] = fma_t<TL>((TL)(-B2), ek, acc[c][(r + 1) % 5]);
          const TL lo = fma_t<TL>((TL)B1, ek, acc[c][r]);  // output k complete
          if (m >= 4) {
            VL[buf][c][t] = lo;
            VH[buf][c][(t & 1) * (NT / 2) + (t >> 1)] = hd1[c];
            if constexpr (SEPF) VF[buf][c][t] = (TL)hd1[c];
            if constexpr (N32) VK[buf][c][(t & 1) * (NT / 2) + (t >> 1)] = kd1[c];
          }
          hd1[c] = hd0[c];
          hd0[c] = hk;
          if constexpr (N32) {
            kd1[c] = kd0[c];
            kd0[c] = (__mul24(ycc_w(c, 0), bi[0][0]) + __mul24(ycc_w(c, 1), bi[0][1]) + __mul24(ycc_w(c, 2), bi[0][2])) -
                     (__mul24(ycc_w(c, 0), bi[1][0]) + __mul24(ycc_w(c, 1), bi[1][1]) + __mul24(ycc_w(c, 2), bi[1][2]));
          }
        }
      }
      // refill the slot PF steps ahead, after its last use and outside the column threads' branch
      // (every thread loads; a load under the branch, or into a slot still being read, is copied
      // into the ring at the join and that copy waits for the data at once)
      load(k + PF, rq[r % PF]);
      // accumulator fill, and the steps that pad the band to whole 5-step iterations: their column
      // work is wasted, but every iteration then runs all five steps (wave-uniform).  (A break out of
      // the unrolled steps merges, at the loop header, a path on which the latest ring load is that
      // step's, and the compiler's wait at every slot's first use drops to that path's: the ring
      // would prefetch nothing.)
      if (m < 4 || m >= M) continue;
      __syncthreads();
      const int i = k;  // output row
      if (rowt) {
        const TL* vl = &VL[buf][rc][2 * jj];
        const TH* vhe = &VH[buf][rc][jj];                 // element 2 jj + m, m even: vhe[m / 2]
        const TH* vho = &VH[buf][rc][NT / 2 + jj];   //                   m odd:  vho[m / 2]
        const TL* vf = SEPF ? &VF[buf][rc][2 * jj] : nullptr;
        TL o[2][3];  // [output][aa, ad, da]
        TH odd[2];   // [output] dd
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {  // column low -> aa / ad, column high -> da / dd
          TL S[6], E[6];
#pragma unroll
          for (int nn = 0; nn < 6; ++nn) {
            TL a0, a1;
            if (pass == 0) {
              a0 = vl[2 * nn];
              a1 = vl[2 * nn + 1];
            } else if constexpr (SEPF) {
              a0 = vf[2 * nn];
              a1 = vf[2 * nn + 1];
            } else {
              a0 = (TL)vhe[nn];
              a1 = (TL)vho[nn];
            }
            S[nn] = a0 + a1;
            E[nn] = a1 - a0;
          }
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            o[d][2 * pass] = fma_t<TL>((TL)S2, S[2 + d],
                                       fma_t<TL>((TL)B1, E[4 + d] - E[d], (TL)B2 * (E[1 + d] - E[3 + d])));
            if (pass == 0) o[d][1] = (TL)(-S2) * E[2 + d];
            else odd[d] = (TH)(-S2) * vho[d + 2] + (TH)S2 * vhe[d + 2];  // elements 2d+5, 2d+4
          }
        }
        const size_t e0 = (size_t)i * Wo + oj;
        uint32_t code[2];
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          if (!(d ? ok1 : ok0)) continue;
          const double v1 = (double)o[d][1], v2 = (double)o[d][2], v3 = (double)odd[d];
          sq[0] = __fma_rn(v1, v1, sq[0]);  // (exact squares for the fp32 bands: = mul + add)
          sq[1] = __fma_rn(v2, v2, sq[1]);
          sq[2] = __fma_rn(v3, v3, sq[2]);
          if constexpr (N32) {
            const int* vke = &VK[buf][rc][jj];
            const int* vko = &VK[buf][rc][NT / 2 + jj];
            const int T = vke[d + 2] - vko[d + 2];  // elements 2d + 4 (even), 2d + 5 (odd)
            const uint32_t aT = (uint32_t)(T < 0 ? -T : T);
            const uint32_t hi = (uint32_t)__double2hiint((double)aT * sc1[rc]);
            code[d] = (uint32_t)min(max((int)(hi >> 16) - (1023 - 61) * 16, 0), WL_FBINS - 1) + 1u;
            if (!(aT >= 3u && (hi & 0xFFFFu) - 2u <= 0xFFFBu)) {
              // rare: the median workgroup sets this code from the exact fp64 key (the list sits
              // after the channel's codes, where the median's key scratch starts later)
              code[d] = 0u;
              uint32_t* lst = reinterpret_cast<uint32_t*>(base + (size_t)rc * Hin * Win + (bsz + 3) / 4);
              lst[atomicAdd(reinterpret_cast<uint32_t*>(const_cast<double*>(stats) + (size_t)img * WL_STATS + WL_N32U + rc), 1u)] =
                  (uint32_t)(i * Wo + oj + d);
            }
          } else {
            const unsigned long long key = absbits((double)odd[d]);
            code[d] = key ? wl_fbin(key) + 1 : 0;
          }
        }
        if (emit_codes) {  // the pair's two codes as one dword where it is aligned
          uint16_t* cp = reinterpret_cast<uint16_t*>(base + (size_t)rc * Hin * Win) + e0;
          if (ok1 && (e0 & 1) == 0) {
            *reinterpret_cast<uint32_t*>(cp) = code[0] | code[1] << 16;
          } else {
            if (ok0) cp[0] = (uint16_t)code[0];
            if (ok1) cp[1] = (uint16_t)code[1];
          }
        }
        wreal* ob = base + out_off + (size_t)rc * 4 * bsz;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const double w0 = b < 3 ? (double)o[0][b] : (double)odd[0];
          const double w1 = b < 3 ? (double)o[1][b] : (double)odd[1];
          if (wl_fband(fmask, b)) {
            float* f = reinterpret_cast<float*>(ob + (size_t)b * bsz) + e0;
            if (ok1 && ((uintptr_t)f & 7) == 0) {  // both outputs, one aligned 8-byte store
              *reinterpret_cast<float2*>(f) = make_float2((float)w0, (float)w1);
            } else {
              if (ok0) f[0] = (float)w0;
              if (ok1) f[1] = (float)w1;
            }
          } else {
            wreal* f = ob + (size_t)b * bsz + e0;
            if (ok1 && ((uintptr_t)f & 15) == 0) {
              *reinterpret_cast<double2*>(f) = make_double2(w0, w1);
            } else {
              if (ok0) f[0] = w0;
              if (ok1) f[1] = w1;
            }
          }
        }
      }
      // the group ends at this row: i + 1 = ia - 3 + m is a multiple of WS_G = 5 exactly when
      // r = m - m0 = 3 (ia and m0 are multiples of 5)
      if (r == 3) {
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          sqa[b] = __fma_rn(__builtin_rint(sq[b] * sq_inv), sq_grid, sqa[b]);
          sq[b] = 0.0;
        }
      }
    }
  }
#pragma unroll
  for (int b = 0; b < 3; ++b)  // the image's last group when Ho is not a multiple of 5 (else 0)
    sqa[b] = __fma_rn(__builtin_rint(sq[b] * sq_inv), sq_grid, sqa[b]);
  // per-workgroup sums (exact, see above), channel by channel
  __syncthreads();
  double* red = &RED[0][0];
  if (rowt) {
#pragma unroll
    for (int b = 0; b < 3; ++b) red[b * NT + u] = sqa[b];
  }
  __syncthreads();
  if (t < 9) {
    const int c = t / 3, b = t - 3 * c;
    double s2 = 0.0;
    for (int g = 0; g < half; ++g) s2 += red[b * NT + c * half + g];
    part[img * part_per_img + (size_t)(c * 3 + b) * (part_per_img / 9) + part_tile0 + blockIdx.x] = s2;
  }
}

// resident workgroups of the product's streaming analysis of a level (level 1: u8 / fp32-lowpass;
// deeper: fp32 'aa' input), used by wl_layout's band count for every form of that level
int ws_resident(int level, int block) {
  const void* k = level == 1
      ? reinterpret_cast<const void*>(&wl_dwt_stream<0, float, wreal, 0b1111, 1>)
      : reinterpret_cast<const void*>(&wl_dwt_stream<3, float, float, 0b1111, 0>);
  return cu_count() * occ_wgs(k, block);
}

// ---- 3: sum of squares per detail band ----------------------------------------------------------
__global__ __launch_bounds__(256) void wl_sumsq(double* __restrict__ stats,
                                                const double* __restrict__ part, WlLayout Lt) {
  // block = (img, c, l, b): add the level's tile partials in tile order (deterministic)
  int t = blockIdx.x;
  const int b = t % 3;
  t /= 3;
  const int l = t % Lt.L;
  t /= Lt.L;
  const int c = t % 3;
  const int img = t / 3;
  const int lev = l + 1;
  const double* p = part + img * Lt.part_per_img + (size_t)(c * 3 + b) * (Lt.part_per_img / 9) +
                    Lt.part_tile0[lev];
  double s = 0.0;
  for (int k = threadIdx.x; k < Lt.tiles[lev]; k += 256) s += p[k];
  __shared__ double red[4];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0)
    stats[(size_t)img * WL_STATS + WlStats::sumsq(c, l, b, Lt.L)] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ---- 4: sigma = median(|finest dd| != 0) / ppf(0.75) ------------------------------------------
// The median is over the NONZERO coefficients, so which coefficients are exactly zero must match
// the reference: the analysis runs in fp64 with pywt's op order (normalise (Y - min)/(max - min),
// axis 0 then axis 1, multiply then add), under which equal samples give an exact 0.
// Exact rank selection over the nonzero |d| of one band, on the IEEE bits (non-negative doubles
// order like their bit patterns).  Radix passes of <= 11 bits: the first two run over the band
// (the first also counts the nonzero keys), then the keys sharing the selected 22-bit prefix are
// compacted into a scratch slot and the last four passes run over that (typically a few hundred
// keys).  The upper middle rank (even counts) costs one more band pass: it equals the lower value
// while enough keys are <= it, otherwise it is the smallest key above it.  Compaction slots are
// allocated once per wave (ballot + popcount).
struct RadixState {
  unsigned long long prefix, pmask;
  uint32_t rank;
};


// block-wide selection over an LDS histogram: the bin holding rank `rank` and the rank within
// it.  Thread i owns bins [i*per, (i+1)*per); the thread whose count range holds the rank finds
// the bin (a serial scan of 2048 LDS bins by one thread costs ~100k cycles).  lower_mid: select
// the lower middle rank (total-1)/2 instead, and return the total through *total.
struct BinSel {
  uint32_t bin, rank;
};
__device__ BinSel select_bin(const uint32_t* hist, int nb, uint32_t rank, uint32_t* total,
                             bool lower_mid) {
  __shared__ uint32_t sel_bin, sel_rank, wsum[32], tot_s;
  const int T = blockDim.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int per = (nb + T - 1) / T, b0 = threadIdx.x * per, b1 = min(b0 + per, nb);
  uint32_t own = 0;
  for (int b = b0; b < b1; ++b) own += hist[b];
  uint32_t inc = own;  // inclusive scan within the wave
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)inc, o);
    if (lane >= o) inc += t;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int k = 0; k < (T + 63) / 64; ++k) {
      const uint32_t t = wsum[k];
      wsum[k] = acc;
      acc += t;
    }
    tot_s = acc;
    sel_bin = (uint32_t)(nb - 1);  // fallback: rank beyond the total
    sel_rank = 0;
  }
  __syncthreads();
  if (lower_mid) {
    if (total) *total = tot_s;
    rank = tot_s ? (tot_s - 1) / 2 : 0;
  }
  const uint32_t excl = wsum[wv] + inc - own;
  if (own && rank >= excl && rank < excl + own) {
    uint32_t acc = excl;
    int b = b0;
    for (; b < b1 - 1; ++b) {
      if (acc + hist[b] > rank) break;
      acc += hist[b];
    }
    sel_bin = (uint32_t)b;
    sel_rank = rank - acc;
  }
  __syncthreads();
  const BinSel r{sel_bin, sel_rank};
  __syncthreads();
  return r;
}

// one histogram pass over keys[0..n) (only keys matching the prefix); narrows the state.
// total (optional) receives the number of nonzero keys seen (first pass only).
__device__ void radix_pass(const double* __restrict__ d, size_t n, int sh, int wd, RadixState& rsx,
                           uint32_t* hist, uint32_t* total) {
  const int nb = 1 << wd;
  for (int k = threadIdx.x; k < nb; k += blockDim.x) hist[k] = 0;
  __syncthreads();
  const unsigned long long prefix = rsx.prefix, pmask = rsx.pmask;
  // 8 loads in flight per thread (a one-load-per-iteration loop is latency-bound)
  for (size_t k0 = threadIdx.x; k0 < n; k0 += 8 * (size_t)blockDim.x) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const size_t k = k0 + (size_t)u * blockDim.x;
      v[u] = k < n ? d[k] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const unsigned long long key = absbits(v[u]);
      if (key != 0 && (key & pmask) == prefix) atomicAdd(&hist[(key >> sh) & (nb - 1)], 1u);
    }
  }
  __syncthreads();
  const BinSel bs = select_bin(hist, nb, rsx.rank, total, total != nullptr);
  rsx.prefix |= (unsigned long long)bs.bin << sh;
  rsx.pmask |= (unsigned long long)(nb - 1) << sh;
  rsx.rank = bs.rank;
  __syncthreads();
}

__global__ __launch_bounds__(1024) void wl_median(wreal* __restrict__ ws, size_t img_floats,
                                                  double* __restrict__ stats, WlLayout Lt) {
  const int img = blockIdx.x / 3, c = blockIdx.x % 3;
  const size_t bsz = (size_t)Lt.H[1] * Lt.W[1];
  const wreal* d = ws + img * img_floats + Lt.off_band[1] + (size_t)c * 4 * bsz + 3 * bsz;  // dd
  // scratch: this channel's input-plane slot (h*w >= band size), unused by the transform
  double* scratch = ws + img * img_floats + (size_t)c * Lt.h * Lt.w;
  __shared__ uint32_t hist[2048];
  __shared__ uint32_t total_s, m_s, le_s;
  __shared__ unsigned long long gt_s;
  if (threadIdx.x == 0) {
    m_s = 0;
    le_s = 0;
    gt_s = ~0ull;
  }
  RadixState rsx{0ull, 0ull, 0u};
  radix_pass(d, bsz, 52, 11, rsx, hist, &total_s);  // also counts the nonzero keys
  const uint32_t total = total_s;
  double med;
  if (total == 0) {
    med = NAN;  // np.median of an empty selection
  } else {
    const uint32_t klo = (total - 1) / 2, khi = total / 2;
    radix_pass(d, bsz, 41, 11, rsx, hist, nullptr);
    // compact the keys with the selected 22-bit prefix (wave-aggregated slot allocation)
    const int lane = threadIdx.x & 63;
    const size_t nr = (bsz + 1023) / 1024 * 1024;
    for (size_t k = threadIdx.x; k < nr; k += 1024) {
      const double v = k < bsz ? d[k] : 0.0;
      const unsigned long long key = absbits(v);
      const bool hit = key != 0 && (key & rsx.pmask) == rsx.prefix;
      const unsigned long long m = __ballot(hit);
      if (m) {
        uint32_t base = 0;
        const int leader = __ffsll((long long)m) - 1;
        if (lane == leader) base = atomicAdd(&m_s, (uint32_t)__popcll(m));
        base = (uint32_t)__shfl((int)base, leader);
        if (hit) scratch[base + __popcll(m & ((1ull << lane) - 1))] = v;
      }
    }
    __syncthreads();
    const size_t mcnt = m_s;
    radix_pass(scratch, mcnt, 30, 11, rsx, hist, nullptr);
    radix_pass(scratch, mcnt, 19, 11, rsx, hist, nullptr);
    radix_pass(scratch, mcnt, 8, 11, rsx, hist, nullptr);
    radix_pass(scratch, mcnt, 0, 8, rsx, hist, nullptr);
    const unsigned long long lo_key = rsx.prefix;
    const double vlo = __longlong_as_double((long long)lo_key);
    double vhi = vlo;
    if (khi != klo) {
      uint32_t le = 0;
      unsigned long long gt = ~0ull;
      for (size_t k = threadIdx.x; k < bsz; k += 1024) {
        const unsigned long long key = absbits(d[k]);
        if (key == 0) continue;
        if (key <= lo_key) ++le;
        else gt = key < gt ? key : gt;
      }
      for (int o = 32; o > 0; o >>= 1) {
        le += __shfl_xor(le, o);
        const unsigned long long og = (unsigned long long)__shfl_xor((long long)gt, o);
        gt = og < gt ? og : gt;
      }
      if (lane == 0) {
        atomicAdd(&le_s, le);
        atomicMin(&gt_s, gt);
      }
      __syncthreads();
      if (le_s <= khi) vhi = __longlong_as_double((long long)gt_s);
    }
    med = (vlo + vhi) / 2.0;  // np.median: mean of the two middle values
  }
  if (threadIdx.x == 0) {
    stats[(size_t)img * WL_STATS + WlStats::median(c, Lt.L)] = med;
    stats[(size_t)img * WL_STATS + WlStats::DIAG + c] = (double)total;  // diagnostics
  }
}

// ---- 5: BayesShrink thresholds ------------------------------------------------------------------
__global__ void wl_thresh(double* __restrict__ stats, WlLayout Lt) {
  const int img = blockIdx.x;
  if (threadIdx.x != 0) return;
  double* st = stats + (size_t)img * WL_STATS;
  bool bad = false;
  for (int c = 0; c < 3; ++c) {
    double mn, mx;
    wl_minmax64(st, c, mn, mx);
    if (!(mx > mn)) bad = true;  // 0.14.2 divides by zero -> NaN everywhere -> U8 0
    const double sigma = st[WlStats::median(c, Lt.L)] / 0.6744897501960817;
    if (!(sigma == sigma)) bad = true;
    const double var = sigma * sigma;
    for (int l = 0; l < Lt.L; ++l)
      for (int b = 0; b < 3; ++b) {
        const int lev = l + 1;
        const double cnt = (double)Lt.H[lev] * Lt.W[lev];
        const double dvar = st[WlStats::sumsq(c, l, b, Lt.L)] / cnt;
        const double t = var / sqrt(fmax(dvar - var, 2.220446049250313e-16));
        st[WlStats::thr(c, l, b, Lt.L)] = t;
        if (Lt.L <= 3) st[WlStats::thrh(c, l, b)] = 0.5 * t;
      }
  }
  st[WlStats::FLAG] = bad ? 1.0 : 0.0;
}

// pywt.threshold(d, t, 'soft') = d * max(1 - t/|d|, 0) = sign(d) * max(|d| - t, 0): the same value
// to a few ulps (t >= 0), without the fp64 division per coefficient
__device__ __forceinline__ wreal soft(wreal d, wreal t) {
  const wreal m = fabs(d) - t;
  return m > 0.0 ? __builtin_copysign(m, d) : 0.0;
}

// ---- 6/7: synthesis, LDS-tiled and separable ---------------------------------------------------
// One workgroup per ST_O x ST_O output tile of the level being synthesised: it stages the
// (ST_O/2 + HF-1)^2 coefficients of the four bands the tile needs (details soft-thresholded on
// load), runs pywt idwtn's axis-1 pass into LDS ('a' from
// aa/ad, 'd' from da/dd) and then the axis-0 pass, each as upsampling_convolution_valid_sf's
// sum_even / sum_odd (lowpass sum + highpass sum, multiply then add, zero taps skipped); each
// thread computes an output pair from one set of HF coefficients.
// Levels L..2 write the approximation of the level below (cropped to its size); level 1
// (FINAL) runs the three channels of the tile in turn and fuses the inner clip [0, 1],
// de-normalisation, YCbCr -> RGB, the outer clip and the U8 / f32 stores.
// Round 1's per-pixel form gathered 36 coefficients per channel and pixel from L2 (7.0 ms per
// 256 bior1.5 images for the last level alone).
constexpr int ST_O = 32;

template <int WV>
struct SynthTile {
  static constexpr int F = Wav<WV>::F, HF = F / 2;
  static constexpr int CR = ST_O / 2 + HF - 1;  // staged coefficient rows / cols
  wreal co[4][CR][CR + 1];
  wreal sa[CR][ST_O + 1], sd[CR][ST_O + 1];
};

// one upsampling_convolution_valid_sf output pair (even, odd) from the HF coefficients
// c[j] = x[i - j]: lowpass part of the even / odd filter taps, multiply then add, zero taps
// skipped (they add +-0)
template <int WV, bool HI>
__device__ __forceinline__ void synth_pair(const wreal (&c)[Wav<WV>::F / 2], wreal& ev, wreal& od) {
  using Wv = Wav<WV>;
  constexpr int HF = Wv::F / 2;
  ev = 0;
  od = 0;
#pragma unroll
  for (int j = 0; j < HF; ++j) {
    const wreal fe = HI ? Wv::rhi[2 * j] : Wv::rlo[2 * j];
    const wreal fo = HI ? Wv::rhi[2 * j + 1] : Wv::rlo[2 * j + 1];
    if (fe != 0) ev = __dadd_rn(ev, __dmul_rn(fe, c[j]));
    if (fo != 0) od = __dadd_rn(od, __dmul_rn(fo, c[j]));
  }
}

// synthesise one channel's tile (bands at A, band size Nh x Nw, coefficient origin (m0, n0));
// thread t receives the tile outputs (row 2 * (t / ST_O) + r, column t % ST_O) for the row pairs
// of i (v[2 i + r]).  Split in two so a caller can keep the next channel's loads in flight while
// this one is synthesised: synth_load issues the thread's staging loads, synth_run stages them
// (details soft-thresholded) and runs the two passes.
template <int WV>
struct SynthLoad {
  static constexpr int CR = SynthTile<WV>::CR;
  static constexpr int RPT = 256 / CR;            // staging: band rows per pass (CR columns each)
  static constexpr int NRW = 4 * CR;              // band rows to stage
  static constexpr int NLD = (NRW + RPT - 1) / RPT;
  static_assert(NLD <= 32, "odd-index bits");
  wreal x[NLD];
  uint32_t odd;  // bit u set when x[u] holds an fp32 band pair whose odd element is wanted
};
template <int WV>
__device__ __forceinline__ void synth_load(SynthLoad<WV>& L, const wreal* __restrict__ A,
                                           size_t bsz, int Nh, int Nw, int m0, int n0, int fmask) {
  using SL = SynthLoad<WV>;
  const int cc = threadIdx.x % SL::CR, rr0 = threadIdx.x / SL::CR;
  // coefficients past the band's end feed only outputs past the level's valid length (pywt's
  // stage-2 valid convolution), which are never stored: clamped reads keep them finite
  const int col = min(n0 + cc, Nw - 1);
  L.odd = 0;
#pragma unroll
  for (int u = 0; u < SL::NLD; ++u) {  // all loads in flight before any use
    const int br = min(rr0 + SL::RPT * u, SL::NRW - 1);  // band * CR + row
    const int b = br / SL::CR, r = br - b * SL::CR;
    const size_t e = (size_t)min(m0 + r, Nh - 1) * Nw + col;
    // an fp32 band is read as the 8-byte pair holding element e (the same dwordx2 load for every
    // lane; the band's unique bytes halve), the half is picked in synth_run
    const bool f = wl_fband(fmask, b);
    L.x[u] = A[(size_t)b * bsz + (f ? e >> 1 : e)];
    if (f) L.odd |= (uint32_t)(e & 1) << u;
  }
}
// one output pair of the full synthesis step, lowpass band coefficients cl[j] and highpass
// cd[j] (c[j] = x[i - j]), written to (ev, od).  Haar / generic: pywt's sums (synth_pair).
// bior1.5: rlo has the two taps S2 (even, odd) at j = 2, and rhi's even / odd taps are
// B1, -B2, +-S2, B2, -B1, so with common = B1 (d0 - d4) + B2 (d3 - d1)
//   ev = common + S2 (a + d2),  od = common + S2 (a - d2)      (a = cl[2], d = cd)
// 8 operations for the pair instead of pywt's 26; the rounding differs from pywt's by a few ulps
// (the synthesis is checked within 1e-5, and no exact zero depends on it).
template <int WV>
__device__ __forceinline__ void synth_full(const wreal (&cl)[Wav<WV>::F / 2],
                                           const wreal (&cd)[Wav<WV>::F / 2], wreal& ev,
                                           wreal& od) {
  if constexpr (WV == IDN_WAVELET_BIOR15) {
    const wreal common = __fma_rn(B1, cd[0] - cd[4], B2 * (cd[3] - cd[1]));
    ev = __fma_rn(S2, cl[2] + cd[2], common);
    od = __fma_rn(S2, cl[2] - cd[2], common);
  } else {
    wreal le, lo, he, ho;
    synth_pair<WV, false>(cl, le, lo);
    synth_pair<WV, true>(cd, he, ho);
    ev = __dadd_rn(le, he);
    od = __dadd_rn(lo, ho);
  }
}

template <int WV, typename Between>
__device__ __forceinline__ void synth_run(SynthTile<WV>& S, const SynthLoad<WV>& L,
                                          const wreal (&thr)[3], wreal (&v)[ST_O * ST_O / 256],
                                          int fmask, Between between) {
  using SL = SynthLoad<WV>;
  constexpr int HF = SynthTile<WV>::HF, CR = SL::CR;
  const int cc = threadIdx.x % CR, rr0 = threadIdx.x / CR;
#pragma unroll
  for (int u = 0; u < SL::NLD; ++u) {
    const int br = rr0 + SL::RPT * u;
    if (rr0 < SL::RPT && br < SL::NRW) {
      const int b = br / CR, r = br - b * CR;
      wreal x = L.x[u];
      if (wl_fband(fmask, b)) {
        const unsigned long long bits = (unsigned long long)__double_as_longlong(x);
        x = (wreal)__uint_as_float((uint32_t)(((L.odd >> u) & 1u) ? bits >> 32 : bits));
      }
      S.co[b][r][cc] = b > 0 ? soft(x, thr[b - 1]) : x;
    }
  }
  __syncthreads();
  between();  // the staged registers are free: e.g. the next channel's loads
  for (int k = threadIdx.x; k < CR * (ST_O / 2); k += 256) {  // axis 1: column pairs
    const int r = k / (ST_O / 2), nn = k - r * (ST_O / 2);
    wreal c0[HF], c1[HF], c2[HF], c3[HF];
#pragma unroll
    for (int j = 0; j < HF; ++j) {
      const int col = nn + HF - 1 - j;
      c0[j] = S.co[0][r][col];
      c1[j] = S.co[1][r][col];
      c2[j] = S.co[2][r][col];
      c3[j] = S.co[3][r][col];
    }
    synth_full<WV>(c0, c1, S.sa[r][2 * nn], S.sa[r][2 * nn + 1]);
    synth_full<WV>(c2, c3, S.sd[r][2 * nn], S.sd[r][2 * nn + 1]);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < ST_O * ST_O / 512; ++i) {  // axis 0: row pairs
    const int k = threadIdx.x + 256 * i;
    const int m = k / ST_O, q = k - m * ST_O;
    wreal ca[HF], cd[HF];
#pragma unroll
    for (int j = 0; j < HF; ++j) {
      ca[j] = S.sa[m + HF - 1 - j][q];
      cd[j] = S.sd[m + HF - 1 - j][q];
    }
    synth_full<WV>(ca, cd, v[2 * i], v[2 * i + 1]);
  }
  __syncthreads();  // S is restaged by the next call
}
template <int WV>
__device__ __forceinline__ void synth_tile(SynthTile<WV>& S, const wreal* __restrict__ A,
                                           size_t bsz, int Nh, int Nw, int m0, int n0,
                                           const wreal (&thr)[3], wreal (&v)[ST_O * ST_O / 256],
                                           int fmask) {
  SynthLoad<WV> L;
  synth_load<WV>(L, A, bsz, Nh, Nw, m0, n0, fmask);
  synth_run<WV>(S, L, thr, v, fmask, [] {});
}
// output position of v[e] of thread t: (row, column) inside the tile
__device__ __forceinline__ int synth_row(int e) {
  return 2 * ((threadIdx.x + 256 * (e >> 1)) / ST_O) + (e & 1);
}
__device__ __forceinline__ int synth_col(int e) { return (threadIdx.x + 256 * (e >> 1)) % ST_O; }

// levels L..2: grid (tiles, n * 3); the level-(l-1) 'aa' slot receives the reconstruction
template <int WV>
__global__ __launch_bounds__(256) void wl_synth(wreal* __restrict__ ws, size_t img_floats,
                                                const double* __restrict__ stats, int level, int L,
                                                size_t in_off, int Nh, int Nw, size_t out_off,
                                                int Hout, int Wout, size_t out_chan_stride,
                                                int tiles_x, int fmask) {
  __shared__ SynthTile<WV> S;
  const int img = blockIdx.y / 3, c = blockIdx.y % 3;
  wreal* base = ws + img * img_floats;
  const size_t bsz = (size_t)Nh * Nw;
  const double* st = stats + (size_t)img * WL_STATS;
  const wreal thr[3] = {st[WlStats::thr(c, level - 1, 0, L)], st[WlStats::thr(c, level - 1, 1, L)],
                        st[WlStats::thr(c, level - 1, 2, L)]};
  const int ti = blockIdx.x / tiles_x, tj = blockIdx.x - ti * tiles_x;
  const int p0 = ti * ST_O, q0 = tj * ST_O;
  wreal v[ST_O * ST_O / 256];
  synth_tile<WV>(S, base + in_off + (size_t)c * 4 * bsz, bsz, Nh, Nw, p0 / 2, q0 / 2, thr, v, fmask);
  wreal* out = base + out_off + (size_t)c * out_chan_stride;
#pragma unroll
  for (int i = 0; i < ST_O * ST_O / 256; ++i) {
    const int p = p0 + synth_row(i), q = q0 + synth_col(i);
    if (p < Hout && q < Wout) out[(size_t)p * Wout + q] = v[i];
  }
}

// level 1 of all three channels + colour + casts: grid (tiles, n)
template <int WV>
__global__ __launch_bounds__(256) void wl_synth_final(const wreal* __restrict__ ws,
                                                      size_t img_floats,
                                                      const double* __restrict__ stats, int L,
                                                      size_t in_off, int Nh, int Nw, int h, int w,
                                                      int tiles_x, uint8_t* __restrict__ out_u8,
                                                      int64_t row_stride,
                                                      float* __restrict__ out_f32, int fmask) {
  __shared__ SynthTile<WV> S;
  __shared__ uint32_t obuf[ST_O][ST_O * 3 / 4];  // the tile's U8 BGR rows
  constexpr int NV = ST_O * ST_O / 256;
  const int img = blockIdx.y;
  const wreal* base = ws + img * img_floats + in_off;
  const size_t bsz = (size_t)Nh * Nw;
  const double* st = stats + (size_t)img * WL_STATS;
  const bool bad = st[WlStats::FLAG] != 0.0;
  const int ti = blockIdx.x / tiles_x, tj = blockIdx.x - ti * tiles_x;
  const int p0 = ti * ST_O, q0 = tj * ST_O;
  double ych[3][NV];
  // channel c + 1's coefficient loads are issued as soon as channel c is staged in LDS, so they
  // are in flight while channel c is synthesised (the level-1 synthesis is bound by these fp64
  // reads: 37.5 B per output pixel)
  SynthLoad<WV> ld;
  synth_load<WV>(ld, base, bsz, Nh, Nw, p0 / 2, q0 / 2, fmask);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    wreal mn, mx;
    wl_minmax64(st, c, mn, mx);
    const wreal sc = mx - mn;
    const wreal thr[3] = {st[WlStats::thr(c, 0, 0, L)], st[WlStats::thr(c, 0, 1, L)],
                          st[WlStats::thr(c, 0, 2, L)]};
    wreal v[NV];
    synth_run<WV>(S, ld, thr, v, fmask, [&] {
      if (c < 2)
        synth_load<WV>(ld, base + (size_t)(c + 1) * 4 * bsz, bsz, Nh, Nw, p0 / 2, q0 / 2, fmask);
    });
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      // inner denoise_wavelet clip (0.14.2), then * (max - min) + min
      const double x = fmin(fmax((double)v[i], 0.0), 1.0);
      const double yv = x * sc + mn;
      if (c == 0) ych[0][i] = yv;  // (selects: no dynamic register indexing)
      else if (c == 1) ych[1][i] = yv;
      else ych[2][i] = yv;
    }
  }
  uint8_t* ob = reinterpret_cast<uint8_t*>(&obuf[0][0]);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int y = p0 + synth_row(i), x = q0 + synth_col(i);
    // ycbcr2rgb: (arr - [16,128,128]) @ inv(ycbcr_from_rgb).T (numpy.linalg.inv, full precision,
    // fma-chain dot as numpy's matmul), then clip [0, 1]
    const double Y = ych[0][i] - 16.0, Cb = ych[1][i] - 128.0, Cr = ych[2][i] - 128.0;
    double o3[3];
    o3[0] = dot3(Y, Cb, Cr, 0.004566210045662101, 1.1808799897950177e-09, 0.006258928969943937);
    o3[1] = dot3(Y, Cb, Cr, 0.004566210045662101, -0.0015363236860449021, -0.003188110949655707);
    o3[2] = dot3(Y, Cb, Cr, 0.004566210045662101, 0.007910716233554741, 1.1977497040511743e-08);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      double vv = fmin(fmax(o3[c], 0.0), 1.0);
      if (bad) vv = 0.0;
      ob[synth_row(i) * (ST_O * 3) + synth_col(i) * 3 + c] = (uint8_t)(int)(255.0 * vv);
      if (out_f32 && y < h && x < w) out_f32[(((int64_t)img * h + y) * w + x) * 3 + c] = (float)vv;
    }
  }
  if (!out_u8) return;
  __syncthreads();
  uint8_t* orow = out_u8 + (int64_t)img * h * row_stride + (int64_t)q0 * 3;
  if (q0 + ST_O <= w && ((uintptr_t)orow & 3) == 0 && (row_stride & 3) == 0) {
    for (int k = threadIdx.x; k < ST_O * ST_O * 3 / 4; k += 256) {  // whole dwords of full rows
      const int r = k / (ST_O * 3 / 4), d = k - r * (ST_O * 3 / 4);
      if (p0 + r < h)
        reinterpret_cast<uint32_t*>(orow + (int64_t)(p0 + r) * row_stride)[d] = obuf[r][d];
    }
  } else {
    for (int k = threadIdx.x; k < ST_O * ST_O * 3; k += 256) {
      const int r = k / (ST_O * 3), b = k - r * (ST_O * 3);
      if (p0 + r < h && q0 + b / 3 < w) orow[(int64_t)(p0 + r) * row_stride + b] = ob[r * (ST_O * 3) + b];
    }
  }
}

// ---- 6/7 (bior1.5): synthesis, streaming form -------------------------------------------------
// One workgroup per (image, strip of SWo output columns, band of output row pairs) walks down the
// band's coefficient rows; every coefficient is loaded and soft-thresholded once per strip (the
// tiled form staged 1.56x with its halos).  Output pair (2m, 2m+1) x (2n, 2n+1) uses coefficient
// rows m .. m+4 and columns n .. n+4 (pywt upsampling_convolution_valid_sf, c[j] = x[i - j]).
// Per step, coefficient row r:
//   stage    the row's 4 bands x 3 channels over columns [n0, n0 + SWo/2 + 4) into LDS (details
//            soft-thresholded), from a register ring SS_PF rows ahead; every load is issued
//            unconditionally (an fp32 band is read as the 8-byte pair holding its element, the
//            half picked by a select) so no load sits behind a branch and its wait
//   axis 1   thread (c, np): the pair form (synth_full) on row r for output columns 2np, 2np+1:
//            sa = idwt(aa, ad), sd = idwt(da, dd) -> a five-row register ring (shifted by moves)
//   axis 0   once five rows are in: output rows 2m, 2m+1 (m = r - 4) of both columns from the
//            ring; levels >= 2 store the reconstruction (fp64) into the level above's 'aa' slot,
//            level 1 (FINAL) clips, de-normalises and hands Y / Cb / Cr to LDS; there every pixel
//            pair is converted to BGR (inverse YCbCr, clip, U8 / f32) into an LDS row image that
//            the next step stores as whole dwords.
constexpr int SS_MAXT = 256;
constexpr int SS_MAXSW = 168;  // 3 x 84 column pairs <= 256 threads
inline int ss_strips(int Wout) { return (Wout + SS_MAXSW - 1) / SS_MAXSW; }
inline int ss_sw(int Wout) {
  const int st = ss_strips(Wout);
  return ((Wout + st - 1) / st + 3) & ~3;  // strips start on 4 pixels: 12-byte (dword) multiples
}
inline int ss_bands(int n, int Mo, int strips) {  // Mo output row pairs; bands >= 32 pairs
  const int want = (4096 + n * strips - 1) / (n * strips);
  return std::max(1, std::min(want, Mo / 32));
}
// the same on the measured residency of the launched kernel (>= 16 row pairs per band)
inline int ss_bands_occ(int n, int Mo, int strips, const void* kernel, int block) {
  return best_bands((int64_t)n * strips, Mo, 4, (int64_t)cu_count() * occ_wgs(kernel, block), 16);
}
constexpr int SS_PF = 4;                   // coefficient rows in flight ahead of the one staged
constexpr int SS_NCOL = SS_MAXSW / 2 + 4;  // staged coefficient columns (max)
constexpr int SS_ITEMS = 5;                // staging items per thread: 12 x SS_NCOL <= 5 x 256
constexpr int SS_OBW = SS_MAXSW * 3 / 4;   // dwords of one U8 BGR strip row

// T: the synthesis arithmetic.  double: pywt's fp64 (bit-identical to the tiled form's pair
// arithmetic); float: fp32 coefficients, taps, de-normalisation and YCbCr -> RGB (the synthesis
// is continuous in its inputs and no exact zero depends on it: ~3e-7 from the fp64 form on the
// [0, 1] output scale, against the 1e-5 tolerance), with levels >= 2 storing their
// reconstruction as fp32 (the level above reads its 'aa' through WL_FB bit 0).
template <typename T>
__device__ __forceinline__ void synth_bior(const T (&cl)[5], const T (&cd)[5], T& ev, T& od) {
  const T common = fma_t<T>((T)B1, cd[0] - cd[4], (T)B2 * (cd[3] - cd[1]));
  ev = fma_t<T>((T)S2, cl[2] + cd[2], common);
  od = fma_t<T>((T)S2, cl[2] - cd[2], common);
}
// type-exact helpers (the plain builtins are the double versions: a float argument would be
// promoted and the arithmetic done in fp64)
template <typename T>
__device__ __forceinline__ T abs_t(T x) {
  if constexpr (sizeof(T) == 4) return __builtin_fabsf(x);
  else return __builtin_fabs(x);
}
#ifndef IDN_SOFT_MED3  // fp32 soft thresholds as d - med3(d, -t, t) (A/B: 0 = compare / copysign)
#define IDN_SOFT_MED3 1
#endif
template <typename T>
__device__ __forceinline__ T clip01_t(T x) {
  if constexpr (sizeof(T) == 4) return __builtin_fminf(__builtin_fmaxf(x, 0.f), 1.f);
  else return __builtin_fmin(__builtin_fmax(x, 0.0), 1.0);
}
template <typename T>
__device__ __forceinline__ T soft_t(T d, T t) {
  // fp32: d - clamp(d, -t, t), one v_med3 and a subtraction -- the same value (d -+ t rounds as
  // |d| - t does, +0 inside the threshold) for the compare / copysign / select of the fp64 form
  if constexpr (sizeof(T) == 4) {
    if (IDN_SOFT_MED3) return d - __builtin_amdgcn_fmed3f(d, -t, t);
    const T m = abs_t<T>(d) - t;
    return m > 0.f ? __builtin_copysignf(m, d) : 0.f;
  } else {
    const T m = abs_t<T>(d) - t;
    return m > 0.0 ? __builtin_copysign(m, d) : 0.0;
  }
}
template <typename T>
__device__ __forceinline__ T dot3_t(T x0, T x1, T x2, T m0, T m1, T m2) {
  return fma_t<T>(x2, m2, fma_t<T>(x1, m1, x0 * m0));
}

template <bool FINAL, typename T = wreal>
__global__ __launch_bounds__(SS_MAXT) void wl_synth_stream(
    wreal* __restrict__ ws, size_t img_floats, const double* __restrict__ stats, int level, int L,
    size_t in_off, int Nh, int Nw, size_t out_off, int Hout, int Wout, size_t out_chan_stride,
    int fmask, int SWo, int strips, int bands, uint8_t* __restrict__ out_u8, int64_t row_stride,
    float* __restrict__ out_f32) {
  __shared__ T SB[2][12][SS_NCOL];  // staged row: [c * 4 + band][column]
  __shared__ T YB[FINAL ? 3 : 1][2][FINAL ? SS_MAXSW : 1];
  __shared__ uint32_t OB[FINAL ? 2 : 1][FINAL ? SS_OBW : 1];
  __shared__ T TH[12];  // soft thresholds by [c * 4 + band] (0 for aa)
  const int img = blockIdx.z;
  const int strip = (int)blockIdx.x % strips, band = (int)blockIdx.x / strips;
  const int x0 = strip * SWo, n0 = x0 / 2;
  const int Mo = (Hout + 1) / 2;  // output row pairs
  const int ma = (int)((int64_t)band * Mo / bands), mb = (int)((int64_t)(band + 1) * Mo / bands);
  const int t = threadIdx.x;
  wreal* base = ws + img * img_floats;
  const double* st = stats + (size_t)img * WL_STATS;
  const size_t bsz = (size_t)Nh * Nw;
  const int ncol = SWo / 2 + 4;
  const int nitems = 12 * ncol;
  // staging items k = t + 256 u -> (band cb, column); items past the end load a valid address
  const wreal* ip[SS_ITEMS];
  int icb[SS_ITEMS], icl[SS_ITEMS];
  uint32_t fb = 0;  // bit u: item u's band is stored fp32
#pragma unroll
  for (int u = 0; u < SS_ITEMS; ++u) {
    const int k = t + SS_MAXT * u;
    const bool ok = k < nitems;
    const int cb = ok ? k / ncol : 0;
    icb[u] = ok ? cb : -1;
    icl[u] = ok ? k - cb * ncol : 0;
    ip[u] = base + in_off + (size_t)cb * bsz;
    fb |= (uint32_t)wl_fband(fmask, cb & 3) << u;
  }
  if (t < 12) TH[t] = (T)((t & 3) ? st[WlStats::thr(t >> 2, level - 1, (t & 3) - 1, L)] : 0.0);
  __syncthreads();
  // coefficients past the band's end feed only outputs past the level's valid length (never
  // stored): clamped reads keep them finite
  auto load = [&](int r, double (&v)[SS_ITEMS], uint32_t& odd) {
    const size_t rb = (size_t)min(r, Nh - 1) * Nw;
    odd = 0;
#pragma unroll
    for (int u = 0; u < SS_ITEMS; ++u) {
      const size_t e = rb + min(n0 + icl[u], Nw - 1);
      const uint32_t f = (fb >> u) & 1u;
      v[u] = ip[u][e >> f];
      odd |= ((uint32_t)e & f) << u;
    }
  };
  // ---- axis roles: thread (c, np)
  const int half = SWo / 2;
  const bool ct = t < 3 * half;
  const int c = ct ? t / half : 0, np = ct ? t - c * half : 0;
  T ring[5][4];  // coefficient rows r-4 .. r of (sa(2np), sa(2np+1), sd(2np), sd(2np+1))
#pragma unroll
  for (int s5 = 0; s5 < 5; ++s5)
#pragma unroll
    for (int q = 0; q < 4; ++q) ring[s5][q] = (T)0;
  T mn = 0, sc = 0;
  bool bad = false;
  if (FINAL) {
    wreal mn64, mx64;
    wl_minmax64(st, c, mn64, mx64);
    sc = (T)(mx64 - mn64);
    mn = (T)mn64;
    bad = st[WlStats::FLAG] != 0.0;
  }
  // FINAL: the strip's U8 row bytes, stored whole dwords when the rows are dword aligned
  const int nb = 3 * min(SWo, Wout - x0);
  const bool al = ((uintptr_t)out_u8 & 3) == 0 && (row_stride & 3) == 0;
  auto flush = [&](int m) {
    if (!out_u8) return;
    const int nw = SWo * 3 / 4;
    for (int k = t; k < 2 * nw; k += SS_MAXT) {
      const int rr2 = k >= nw, d = k - rr2 * nw;
      const int y = 2 * m + rr2;
      if (y >= Hout || 4 * d >= nb) continue;
      uint8_t* orow = out_u8 + ((int64_t)img * Hout + y) * row_stride + (int64_t)x0 * 3;
      const uint32_t wv = OB[rr2][d];
      if (al && 4 * d + 4 <= nb) {
        reinterpret_cast<uint32_t*>(orow)[d] = wv;
      } else {
        for (int bi = 4 * d; bi < min(4 * d + 4, nb); ++bi) orow[bi] = (uint8_t)(wv >> (8 * (bi & 3)));
      }
    }
  };
  const int r0 = ma, R = (mb - ma) + 4;  // coefficient rows r0 .. r0 + R - 1
  double pf[SS_PF][SS_ITEMS];
  uint32_t podd[SS_PF];
#pragma unroll
  for (int f = 0; f < SS_PF; ++f)
    if (f < R) load(r0 + f, pf[f], podd[f]);
  for (int s0 = 0; s0 < R; s0 += SS_PF) {
#pragma unroll
    for (int rs = 0; rs < SS_PF; ++rs) {
      const int sidx = s0 + rs;
      if (sidx >= R) break;
      const int r = r0 + sidx, buf = sidx & 1;
      // stage row r (details soft-thresholded; thr = 0 keeps aa), refill its prefetch slot
#pragma unroll
      for (int u = 0; u < SS_ITEMS; ++u) {
        const wreal x = pf[rs][u];
        const unsigned long long bits = (unsigned long long)__double_as_longlong(x);
        const float h = __uint_as_float((uint32_t)(((podd[rs] >> u) & 1u) ? bits >> 32 : bits));
        const T xt = ((fb >> u) & 1u) ? (T)h : (T)x;
        if (icb[u] >= 0) SB[buf][icb[u]][icl[u]] = soft_t<T>(xt, TH[icb[u]]);
      }
      if (sidx + SS_PF < R) load(r + SS_PF, pf[rs], podd[rs]);
      __syncthreads();
      if (FINAL && sidx >= 5) flush(r - 5);  // the previous step's U8 rows
      if (ct) {
#pragma unroll
        for (int pb = 0; pb < 2; ++pb) {  // sa: aa (lowpass) / ad (highpass); sd: da / dd
          const T* lo = SB[buf][c * 4 + 2 * pb];
          const T* hi = SB[buf][c * 4 + 2 * pb + 1];
          T cl[5], cd[5];
#pragma unroll
          for (int j = 0; j < 5; ++j) {  // c[j] = column np + 4 - j
            cl[j] = lo[np + 4 - j];
            cd[j] = hi[np + 4 - j];
          }
          synth_bior<T>(cl, cd, ring[4][2 * pb], ring[4][2 * pb + 1]);
        }
      }
      if (sidx >= 4) {
        const int m = r - 4;  // output row pair 2m, 2m+1
        T v[2][2];            // [row][column]
#pragma unroll
        for (int col = 0; col < 2; ++col) {
          T cl[5], cd[5];
#pragma unroll
          for (int j = 0; j < 5; ++j) {  // c[j] = coefficient row m + 4 - j
            cl[j] = ring[4 - j][col];
            cd[j] = ring[4 - j][2 + col];
          }
          synth_bior<T>(cl, cd, v[0][col], v[1][col]);
        }
        if (!FINAL) {
          T* out = reinterpret_cast<T*>(base + out_off + (size_t)c * out_chan_stride);
          const int x = x0 + 2 * np;
#pragma unroll
          for (int rr2 = 0; rr2 < 2; ++rr2) {
            const int y = 2 * m + rr2;
            if (!ct || y >= Hout || x >= Wout) continue;
            T* o = out + (size_t)y * Wout + x;
            if (x + 1 < Wout && ((uintptr_t)o & (2 * sizeof(T) - 1)) == 0) {
              if constexpr (sizeof(T) == 4) *reinterpret_cast<float2*>(o) = make_float2(v[rr2][0], v[rr2][1]);
              else *reinterpret_cast<double2*>(o) = make_double2(v[rr2][0], v[rr2][1]);
            } else {
              o[0] = v[rr2][0];
              if (x + 1 < Wout) o[1] = v[rr2][1];
            }
          }
        } else {
          // inner clip (0.14.2) and de-normalisation
          if (ct) {
#pragma unroll
            for (int rr2 = 0; rr2 < 2; ++rr2)
#pragma unroll
              for (int col = 0; col < 2; ++col)
                YB[c][rr2][2 * np + col] = clip01_t<T>(v[rr2][col]) * sc + mn;
          }
          __syncthreads();
          // pixel pairs: thread q -> row q / half, pixels 2 (q % half), +1
          if (t < 2 * half) {
            const int rr2 = t >= half, pp = t - rr2 * half;
            const int y = 2 * m + rr2;
            uint16_t* ob = reinterpret_cast<uint16_t*>(&OB[rr2][0]) + 3 * pp;
            uint32_t b6[2] = {0u, 0u};  // the pair's 6 bytes
#pragma unroll
            for (int p = 0; p < 2; ++p) {
              const int xx = 2 * pp + p;
              // ycbcr2rgb: (arr - [16,128,128]) @ inv(ycbcr_from_rgb).T (fma-chain dot), clip
              const T Y = YB[0][rr2][xx] - (T)16, Cb = YB[1][rr2][xx] - (T)128,
                      Cr = YB[2][rr2][xx] - (T)128;
              T o3[3];
              o3[0] = dot3_t<T>(Y, Cb, Cr, (T)0.004566210045662101, (T)1.1808799897950177e-09,
                                (T)0.006258928969943937);
              o3[1] = dot3_t<T>(Y, Cb, Cr, (T)0.004566210045662101, (T)-0.0015363236860449021,
                                (T)-0.003188110949655707);
              o3[2] = dot3_t<T>(Y, Cb, Cr, (T)0.004566210045662101, (T)0.007910716233554741,
                                (T)1.1977497040511743e-08);
#pragma unroll
              for (int k3 = 0; k3 < 3; ++k3) {
                T vv = clip01_t<T>(o3[k3]);
                if (bad) vv = (T)0;
                const int bi = 3 * p + k3;
                b6[bi >> 2] |= (uint32_t)(uint8_t)(int)((T)255 * vv) << (8 * (bi & 3));
                if (out_f32 && y < Hout && x0 + xx < Wout)
                  out_f32[(((int64_t)img * Hout + y) * Wout + x0 + xx) * 3 + k3] = (float)vv;
              }
            }
            ob[0] = (uint16_t)b6[0];
            ob[1] = (uint16_t)(b6[0] >> 16);
            ob[2] = (uint16_t)b6[1];
          }
        }
      }
#pragma unroll
      for (int s5 = 0; s5 < 4; ++s5)
#pragma unroll
        for (int q = 0; q < 4; ++q) ring[s5][q] = ring[s5 + 1][q];
    }
  }
  if (FINAL && R >= 5) {
    __syncthreads();
    flush(r0 + R - 5);
  }
}

// ---- 7b (bior1.5): level-1 synthesis, fp32, three channels per thread ----------------------------
// wl_synth_stream<true, float> splits a column pair's three channels over three threads, so the
// YCbCr -> RGB step needs a second barrier per coefficient row (and 48 register moves shift its
// ring).  Here thread np owns output columns 2np, 2np+1 of ALL three channels: one barrier per
// coefficient row, and the five-row ring rotates by index (the loop is unrolled by 10 = lcm(5,
// S3_PF)).  Thread t < SWo/2 + 4 stages coefficient column n0 + t of the 12 (channel, band) rows;
// FM (compile time) says which bands are fp32 in HBM (aa / ad / da; the finest dd is fp64), so each
// thread keeps S3_PF rows of raw loads in flight with no per-item selects.  The U8 rows go through
// an LDS row image flushed as dwords after the next step's barrier.  Arithmetic as
// wl_synth_stream<.., float>.
constexpr int S3_T = 256;
constexpr int S3_MAXSW = 2 * (S3_T - 4);  // 504 output columns per strip
constexpr int S3_PF = 1;                  // coefficient rows in flight ahead of the one staged
inline int s3_strips(int Wout) { return (Wout + S3_MAXSW - 1) / S3_MAXSW; }
inline int s3_sw(int Wout) {
  const int st = s3_strips(Wout);
  return ((Wout + st - 1) / st + 3) & ~3;  // multiple of 4 pixels (12-byte strip starts)
}
template <int FM>
struct S3Raw {  // one coefficient row of one staged column: the 12 (channel, band) values
  float f[3][4];   // fp32 bands, by s3_slot (unused slots are never written)
  double d[3][2];  // fp64 bands
};
template <int FM>
__device__ __forceinline__ constexpr int s3_slot(int b) {  // slot of band b in f (fp32) or d (fp64)
  int k = 0;
  for (int q = 0; q < b; ++q) k += (((FM >> q) & 1) == ((FM >> b) & 1)) ? 1 : 0;
  return k;
}
// FINAL = false (levels >= 2): the same structure without the colour step; the three channels'
// reconstructions go to the level below's 'aa' slots as fp32 (out_off + c * out_chan_stride).
template <int FM, bool FINAL = true>
__global__ __launch_bounds__(S3_T, IDN_S3_WPE) void wl_synth_final3(
    wreal* __restrict__ ws, size_t img_floats, const double* __restrict__ stats, int L,
    size_t in_off, int Nh, int Nw, int Hout, int Wout, int SWo, int strips, int bands,
    uint8_t* __restrict__ out_u8, int64_t row_stride, float* __restrict__ out_f32, int level = 1,
    size_t out_off = 0, size_t out_chan_stride = 0) {
  static_assert(!FINAL || (FM & 0b0110) == 0b0110, "level 1: ad / da fp32");
  __shared__ float SB[2][12][S3_T];                  // staged row: [c * 4 + band][column]
  __shared__ uint32_t OB[FINAL ? 2 : 1][2][FINAL ? S3_MAXSW * 3 / 4 : 1];  // U8 rows (FINAL)
  __shared__ float TH[12];
  const int img = blockIdx.z;
  const int strip = (int)blockIdx.x % strips, band = (int)blockIdx.x / strips;
  const int x0 = strip * SWo, n0 = x0 / 2;
  const int Mo = (Hout + 1) / 2;
  const int ma = (int)((int64_t)band * Mo / bands), mb = (int)((int64_t)(band + 1) * Mo / bands);
  const int t = threadIdx.x;
  const wreal* base = ws + img * img_floats + in_off;
  const double* st = stats + (size_t)img * WL_STATS;
  const size_t bsz = (size_t)Nh * Nw;
  const int half = SWo / 2, ncol = half + 4;
  if (t < 12) TH[t] = (float)((t & 3) ? st[WlStats::thr(t >> 2, level - 1, (t & 3) - 1, L)] : 0.0);
  float mn[3], sc[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    wreal a, b;
    wl_minmax64(st, c, a, b);
    mn[c] = (float)a;
    sc[c] = (float)(b - a);
  }
  const bool bad = st[WlStats::FLAG] != 0.0;
  // staging role: coefficient column n0 + t (clamped: columns past the band's end feed only
  // outputs past the valid width, never stored)
  const bool stg = t < ncol;
  const int scol = min(n0 + t, Nw - 1);
  auto load = [&](int r, S3Raw<FM>& R) {
    const size_t e = (size_t)min(r, Nh - 1) * Nw + scol;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const wreal* X = base + (size_t)(c * 4 + b) * bsz;
        if ((FM >> b) & 1) R.f[c][s3_slot<FM>(b)] = reinterpret_cast<const float*>(X)[e];
        else R.d[c][s3_slot<FM>(b)] = X[e];
      }
  };
  // compute role: column pair np (outputs x0 + 2np, +1), all three channels
  const bool cmp = t < half;
  const int np = t;
  float ring[3][5][4];  // [c][slot = coefficient row % 5][sa(2np), sa(2np+1), sd(2np), sd(2np+1)]
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int s5 = 0; s5 < 5; ++s5)
#pragma unroll
      for (int q = 0; q < 4; ++q) ring[c][s5][q] = 0.f;
  const int nb = 3 * min(SWo, Wout - x0);  // U8 bytes of the strip's rows
  const bool al = ((uintptr_t)out_u8 & 3) == 0 && (row_stride & 3) == 0;
  auto flush = [&](int m, int ob) {  // output rows 2m, 2m+1 from OB[ob]
    if (!FINAL || !out_u8) return;
    const int nw = (nb + 3) / 4;
    for (int k = t; k < 2 * nw; k += S3_T) {
      const int rr2 = k >= nw, d = k - rr2 * nw;
      const int y = 2 * m + rr2;
      if (y >= Hout) continue;
      uint8_t* orow = out_u8 + ((int64_t)img * Hout + y) * row_stride + (int64_t)x0 * 3;
      const uint32_t wv = OB[ob][rr2][d];
      if (al && 4 * d + 4 <= nb) {
        reinterpret_cast<uint32_t*>(orow)[d] = wv;
      } else {
        for (int bi = 4 * d; bi < min(4 * d + 4, nb); ++bi) orow[bi] = (uint8_t)(wv >> (8 * (bi & 3)));
      }
    }
  };
  __syncthreads();  // TH
  const int r0 = ma, R = (mb - ma) + 4;  // coefficient rows r0 .. r0 + R - 1
  // IDN_S3_PAD (A/B builds): wl_dwt_stream's ring form -- unconditional refills, the last iteration
  // padded instead of left by a break
  S3Raw<FM> pf[S3_PF];
  if (stg || IDN_S3_PAD) {
#pragma unroll
    for (int f = 0; f < S3_PF; ++f)
      if (IDN_S3_PAD || f < R) load(r0 + f, pf[f]);
  }
  for (int s0 = 0; s0 < R; s0 += 10) {
#pragma unroll
    for (int rs = 0; rs < 10; ++rs) {
      const int sidx = s0 + rs;
      if (!IDN_S3_PAD && sidx >= R) break;
      const int r = r0 + sidx, buf = sidx & 1, slot = rs % 5;
      if (stg) {  // stage row r (details soft-thresholded), refill its prefetch slot
        const S3Raw<FM>& q = pf[rs % S3_PF];
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const float x = ((FM >> b) & 1) ? q.f[c][s3_slot<FM>(b)] : (float)q.d[c][s3_slot<FM>(b)];
            SB[buf][c * 4 + b][t] = b ? soft_t<float>(x, TH[c * 4 + b]) : x;
          }
        if (!IDN_S3_PAD && sidx + S3_PF < R) load(r + S3_PF, pf[rs % S3_PF]);
      }
      if (IDN_S3_PAD) {
        load(r + S3_PF, pf[rs % S3_PF]);
        if (sidx >= R) continue;
      }
      __syncthreads();
      if (sidx >= 5) flush(r - 5, buf ^ 1);  // the previous step's U8 rows
      if (cmp) {
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
          for (int pb = 0; pb < 2; ++pb) {  // sa: aa / ad; sd: da / dd
            const float* lo = SB[buf][c * 4 + 2 * pb];
            const float* hi = SB[buf][c * 4 + 2 * pb + 1];
            float cl[5], cd[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) {  // c[j] = column np + 4 - j
              cl[j] = lo[np + 4 - j];
              cd[j] = hi[np + 4 - j];
            }
            synth_bior<float>(cl, cd, ring[c][slot][2 * pb], ring[c][slot][2 * pb + 1]);
          }
      }
      if (!FINAL && sidx >= 4 && cmp) {  // reconstruction of the level below, fp32
        const int m = r - 4;
        const int x = x0 + 2 * np;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          float v[2][2];  // [row][column]
#pragma unroll
          for (int col = 0; col < 2; ++col) {
            float cl[5], cd[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) {
              cl[j] = ring[c][(rs + 5 - j) % 5][col];
              cd[j] = ring[c][(rs + 5 - j) % 5][2 + col];
            }
            synth_bior<float>(cl, cd, v[0][col], v[1][col]);
          }
          float* out = reinterpret_cast<float*>(ws + img * img_floats + out_off +
                                                (size_t)c * out_chan_stride);
#pragma unroll
          for (int rr2 = 0; rr2 < 2; ++rr2) {
            const int y = 2 * m + rr2;
            if (y >= Hout || x >= Wout) continue;
            float* o = out + (size_t)y * Wout + x;
            if (x + 1 < Wout && ((uintptr_t)o & 7) == 0) {
              *reinterpret_cast<float2*>(o) = make_float2(v[rr2][0], v[rr2][1]);
            } else {
              o[0] = v[rr2][0];
              if (x + 1 < Wout) o[1] = v[rr2][1];
            }
          }
        }
      }
      if (FINAL && sidx >= 4 && cmp) {
        const int m = r - 4;  // output row pair 2m, 2m+1
        float Yv[3][2][2];    // [c][row][column], de-normalised
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
          for (int col = 0; col < 2; ++col) {
            float cl[5], cd[5], v0, v1;
#pragma unroll
            for (int j = 0; j < 5; ++j) {  // c[j] = coefficient row m + 4 - j
              cl[j] = ring[c][(rs + 5 - j) % 5][col];
              cd[j] = ring[c][(rs + 5 - j) % 5][2 + col];
            }
            synth_bior<float>(cl, cd, v0, v1);
            Yv[c][0][col] = clip01_t<float>(v0) * sc[c] + mn[c];
            Yv[c][1][col] = clip01_t<float>(v1) * sc[c] + mn[c];
          }
#pragma unroll
        for (int rr2 = 0; rr2 < 2; ++rr2) {
          const int y = 2 * m + rr2;
          uint32_t b6[2] = {0u, 0u};  // the pair's 6 bytes
          float o6[6];
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const float Y = Yv[0][rr2][p] - 16.f, Cb = Yv[1][rr2][p] - 128.f, Cr = Yv[2][rr2][p] - 128.f;
            float o3[3];
            // (float) of the fp64 constants, as wl_synth_stream (a float literal of the decimal
            // can round differently: double rounding)
            o3[0] = dot3_t<float>(Y, Cb, Cr, (float)0.004566210045662101, (float)1.1808799897950177e-09,
                                  (float)0.006258928969943937);
            o3[1] = dot3_t<float>(Y, Cb, Cr, (float)0.004566210045662101, (float)-0.0015363236860449021,
                                  (float)-0.003188110949655707);
            o3[2] = dot3_t<float>(Y, Cb, Cr, (float)0.004566210045662101, (float)0.007910716233554741,
                                  (float)1.1977497040511743e-08);
#pragma unroll
            for (int k3 = 0; k3 < 3; ++k3) {
              float vv = clip01_t<float>(o3[k3]);
              if (bad) vv = 0.f;
              const int bi = 3 * p + k3;
              o6[bi] = vv;
              b6[bi >> 2] |= (uint32_t)(uint8_t)(int)(255.f * vv) << (8 * (bi & 3));
            }
          }
          uint16_t* ob = reinterpret_cast<uint16_t*>(&OB[buf][rr2][0]) + 3 * np;
          ob[0] = (uint16_t)b6[0];
          ob[1] = (uint16_t)(b6[0] >> 16);
          ob[2] = (uint16_t)b6[1];
          const int x = x0 + 2 * np;
          if (out_f32 && y < Hout && x < Wout) {
            float* o = out_f32 + (((int64_t)img * Hout + y) * Wout + x) * 3;
            if (x + 1 < Wout && ((uintptr_t)o & 7) == 0) {
              reinterpret_cast<float2*>(o)[0] = make_float2(o6[0], o6[1]);
              reinterpret_cast<float2*>(o)[1] = make_float2(o6[2], o6[3]);
              reinterpret_cast<float2*>(o)[2] = make_float2(o6[4], o6[5]);
            } else {
#pragma unroll
              for (int k = 0; k < 6; ++k)
                if (k < 3 || x + 1 < Wout) o[k] = o6[k];
            }
          }
        }
      }
    }
  }
  if (FINAL && R >= 5) {
    __syncthreads();
    flush(r0 + R - 5, (R - 1) & 1);
  }
}

// ---- Haar fast path: every level is local to a 2^L x 2^L block ---------------------------------
// For db1 with h and w divisible by 2^L, pywt's 'symmetric' extension never triggers and level l's
// coefficients of a 2^L x 2^L block depend on that block alone.  So the whole denoiser runs as
//   wl_color_minmax -> wl_haar_analyze -> wl_sumsq -> wl_median -> wl_thresh -> wl_haar_synth
// where wl_haar_analyze reads the image once and writes only the finest dd band (for sigma) and
// per-workgroup sums of squares of every detail band, and wl_haar_synth reads the image again,
// recomputes the analysis of its block, thresholds, synthesises all levels, converts back to
// RGB and stores the U8 / f32 output: no fp64 band ever makes a round trip through HBM except dd1.
// The arithmetic is op for op the general path's (multiply then add, axis 0 then axis 1; the
// synthesis sums A, AD, DA, DD in that order), so the coefficients are bitwise the same.
constexpr int WLH_WG = 128;  // threads per workgroup (wl_layout sizes the partials for it)
constexpr int WLH_IT = 4;    // wl_haar_analyze: chunks of WLH_WG sub-blocks per thread

// pywt dwt2 of one 2x2 group, rows 2i / 2i+1 (x0j / x1j), columns 2j / 2j+1
__device__ __forceinline__ void haar2x2(wreal x00, wreal x01, wreal x10, wreal x11, wreal& aa,
                                        wreal& ad, wreal& da, wreal& dd) {
  const wreal lo0 = S2 * x10 + S2 * x00, lo1 = S2 * x11 + S2 * x01;    // axis 0 low
  const wreal hi0 = -S2 * x10 + S2 * x00, hi1 = -S2 * x11 + S2 * x01;  // axis 0 high
  aa = S2 * lo1 + S2 * lo0;
  ad = -S2 * lo1 + S2 * lo0;
  da = S2 * hi1 + S2 * hi0;
  dd = -S2 * hi1 + S2 * hi0;
}
// pywt idwt2 of one coefficient quadruple to output (r, s) of its 2x2 group (details thresholded)
__device__ __forceinline__ wreal ihaar(wreal A, wreal AD, wreal DA, wreal DD, int r, int s) {
  const wreal fd = r ? -S2 : S2, gd = s ? -S2 : S2;
  wreal acc = 0;
  acc = acc + S2 * S2 * A;
  acc = acc + S2 * gd * AD;
  acc = acc + fd * S2 * DA;
  acc = acc + fd * gd * DD;
  return acc;
}

// one row of 4 pixels (x .. x+3) of image img, normalised YCbCr per channel: v[s][c]
__device__ __forceinline__ void haar_row4(const uint8_t* __restrict__ src,
                                          const double* __restrict__ in64, int img, int h, int w,
                                          int64_t row_stride, int y, int x, const wreal (&mn)[3],
                                          const wreal (&inv)[3], wreal (&v)[4][3]) {
  double px[4][3];
  if (in64) {
    const double* p = in64 + (((int64_t)img * h + y) * w + x) * 3;
#pragma unroll
    for (int k = 0; k < 12; ++k) px[k / 3][k % 3] = p[k];
  } else {  // 12 bytes, 4-byte aligned (checked on the host): three dword loads
    const uint32_t* p = reinterpret_cast<const uint32_t*>(src + (int64_t)img * h * row_stride +
                                                          (int64_t)y * row_stride + (int64_t)x * 3);
    const uint32_t d[3] = {p[0], p[1], p[2]};
#pragma unroll
    for (int k = 0; k < 12; ++k)
      px[k / 3][k % 3] = (double)((d[k >> 2] >> (8 * (k & 3))) & 0xFFu) * (1.0 / 255.0);
  }
  // the synthesis is continuous in the coefficients: a reciprocal multiply (<= 1 ulp from the
  // quotient) is enough here; sigma's exact zeros come from wl_haar_analyze's exact quotients
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const wreal rcp = 1.0 / inv[c];
#pragma unroll
    for (int s = 0; s < 4; ++s) v[s][c] = (ycbcr_c(px[s], c) - mn[c]) * rcp;
  }
}

// Work split: one thread per 4x4 sub-block (levels 1 and 2 in registers); for L = 3 the four
// threads of an 8x8 block are consecutive lanes and level 3 runs on their level-2 approximations
// gathered by shuffles (redundantly in all four; only sub-block 0 counts its squares).
template <int L>
struct HaarSplit {
  static constexpr int B = 1 << L;          // block side
  static constexpr int SB = B < 4 ? B : 4;  // sub-block side per thread
  static constexpr int NS = (B / SB) * (B / SB);
  static constexpr int QS = SB / 2;         // level-1 groups per sub-block side
};

// channel c of one row of 4 pixels (x .. x+3), normalised: v[s]
__device__ __forceinline__ void haar_row4_c(const uint8_t* __restrict__ src,
                                            const double* __restrict__ in64, int img, int h, int w,
                                            int64_t row_stride, int y, int x, int c, wreal mn,
                                            wreal inv, wreal (&v)[4]) {
  double px[4][3];
  if (in64) {
    const double* p = in64 + (((int64_t)img * h + y) * w + x) * 3;
#pragma unroll
    for (int k = 0; k < 12; ++k) px[k / 3][k % 3] = p[k];
  } else {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(src + (int64_t)img * h * row_stride +
                                                          (int64_t)y * row_stride + (int64_t)x * 3);
    const uint32_t d[3] = {p[0], p[1], p[2]};
#pragma unroll
    for (int k = 0; k < 12; ++k)
      px[k / 3][k % 3] = (double)((d[k >> 2] >> (8 * (k & 3))) & 0xFFu) * (1.0 / 255.0);
  }
  // (Y - min) / (max - min) correctly rounded without a division per value: q0 = a * (1/b),
  // q1 = q0 + (a - q0 b)(1/b) with exact fma residuals (Markstein) -- bitwise the IEEE quotient
  // (also checked over every u8 triple for 24 channel ranges: tools/check_div.c)
  const wreal rcp = 1.0 / inv;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const wreal a = ycbcr_c(px[s], c) - mn;
    const wreal q0 = a * rcp;
    v[s] = __fma_rn(__fma_rn(-q0, inv, a), rcp, q0);
  }
}

// level 1 of channel c of one thread's 4x4 sub-block (L >= 2)
__device__ __forceinline__ void haar_sub4_c(const uint8_t* __restrict__ src,
                                            const double* __restrict__ in64, int img, int h, int w,
                                            int64_t row_stride, int y0, int x0, int c, wreal mn,
                                            wreal inv, wreal (&a1)[4], wreal (&d1)[3][4]) {
#pragma unroll
  for (int qy = 0; qy < 2; ++qy) {
    wreal r0[4], r1[4];
    haar_row4_c(src, in64, img, h, w, row_stride, y0 + 2 * qy, x0, c, mn, inv, r0);
    haar_row4_c(src, in64, img, h, w, row_stride, y0 + 2 * qy + 1, x0, c, mn, inv, r1);
#pragma unroll
    for (int qx = 0; qx < 2; ++qx) {
      const int k = qy * 2 + qx;
      haar2x2(r0[2 * qx], r0[2 * qx + 1], r1[2 * qx], r1[2 * qx + 1], a1[k], d1[0][k], d1[1][k],
              d1[2][k]);
    }
  }
}

// level 1 of one thread's sub-block, all channels: a1[c][k] approximations, d1[c][band][k] details
template <int L>
__device__ __forceinline__ void haar_sub_analysis(
    const uint8_t* __restrict__ src, const double* __restrict__ in64, int img, int h, int w,
    int64_t row_stride, int y0, int x0, const wreal (&mn)[3], const wreal (&inv)[3],
    wreal (&a1)[3][HaarSplit<L>::QS * HaarSplit<L>::QS],
    wreal (&d1)[3][3][HaarSplit<L>::QS * HaarSplit<L>::QS]) {
  using HS = HaarSplit<L>;
#pragma unroll
  for (int qy = 0; qy < HS::QS; ++qy) {
    wreal r0[4][3], r1[4][3];
    if constexpr (HS::SB == 4) {
      haar_row4(src, in64, img, h, w, row_stride, y0 + 2 * qy, x0, mn, inv, r0);
      haar_row4(src, in64, img, h, w, row_stride, y0 + 2 * qy + 1, x0, mn, inv, r1);
    } else {  // 2x2 sub-block (L = 1): two pixels per row
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        double p0[3], p1[3];
        load_rgb64(src, in64, img, h, w, row_stride, y0 + 2 * qy, x0 + s, p0);
        load_rgb64(src, in64, img, h, w, row_stride, y0 + 2 * qy + 1, x0 + s, p1);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          r0[s][c] = (ycbcr_c(p0, c) - mn[c]) / inv[c];
          r1[s][c] = (ycbcr_c(p1, c) - mn[c]) / inv[c];
        }
      }
    }
#pragma unroll
    for (int qx = 0; qx < HS::QS; ++qx)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int k = qy * HS::QS + qx;
        haar2x2(r0[2 * qx][c], r0[2 * qx + 1][c], r1[2 * qx][c], r1[2 * qx + 1][c], a1[c][k],
                d1[c][0][k], d1[c][1][k], d1[c][2][k]);
      }
  }
}

template <int L>
__global__ __launch_bounds__(WLH_WG) void wl_haar_analyze(
    const uint8_t* __restrict__ src, const double* __restrict__ in64, int h, int w,
    int64_t row_stride, wreal* __restrict__ ws, size_t img_floats, size_t dd_off,
    const double* __restrict__ stats, double* __restrict__ part, size_t part_per_img) {
  using HS = HaarSplit<L>;
  constexpr int B = HS::B, QS = HS::QS;
  const int img = blockIdx.y;
  const int nbx = w / B, nblk = nbx * (h / B);
  const double* st = stats + (size_t)img * WL_STATS;
  __shared__ double red[3 * L * 3][WLH_WG / 64];
  const size_t W1 = (size_t)(w / 2), bsz = (size_t)(h / 2) * W1;
  // one channel at a time (keeps the live state to one channel's coefficients and sums)
#pragma unroll 1
  for (int c = 0; c < 3; ++c) {
    wreal mn, mx;
    wl_minmax64(st, c, mn, mx);
    const wreal inv = mx - mn;
    double sq[L][3];
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int b = 0; b < 3; ++b) sq[l][b] = 0.0;
    // WLH_IT chunks of WLH_WG sub-blocks per thread, summed in registers before the one wave
    // reduction per channel (the reductions, not the arithmetic, dominated at one chunk)
#pragma unroll 1
    for (int it = 0; it < WLH_IT; ++it) {
      const int tid = (blockIdx.x * WLH_IT + it) * WLH_WG + threadIdx.x;
      const int blk = tid / HS::NS, sub = tid % HS::NS;
      const bool act = blk < nblk;  // uniform over each block's NS consecutive lanes
      int y0 = 0, x0 = 0;
      if (act) {
        const int by = blk / nbx, bx = blk - by * nbx;
        const int sy = sub / (B / HS::SB), sx = sub % (B / HS::SB);
        y0 = by * B + sy * HS::SB;
        x0 = bx * B + sx * HS::SB;
      }
      wreal a2 = 0;
      if (act) {
        wreal a1[QS * QS], d1[3][QS * QS];
        if constexpr (QS == 2) {
          haar_sub4_c(src, in64, img, h, w, row_stride, y0, x0, c, mn, inv, a1, d1);
        } else {  // L = 1: a 2x2 block per thread
          wreal r[2][2];
#pragma unroll
          for (int rr = 0; rr < 2; ++rr)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
              double px[3];
              load_rgb64(src, in64, img, h, w, row_stride, y0 + rr, x0 + ss, px);
              r[rr][ss] = (ycbcr_c(px, c) - mn) / inv;
            }
          haar2x2(r[0][0], r[0][1], r[1][0], r[1][1], a1[0], d1[0][0], d1[1][0], d1[2][0]);
        }
        // the finest dd is kept only as its fine-bin code (0: exact zero, else wl_fbin + 1): the
        // sigma median recomputes the exact values of the one or two bins it needs
        uint16_t* cdp = reinterpret_cast<uint16_t*>(ws + img * img_floats + dd_off +
                                                    (size_t)c * 4 * bsz + 3 * bsz);
#pragma unroll
        for (int k = 0; k < QS * QS; ++k) {
#pragma unroll
          for (int b = 0; b < 3; ++b) sq[0][b] += d1[b][k] * d1[b][k];
          const unsigned long long key = absbits(d1[2][k]);
          cdp[(size_t)(y0 / 2 + k / QS) * W1 + x0 / 2 + k % QS] =
              (uint16_t)(key ? wl_fbin(key) + 1 : 0);
        }
        if constexpr (L >= 2) {  // level 2 on the thread's 2x2 level-1 approximations
          wreal ad, da, dd;
          haar2x2(a1[0], a1[1], a1[2], a1[3], a2, ad, da, dd);
          sq[1][0] += ad * ad;
          sq[1][1] += da * da;
          sq[1][2] += dd * dd;
        }
      }
      if constexpr (L == 3) {  // level 3 across the block's 4 lanes (all lanes take part)
        const int base = (threadIdx.x & 63) & ~3;
        const wreal x00 = __shfl(a2, base), x01 = __shfl(a2, base + 1);
        const wreal x10 = __shfl(a2, base + 2), x11 = __shfl(a2, base + 3);
        wreal aa, ad, da, dd;
        haar2x2(x00, x01, x10, x11, aa, ad, da, dd);
        if (act && sub == 0) {
          sq[2][0] += ad * ad;
          sq[2][1] += da * da;
          sq[2][2] += dd * dd;
        }
      }
    }
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        double v = sq[l][b];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((threadIdx.x & 63) == 0) red[(c * L + l) * 3 + b][threadIdx.x >> 6] = v;
      }
  }
  __syncthreads();
  // workgroup sums of squares in a fixed order (wave shuffles, then the two waves)
  if (threadIdx.x < 3 * L * 3) {
    const int k = threadIdx.x, b = k % 3, l = (k / 3) % L, c = k / (3 * L);
    double t = red[k][0];
#pragma unroll
    for (int wv = 1; wv < WLH_WG / 64; ++wv) t += red[k][wv];
    part[img * part_per_img + (size_t)(c * 3 + b) * (part_per_img / 9) + (size_t)l * gridDim.x +
         blockIdx.x] = t;
  }
}

template <int L>
__global__ __launch_bounds__(WLH_WG) __attribute__((amdgpu_waves_per_eu(3))) void wl_haar_synth(
    const uint8_t* __restrict__ src, const double* __restrict__ in64, int h, int w,
    int64_t row_stride, const double* __restrict__ stats, uint8_t* __restrict__ out_u8,
    float* __restrict__ out_f32) {
  using HS = HaarSplit<L>;
  constexpr int B = HS::B, QS = HS::QS;
  const int img = blockIdx.y;
  const int nbx = w / B, nblk = nbx * (h / B);
  const int tid = blockIdx.x * WLH_WG + threadIdx.x;
  const int blk = tid / HS::NS, sub = tid % HS::NS;
  const bool act = blk < nblk;
  const double* st = stats + (size_t)img * WL_STATS;
  const bool bad = st[WlStats::FLAG] != 0.0;
  wreal mn[3], inv[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    wreal mx;
    wl_minmax64(st, c, mn[c], mx);
    inv[c] = mx - mn[c];
  }
  auto thr = [&](int c, int l, int b) { return st[WlStats::thr(c, l, b, L)]; };
  int y0 = 0, x0 = 0;
  if (act) {
    const int by = blk / nbx, bx = blk - by * nbx;
    const int sy = sub / (B / HS::SB), sx = sub % (B / HS::SB);
    y0 = by * B + sy * HS::SB;
    x0 = bx * B + sx * HS::SB;
  }
  wreal a1[3][QS * QS], d1[3][3][QS * QS];
  if (act) haar_sub_analysis<L>(src, in64, img, h, w, row_stride, y0, x0, mn, inv, a1, d1);
  if constexpr (L >= 2) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      wreal a2 = 0, ad2 = 0, da2 = 0, dd2 = 0;
      if (act) haar2x2(a1[c][0], a1[c][1], a1[c][2], a1[c][3], a2, ad2, da2, dd2);
      if constexpr (L == 3) {  // level 3 across the block's 4 lanes, synthesised back to a2
        const int base = (threadIdx.x & 63) & ~3;
        const wreal x00 = __shfl(a2, base), x01 = __shfl(a2, base + 1);
        const wreal x10 = __shfl(a2, base + 2), x11 = __shfl(a2, base + 3);
        wreal aa, ad, da, dd;
        haar2x2(x00, x01, x10, x11, aa, ad, da, dd);
        a2 = ihaar(aa, soft(ad, thr(c, 2, 0)), soft(da, thr(c, 2, 1)), soft(dd, thr(c, 2, 2)),
                   sub >> 1, sub & 1);
      }
      const wreal AD = soft(ad2, thr(c, 1, 0)), DA = soft(da2, thr(c, 1, 1));
      const wreal DD = soft(dd2, thr(c, 1, 2));
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int s = 0; s < 2; ++s) a1[c][r * 2 + s] = ihaar(a2, AD, DA, DD, r, s);
    }
  }
  if (!act) return;
  // level 1 per 2x2 group with the pixels' own details, colour, casts.  A 4x4 sub-block's rows
  // are 12 contiguous bytes: packed and stored as three dwords per row (single-byte stores made
  // 14x the L2 write requests of the output bytes)
  const bool dw =
      QS == 2 && out_u8 && ((reinterpret_cast<uintptr_t>(out_u8) | (uintptr_t)row_stride) & 3) == 0;
  uint32_t rowp[2][3] = {{0u, 0u, 0u}, {0u, 0u, 0u}};
#pragma unroll
  for (int k = 0; k < QS * QS; ++k) {
    const int qy = k / QS, qx = k % QS;
    if (qx == 0) {
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int j = 0; j < 3; ++j) rowp[r][j] = 0u;
    }
    wreal A[3], AD[3], DA[3], DD[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      A[c] = a1[c][k];
      AD[c] = soft(d1[c][0][k], thr(c, 0, 0));
      DA[c] = soft(d1[c][1][k], thr(c, 0, 1));
      DD[c] = soft(d1[c][2][k], thr(c, 0, 2));
    }
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        // one pixel at a time (three channels live): inner denoise_wavelet clip (0.14.2), then
        // * (max - min) + min, YCbCr -> RGB, clip, cast
        wreal o[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const double vv = fmin(fmax((double)ihaar(A[c], AD[c], DA[c], DD[c], r, s), 0.0), 1.0);
          o[c] = vv * inv[c] + mn[c];
        }
        const double Y = o[0] - 16.0, Cb = o[1] - 128.0, Cr = o[2] - 128.0;
        double o3[3];
        o3[0] = dot3(Y, Cb, Cr, 0.004566210045662101, 1.1808799897950177e-09, 0.006258928969943937);
        o3[1] = dot3(Y, Cb, Cr, 0.004566210045662101, -0.0015363236860449021, -0.003188110949655707);
        o3[2] = dot3(Y, Cb, Cr, 0.004566210045662101, 0.007910716233554741, 1.1977497040511743e-08);
        const int y = y0 + 2 * qy + r, x = x0 + 2 * qx + s;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          double vv = fmin(fmax(o3[c], 0.0), 1.0);
          if (bad) vv = 0.0;
          const uint32_t u = (uint32_t)(int)(255.0 * vv);
          if (dw) {
            const int bi = (2 * qx + s) * 3 + c;
            rowp[r][bi >> 2] |= u << (8 * (bi & 3));
          } else if (out_u8) {
            out_u8[(int64_t)img * h * row_stride + (int64_t)y * row_stride + (int64_t)x * 3 + c] =
                (uint8_t)u;
          }
          if (out_f32) out_f32[(((int64_t)img * h + y) * w + x) * 3 + c] = (float)vv;
        }
      }
    if (dw && qx == QS - 1) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        uint32_t* p = reinterpret_cast<uint32_t*>(out_u8 + (int64_t)img * h * row_stride +
                                                  (int64_t)(y0 + 2 * qy + r) * row_stride +
                                                  (int64_t)x0 * 3);
#pragma unroll
        for (int j = 0; j < 3; ++j) p[j] = rowp[r][j];
      }
    }
  }
}

// sigma for the fused path.  wl_haar_analyze left one fine-bin code per finest dd (u16: 0 for an
// exact zero, else wl_fbin(|dd|) + 1).  Pass 1: histogram of the codes, block-wide selection of
// the fine bin holding the lower middle rank.  Pass 2: the positions of that bin's codes (and of
// the next nonempty bin's, where the upper middle rank may live) are compacted; the exact |dd| of
// just those positions are recomputed from the input (wl_dd1_key: the analysis' loads and op
// order), and the remaining digits are selected on them.  The fp64 band never goes through HBM.
template <bool MARK>
__device__ unsigned long long wl_dd1_key(const uint8_t* __restrict__ src,
                                         const double* __restrict__ in64, int img, int h, int w,
                                         int64_t row_stride, uint32_t pos, int W1, int c, wreal mn,
                                         wreal inv, wreal rcp) {
  const int i = (int)(pos / (uint32_t)W1), j = (int)(pos - (uint32_t)i * (uint32_t)W1);
  wreal r[2][2];
#pragma unroll
  for (int rr = 0; rr < 2; ++rr)
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      double px[3];
      load_rgb64(src, in64, img, h, w, row_stride, 2 * i + rr, 2 * j + ss, px);
      const wreal a = ycbcr_c(px, c) - mn;
      if (MARK) {  // haar_row4_c
        const wreal q0 = a * rcp;
        r[rr][ss] = __fma_rn(__fma_rn(-q0, inv, a), rcp, q0);
      } else {  // L = 1: the plain quotient
        r[rr][ss] = a / inv;
      }
    }
  wreal aa, ad, da, dd;
  haar2x2(r[0][0], r[0][1], r[1][0], r[1][1], aa, ad, da, dd);
  return absbits(dd);
}

// the same for u8 input, split into the loads (two rows of 6 bytes as 3 half-words each: row
// starts are 4-byte aligned on this path, 6 j is even) and the arithmetic, so that a thread can
// keep several positions' loads in flight
struct Dd1Raw {
  uint32_t r[2][3];
};
__device__ __forceinline__ Dd1Raw wl_dd1_load(const uint8_t* __restrict__ src, int img, int h,
                                              int64_t row_stride, uint32_t pos, int W1) {
  const int i = (int)(pos / (uint32_t)W1), j = (int)(pos - (uint32_t)i * (uint32_t)W1);
  Dd1Raw q;
#pragma unroll
  for (int rr = 0; rr < 2; ++rr) {
    const uint16_t* p = reinterpret_cast<const uint16_t*>(
        src + ((int64_t)img * h + 2 * i + rr) * row_stride + (int64_t)6 * j);
#pragma unroll
    for (int k = 0; k < 3; ++k) q.r[rr][k] = p[k];
  }
  return q;
}
template <bool MARK>
__device__ __forceinline__ unsigned long long wl_dd1_eval(const Dd1Raw& q, int c, wreal mn,
                                                          wreal inv, wreal rcp) {
  wreal r[2][2];
#pragma unroll
  for (int rr = 0; rr < 2; ++rr)
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      double px[3];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        const int b = ss * 3 + ch;
        px[ch] = (double)((q.r[rr][b >> 1] >> (8 * (b & 1))) & 0xFFu) * (1.0 / 255.0);
      }
      const wreal a = ycbcr_c(px, c) - mn;
      if (MARK) {
        const wreal q0 = a * rcp;
        r[rr][ss] = __fma_rn(__fma_rn(-q0, inv, a), rcp, q0);
      } else {
        r[rr][ss] = a / inv;
      }
    }
  wreal aa, ad, da, dd;
  haar2x2(r[0][0], r[0][1], r[1][0], r[1][1], aa, ad, da, dd);
  return absbits(dd);
}

__device__ unsigned long long wl_bior_dd1_key64(const double* __restrict__ in64, int img, int h,
                                                int w, uint32_t pos, int W1, int c, wreal mn,
                                                wreal inv) {
  const int i = (int)(pos / (uint32_t)W1), j = (int)(pos - (uint32_t)i * (uint32_t)W1);
  const int y[2] = {sym_idx(2 * i - 4, h), sym_idx(2 * i - 3, h)};
  const int x[2] = {sym_idx(2 * j - 4, w), sym_idx(2 * j - 3, w)};
  double r[2][2];
#pragma unroll
  for (int rr = 0; rr < 2; ++rr)
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      double px[3];
      load_rgb64(nullptr, in64, img, h, w, 0, y[rr], x[cc], px);
      r[rr][cc] = (ycbcr_c(px, c) - mn) / inv;  // wl_dwt_stream's norm for f64 input
    }
  return absbits(bior_dd2x2(r[0][0], r[0][1], r[1][0], r[1][1]));
}

// ---- Haar statistics for u8 input (L >= 2): integer moments instead of fp64 planes ---------------
// BayesShrink needs per (channel, level, band) the sum of squared detail coefficients, and the
// sigma median the fine-bin codes of the finest dd.  For u8 input every Haar detail is an integer
// combination of the pixels times a constant (the channel offsets and the minimum cancel in the
// +-1 combinations):
//     d(c, l) = 2^-l (w_c . D) / (255000 (max_c - min_c)),   w_c = rgb2ycbcr row c x 1000
// with D the integer RGB vector of the band's combination.  So the sums follow from exact integer
// second moments of D (six per band), summed in int32 per thread and in fp64 after that -- a
// rounding-level difference from pywt's own fp64 sums, like any other summation order -- and the
// dd codes from T = w_c . D_dd, ~25 integer / fp64 ops per pixel where wl_haar_analyze recomputes
// the normalised fp64 planes (~100).
// The codes must equal those of the reference's fp64 dd (the median recomputes exact values per
// code).  Its deviation from the exact value 0.5 T / (255000 inv) is below 1e-12 / inv (rounded
// 1/255, YCbCr dot, offset, difference and quotient, each <= 2.8e-14 absolute at magnitude <= 256,
// then the 2x2 combination), so |dd_ref - a| <= 2e-12 / inv for the fp64 approximation a, i.e.
// a relative 1.02e-6 / |T| <= 3.4e-7 for |T| >= 3.  When the mantissa bits below the code's four
// are >= 2^33 away from both ends, a is >= 2^-19 (relative) from every bin edge, so the code is
// certain.  Everything else -- T == 0 (an exact zero or a rounding residue), |T| < 3, values next
// to an edge -- is evaluated exactly (wl_dd1_key, the median's own evaluation).  Groups whose
// pixel pairs are equal RGB triples (rows or columns) have dd exactly 0 in the reference (x - x)
// and need no evaluation; the rest are queued in LDS and evaluated densely by the whole workgroup
// between iterations (heavily clipped noise makes ~6 % of the codes uncertain: evaluated inline,
// every wave would pay for them).
// Channels whose range is only rounding noise (Cb / Cr of a gray image, range ~1e-14) get sums
// that differ from the fp64 planes' (which are noise themselves); their thresholds cannot move the
// output, which is min + v * range for such a channel.
constexpr int WLS_IT = 16;  // sub-blocks per thread (int32 moments stay below 2^31: <= 1.07e9)
constexpr int WLS_XMAX = WLH_WG * 12;  // uncertain codes one iteration can queue (12 per thread)
constexpr int WLS_XCAP = 2 * WLS_XMAX;  // the queue is evaluated once more than half full
__device__ __forceinline__ void haar_int(int x00, int x01, int x10, int x11, int& aa, int& ad,
                                         int& da, int& dd) {
  const int lo0 = x00 + x10, lo1 = x01 + x11, hi0 = x00 - x10, hi1 = x01 - x11;
  aa = lo0 + lo1;
  ad = lo0 - lo1;
  da = hi0 + hi1;
  dd = hi0 - hi1;
}
__device__ __forceinline__ void mom_add(int (&m)[6], int r, int g, int b) {
  m[0] += __mul24(r, r);
  m[1] += __mul24(g, g);
  m[2] += __mul24(b, b);
  m[3] += __mul24(r, g);
  m[4] += __mul24(r, b);
  m[5] += __mul24(g, b);
}

template <int L>
__global__ __launch_bounds__(WLH_WG) void wl_haar_stats(
    const uint8_t* __restrict__ src, int h, int w, int64_t row_stride, wreal* __restrict__ ws,
    size_t img_floats, size_t dd_off, const double* __restrict__ stats, double* __restrict__ part,
    size_t part_per_img) {
  static_assert(L == 2 || L == 3, "4x4 sub-blocks per thread");
  using HS = HaarSplit<L>;
  constexpr int B = HS::B;
  const int img = blockIdx.y;
  const int nbx = w / B, nblk = nbx * (h / B);
  const double* st = stats + (size_t)img * WL_STATS;
  __shared__ double red[3 * L * 3][WLH_WG / 64];
  __shared__ uint32_t xq[WLS_XCAP];  // queued uncertain codes: position * 4 + channel
  __shared__ uint32_t xq_n;
  // levels 2..L moments in LDS, one private column per thread ([k][thread]: consecutive lanes on
  // consecutive banks, ds_add_u32 without conflicts): 36 fewer VGPRs than register accumulators,
  // which with the one-ahead prefetch brings the kernel from 2 to 3 waves per SIMD
  // (level 3: one column per 8x8 block, written by its sub-block-0 lane only)
  __shared__ int ml2[3 * 6][WLH_WG];
  __shared__ int ml3[L == 3 ? 3 * 6 : 1][WLH_WG / 4];
#pragma unroll
  for (int k = 0; k < 3 * 6; ++k) ml2[k][threadIdx.x] = 0;
  if (L == 3 && threadIdx.x < WLH_WG / 4)
#pragma unroll
    for (int k = 0; k < 3 * 6; ++k) ml3[k][threadIdx.x] = 0;
  if (threadIdx.x == 0) xq_n = 0u;
  __syncthreads();
  const size_t W1 = (size_t)(w / 2), bsz = (size_t)(h / 2) * W1;
  // per-channel scales, uniform: kept in SGPRs (min / range / reciprocal are re-read by the rare
  // exact path only) -- the moments already hold 54 VGPRs
  wreal sc[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    wreal mn, mx;
    wl_minmax64(st, c, mn, mx);
    sc[c] = uniform_f64(0.5 / (255000.0 * (mx - mn)));
  }
  int mom[3][6];  // level 1 (levels >= 2: mlds)
#pragma unroll
  for (int b = 0; b < 3; ++b)
#pragma unroll
    for (int k = 0; k < 6; ++k) mom[b][k] = 0;
  auto mom_lds = [&](int l, int b, int r, int g, int bl) {  // level l >= 1 (0-based)
    const int ld = l == 1 ? WLH_WG : WLH_WG / 4;  // row pitch of the level's array
    int* m = l == 1 ? &ml2[b * 6][threadIdx.x] : &ml3[(L == 3 ? b : 0) * 6][threadIdx.x >> 2];
    atomicAdd(m + 0 * ld, __mul24(r, r));
    atomicAdd(m + 1 * ld, __mul24(g, g));
    atomicAdd(m + 2 * ld, __mul24(bl, bl));
    atomicAdd(m + 3 * ld, __mul24(r, g));
    atomicAdd(m + 4 * ld, __mul24(r, bl));
    atomicAdd(m + 5 * ld, __mul24(g, bl));
  };
  const uint8_t* ib = src + (int64_t)img * h * row_stride;
  uint16_t* cdp0 = reinterpret_cast<uint16_t*>(ws + img * img_floats + dd_off + 3 * bsz);
  // sub-block geometry of iteration `it`; its 4 rows x 12 bytes (dword aligned: checked on the
  // host) are loaded one iteration ahead
  auto geom = [&](int it, int& sub, int& y0, int& x0) -> bool {
    const int tid = (blockIdx.x * WLS_IT + it) * WLH_WG + threadIdx.x;
    const int blk = tid / HS::NS;
    sub = tid % HS::NS;
    const int by = blk / nbx, bx = blk - by * nbx;
    y0 = by * B + (sub >> 1) * 4;
    x0 = bx * B + (sub & 1) * 4;
    return blk < nblk;  // uniform over each block's NS consecutive lanes
  };
  auto load_q = [&](int it, uint32_t (&qq)[4][3]) {
    int sub, y0, x0;
    if (!geom(it, sub, y0, x0)) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t* p = reinterpret_cast<const uint32_t*>(ib + (int64_t)(y0 + r) * row_stride +
                                                            (int64_t)x0 * 3);
#pragma unroll
      for (int k = 0; k < 3; ++k) qq[r][k] = p[k];
    }
  };
  uint32_t qn[4][3] = {};
  load_q(0, qn);
#pragma unroll 1
  for (int it = 0; it < WLS_IT; ++it) {
    int sub, y0, x0;
    const bool act = geom(it, sub, y0, x0);
    uint32_t q[4][3];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int k = 0; k < 3; ++k) q[r][k] = qn[r][k];
    if (it + 1 < WLS_IT) load_q(it + 1, qn);
    int a2[3] = {0, 0, 0};
    if (act) {
      auto px = [&](int r, int k) { return (int)((q[r][k >> 2] >> (8 * (k & 3))) & 0xFFu); };
      int a1[4][3];
#pragma unroll
      for (int gy = 0; gy < 2; ++gy)
#pragma unroll
        for (int gx = 0; gx < 2; ++gx) {
          int D[3][3];  // band (ad, da, dd) x rgb
#pragma unroll
          for (int ch = 0; ch < 3; ++ch)
            haar_int(px(2 * gy, 6 * gx + ch), px(2 * gy, 6 * gx + 3 + ch),
                     px(2 * gy + 1, 6 * gx + ch), px(2 * gy + 1, 6 * gx + 3 + ch),
                     a1[gy * 2 + gx][ch], D[0][ch], D[1][ch], D[2][ch]);
#pragma unroll
          for (int b = 0; b < 3; ++b) mom_add(mom[b], D[b][0], D[b][1], D[b][2]);
          const size_t cpos = (size_t)(y0 / 2 + gy) * W1 + (size_t)(x0 / 2 + gx);
          uint32_t code[3], unsure = 0u;
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const int T = __mul24(ycc_w(c, 0), D[2][0]) + __mul24(ycc_w(c, 1), D[2][1]) +
                          __mul24(ycc_w(c, 2), D[2][2]);
            const uint32_t aT = (uint32_t)(T < 0 ? -T : T);
            const uint32_t hi = (uint32_t)__double2hiint((double)aT * sc[c]);
            code[c] = (uint32_t)min(max((int)(hi >> 16) - (1023 - 61) * 16, 0), WL_FBINS - 1) + 1u;
            if (!(aT >= 3u && (hi & 0xFFFFu) - 2u <= 0xFFFBu)) unsure |= 1u << c;
          }
          if (unsure) {
            // equal RGB triples along rows or columns: the reference's dd is x - x = 0 exactly
            auto trip = [&](int r, int k) { return px(r, k) | (px(r, k + 1) << 8) | (px(r, k + 2) << 16); };
            const int t00 = trip(2 * gy, 6 * gx), t01 = trip(2 * gy, 6 * gx + 3);
            const int t10 = trip(2 * gy + 1, 6 * gx), t11 = trip(2 * gy + 1, 6 * gx + 3);
            if ((t00 == t01 && t10 == t11) || (t00 == t10 && t01 == t11)) {
#pragma unroll
              for (int c = 0; c < 3; ++c)
                if ((unsure >> c) & 1u) code[c] = 0u;
              unsure = 0u;
            }
          }
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            if ((unsure >> c) & 1u)  // queued: evaluated exactly below (at most 12 per thread)
              xq[atomicAdd(&xq_n, 1u)] = (uint32_t)cpos * 4u + (uint32_t)c;
            else
              cdp0[(size_t)c * 4 * bsz * (sizeof(wreal) / sizeof(uint16_t)) + cpos] = (uint16_t)code[c];
          }
        }
      int D2[3][3];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch)
        haar_int(a1[0][ch], a1[1][ch], a1[2][ch], a1[3][ch], a2[ch], D2[0][ch], D2[1][ch],
                 D2[2][ch]);
#pragma unroll
      for (int b = 0; b < 3; ++b) mom_lds(1, b, D2[b][0], D2[b][1], D2[b][2]);
    }
    if constexpr (L == 3) {  // level 3 across the block's 4 lanes (all lanes take part)
      const int base = (threadIdx.x & 63) & ~3;
      int D3[3][3];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        int aa;
        haar_int(__shfl(a2[ch], base), __shfl(a2[ch], base + 1), __shfl(a2[ch], base + 2),
                 __shfl(a2[ch], base + 3), aa, D3[0][ch], D3[1][ch], D3[2][ch]);
      }
      if (act && sub == 0)
#pragma unroll
        for (int b = 0; b < 3; ++b) mom_lds(2, b, D3[b][0], D3[b][1], D3[b][2]);
    }
    // the queued uncertain codes, densely over the workgroup, once the queue could overflow in
    // the next iteration (and after the last one)
    __syncthreads();
    const uint32_t nq = xq_n;  // workgroup-uniform
    if (nq > (uint32_t)(WLS_XCAP - WLS_XMAX) || (it == WLS_IT - 1 && nq)) {
      for (uint32_t i = threadIdx.x; i < nq; i += WLH_WG) {
        const uint32_t e = xq[i], pos = e >> 2;
        const int c = (int)(e & 3u);
        wreal mnc, mxc;
        wl_minmax64(st, c, mnc, mxc);
        const wreal invc = mxc - mnc;
        const unsigned long long key = wl_dd1_key<true>(src, nullptr, img, h, w, row_stride, pos,
                                                        (int)W1, c, mnc, invc, 1.0 / invc);
        cdp0[(size_t)c * 4 * bsz * (sizeof(wreal) / sizeof(uint16_t)) + pos] =
            (uint16_t)(key ? (uint32_t)wl_fbin(key) + 1u : 0u);
      }
      __syncthreads();
      if (threadIdx.x == 0) xq_n = 0u;
      __syncthreads();
    }
  }
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const double w0 = ycc_w(c, 0), w1 = ycc_w(c, 1), w2 = ycc_w(c, 2);
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const double s = ldexp(sc[c], -l);  // 2^-(l+1) / (255000 inv)
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        int m[6];
#pragma unroll
        for (int k = 0; k < 6; ++k)
          m[k] = l == 0 ? mom[b][k]
                 : l == 1 ? ml2[b * 6 + k][threadIdx.x]
                          : ((threadIdx.x & 3) == 0 ? ml3[(L == 3 ? b : 0) * 6 + k][threadIdx.x >> 2] : 0);
        double v = w0 * w0 * (double)m[0] + w1 * w1 * (double)m[1] + w2 * w2 * (double)m[2] +
                   2.0 * (w0 * w1 * (double)m[3] + w0 * w2 * (double)m[4] + w1 * w2 * (double)m[5]);
        v *= s * s;
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((threadIdx.x & 63) == 0) red[(c * L + l) * 3 + b][wave] = v;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < 3 * L * 3) {
    const int k = threadIdx.x, b = k % 3, l = (k / 3) % L, c = k / (3 * L);
    double t = red[k][0];
#pragma unroll
    for (int wv = 1; wv < WLH_WG / 64; ++wv) t += red[k][wv];
    part[img * part_per_img + (size_t)(c * 3 + b) * (part_per_img / 9) + (size_t)l * gridDim.x +
         blockIdx.x] = t;
  }
}

// ---- Haar synthesis for u8 input (L >= 2) from the integer combinations -------------------------
// The same algebra as wl_haar_stats: with s1 = 0.5 / (255000 inv) and k = 2 (off - min) / inv,
//     level-l detail  d_l = 2^-(l-1) s1 (w_c . D_l),     level-L approximation
//     a_L = 2^-(L-1) s1 (w_c . S_L) + 2^(L-1) k          (S_L: the integer RGB sum of the block)
// so no normalised plane is evaluated: per coefficient three 24-bit integer multiply-adds, one
// conversion and one multiply.  pywt's idwt2 of one 2x2 group is 0.5 (A +- AD +- DA +- DD) in
// its four outputs; the 0.5 is folded into the coefficients and the soft thresholds (a power of
// two commutes with soft()) and the four outputs come from a butterfly: 8 adds per group and
// channel where ihaar takes 4 multiplies + 4 adds per output.  De-normalisation, YCbCr -> RGB and
// the x255 cast fold into three fma chains per pixel.  Every coefficient agrees with the fp64
// planes' to a few ulps (the error analysis of wl_haar_stats), so outputs agree to ~1e-15 and
// the U8 cast can differ only where 255 x sits on an integer (the documented tolerance).
__device__ __forceinline__ double tdot_sum(int c, const int (&v)[3]) {
  // w_c . S for the non-negative block sums: Y's weights are all positive and its dot reaches
  // 3.6e9 at level 3, past int32: two exact signed parts (<= 2.1e9 each) added in fp64 (an
  // unsigned sum was converted as signed by the compiler).  Cb / Cr stay within +-1.9e9
  if (c == 0)
    return (double)(__mul24(65481, v[0]) + __mul24(24966, v[2])) + (double)__mul24(128553, v[1]);
  return (double)(__mul24(ycc_w(c, 0), v[0]) + __mul24(ycc_w(c, 1), v[1]) +
                  __mul24(ycc_w(c, 2), v[2]));
}
__device__ __forceinline__ double tdot(int c, int d0, int d1, int d2) {  // details: |T| <= 1.83e9
  return (double)(__mul24(ycc_w(c, 0), d0) + __mul24(ycc_w(c, 1), d1) + __mul24(ycc_w(c, 2), d2));
}
// soft(x, t) as x - clamp(x, -t, t): the same value as soft() (x -+ t rounds alike; 0 inside),
// three fp64 ops instead of a compare and two selects
__device__ __forceinline__ double soft_c(double x, double t) { return x - fmin(fmax(x, -t), t); }
// outputs (r, s) = (0,0), (0,1), (1,0), (1,1) of A + g_s AD + f_r DA + f_r g_s DD
__device__ __forceinline__ void haar_bfly(double A, double AD, double DA, double DD, double (&x)[4]) {
  const double p = A + AD, m = A - AD, q0 = DA + DD, q1 = DA - DD;
  x[0] = p + q0;
  x[1] = m + q1;
  x[2] = p - q0;
  x[3] = m - q1;
}

// S32: the level-1 stage (details, soft thresholds, butterflies, clip, de-normalisation,
// YCbCr -> RGB) in fp32 with v_med3 clamps, as bior1.5's synthesis: it is continuous in its
// inputs and no exact zero depends on it (the levels above stay fp64; ~1e-7 on the [0, 1]
// output against the 1e-5 tolerance).  false: all fp64 (A/B: IDN_WAVELET_HS32=0)
template <int L, bool S32 = true>
__global__ __launch_bounds__(WLH_WG) void wl_haar_synth_int(const uint8_t* __restrict__ src, int h,
                                                            int w, int64_t row_stride,
                                                            const double* __restrict__ stats,
                                                            uint8_t* __restrict__ out_u8,
                                                            float* __restrict__ out_f32) {
  static_assert(L == 2 || L == 3, "4x4 sub-blocks per thread");
  using HS = HaarSplit<L>;
  constexpr int B = HS::B;
  const int img = blockIdx.y;
  const int nbx = w / B, nblk = nbx * (h / B);
  const int tid = blockIdx.x * WLH_WG + threadIdx.x;
  const int blk = tid / HS::NS, sub = tid % HS::NS;
  const bool act = blk < nblk;
  const double* st = stats + (size_t)img * WL_STATS;
  const bool bad = st[WlStats::FLAG] != 0.0;  // image-uniform: zeros (0.14.2's NaN -> U8 0)
  int y0 = 0, x0 = 0;
  uint32_t q[4][3] = {};
  if (act) {
    const int by = blk / nbx, bx = blk - by * nbx;
    y0 = by * B + (sub >> 1) * 4;
    x0 = bx * B + (sub & 1) * 4;
    const uint8_t* ib = src + (int64_t)img * h * row_stride;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t* p = reinterpret_cast<const uint32_t*>(ib + (int64_t)(y0 + r) * row_stride +
                                                            (int64_t)x0 * 3);
#pragma unroll
      for (int k = 0; k < 3; ++k) q[r][k] = p[k];
    }
  }
  auto px = [&](int r, int k) { return (int)((q[r][k >> 2] >> (8 * (k & 3))) & 0xFFu); };
  // integer sums of the four level-1 groups and the level-2 combinations
  int S4[4][3];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const int gy = g >> 1, gx = g & 1;
      S4[g][ch] = px(2 * gy, 6 * gx + ch) + px(2 * gy, 6 * gx + 3 + ch) +
                  px(2 * gy + 1, 6 * gx + ch) + px(2 * gy + 1, 6 * gx + 3 + ch);
    }
  int S16[3], D2[3][3];
#pragma unroll
  for (int ch = 0; ch < 3; ++ch)
    haar_int(S4[0][ch], S4[1][ch], S4[2][ch], S4[3][ch], S16[ch], D2[0][ch], D2[1][ch], D2[2][ch]);
  int S64[3] = {0, 0, 0}, D3[3][3] = {};
  if constexpr (L == 3) {  // level 3 across the block's 4 lanes
    const int base = (threadIdx.x & 63) & ~3;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch)
      haar_int(__shfl(S16[ch], base), __shfl(S16[ch], base + 1), __shfl(S16[ch], base + 2),
               __shfl(S16[ch], base + 3), S64[ch], D3[0][ch], D3[1][ch], D3[2][ch]);
  }
  if (!act) return;
  if (bad) {
#pragma unroll 1
    for (int r = 0; r < 4; ++r)
#pragma unroll 1
      for (int k = 0; k < 12; ++k) {
        const int y = y0 + r, xx = x0 + k / 3, c = k % 3;
        if (out_u8) out_u8[(int64_t)img * h * row_stride + (int64_t)y * row_stride + (int64_t)xx * 3 + c] = 0;
        if (out_f32) out_f32[(((int64_t)img * h + y) * w + xx) * 3 + c] = 0.0f;
      }
    return;
  }
  // per-channel constants (uniform: SGPRs)
  double mnc[3], invc[3], s1c[3], kc[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double mn, mx;
    wl_minmax64(st, c, mn, mx);
    mnc[c] = mn;
    invc[c] = mx - mn;
    s1c[c] = uniform_f64(0.5 / (255000.0 * invc[c]));
    kc[c] = uniform_f64(2.0 * ((c == 0 ? 16.0 : 128.0) - mn) / invc[c]);
  }
  // level L .. 2 per channel -> half the level-1 approximations of the four groups
  double Ah1[4][3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const double s1 = s1c[c], k = kc[c];
    auto th = [&](int l, int b) { return st[WlStats::thrh(c, l, b)]; };
    double a2;  // level-2 approximation at this sub-block (after level-3 synthesis)
    if constexpr (L == 3) {
      const double Ah = tdot_sum(c, S64) * ldexp(s1, -3) + 2.0 * k;
      const double x3 = ldexp(s1, -3);
      double x[4];
      haar_bfly(Ah, soft_c(tdot(c, D3[0][0], D3[0][1], D3[0][2]) * x3, th(2, 0)),
                soft_c(tdot(c, D3[1][0], D3[1][1], D3[1][2]) * x3, th(2, 1)),
                soft_c(tdot(c, D3[2][0], D3[2][1], D3[2][2]) * x3, th(2, 2)), x);
      a2 = sub == 0 ? x[0] : sub == 1 ? x[1] : sub == 2 ? x[2] : x[3];
    } else {
      a2 = tdot_sum(c, S16) * ldexp(s1, -1) + 2.0 * k;
    }
    const double x2 = ldexp(s1, -2);
    double x[4];
    haar_bfly(0.5 * a2, soft_c(tdot(c, D2[0][0], D2[0][1], D2[0][2]) * x2, th(1, 0)),
              soft_c(tdot(c, D2[1][0], D2[1][1], D2[1][2]) * x2, th(1, 1)),
              soft_c(tdot(c, D2[2][0], D2[2][1], D2[2][2]) * x2, th(1, 2)), x);
#pragma unroll
    for (int g = 0; g < 4; ++g) Ah1[g][c] = 0.5 * x[g];
  }
  // YCbCr -> RGB x 255 (skimage's ycbcr2rgb rows) on (v' * inv + min - off)
  constexpr double R[3][3] = {{0.004566210045662101 * 255, 1.1808799897950177e-09 * 255, 0.006258928969943937 * 255},
                              {0.004566210045662101 * 255, -0.0015363236860449021 * 255, -0.003188110949655707 * 255},
                              {0.004566210045662101 * 255, 0.007910716233554741 * 255, 1.1977497040511743e-08 * 255}};
  const bool dw = out_u8 && ((reinterpret_cast<uintptr_t>(out_u8) | (uintptr_t)row_stride) & 3) == 0;
  uint32_t rowp[2][3];
  float x1f[3], thf[3][3], invf[3], mof[3];  // S32: the level-1 constants in fp32
  if constexpr (S32) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      x1f[c] = (float)(0.5 * s1c[c]);
#pragma unroll
      for (int b = 0; b < 3; ++b) thf[c][b] = (float)st[WlStats::thrh(c, 0, b)];
      invf[c] = (float)invc[c];
      mof[c] = (float)(mnc[c] - (c == 0 ? 16.0 : 128.0));
    }
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int gy = g >> 1, gx = g & 1;
    if (gx == 0) {
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int j = 0; j < 3; ++j) rowp[r][j] = 0u;
    }
    double v[4][3];  // the group's four pixels, three channels: v' (normalised)
    int D[3][3];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      int aa;
      haar_int(px(2 * gy, 6 * gx + ch), px(2 * gy, 6 * gx + 3 + ch), px(2 * gy + 1, 6 * gx + ch),
               px(2 * gy + 1, 6 * gx + 3 + ch), aa, D[0][ch], D[1][ch], D[2][ch]);
    }
    if constexpr (S32) {
      constexpr float Rf[3][3] = {
          {(float)(0.004566210045662101 * 255), (float)(1.1808799897950177e-09 * 255), (float)(0.006258928969943937 * 255)},
          {(float)(0.004566210045662101 * 255), (float)(-0.0015363236860449021 * 255), (float)(-0.003188110949655707 * 255)},
          {(float)(0.004566210045662101 * 255), (float)(0.007910716233554741 * 255), (float)(1.1977497040511743e-08 * 255)}};
      float vf[4][3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float d[3];
#pragma unroll
        for (int b = 0; b < 3; ++b) {  // soft(x, t) = x - clamp(x, -t, t), one v_med3
          const float xb = (float)(__mul24(ycc_w(c, 0), D[b][0]) + __mul24(ycc_w(c, 1), D[b][1]) +
                                   __mul24(ycc_w(c, 2), D[b][2])) * x1f[c];
          d[b] = xb - __builtin_amdgcn_fmed3f(xb, -thf[c][b], thf[c][b]);
        }
        const float A = (float)Ah1[g][c];
        const float p = A + d[0], m = A - d[0], q0 = d[1] + d[2], q1 = d[1] - d[2];
        vf[0][c] = p + q0;
        vf[1][c] = m + q1;
        vf[2][c] = p - q0;
        vf[3][c] = m - q1;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = i >> 1, s = i & 1;
        float e[3];
#pragma unroll
        for (int c = 0; c < 3; ++c)
          e[c] = __fmaf_rn(__builtin_amdgcn_fmed3f(vf[i][c], 0.f, 1.f), invf[c], mof[c]);
        const int y = y0 + 2 * gy + r, xx = x0 + 2 * gx + s;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float o = __fmaf_rn(e[2], Rf[c][2], __fmaf_rn(e[1], Rf[c][1], e[0] * Rf[c][0]));
          const uint32_t u = (uint32_t)min(max((int)o, 0), 255);  // as the fp64 form
          if (dw) {
            const int bi = (2 * gx + s) * 3 + c;
            rowp[r][bi >> 2] |= u << (8 * (bi & 3));
          } else if (out_u8) {
            out_u8[(int64_t)img * h * row_stride + (int64_t)y * row_stride + (int64_t)xx * 3 + c] =
                (uint8_t)u;
          }
          if (out_f32)
            out_f32[(((int64_t)img * h + y) * w + xx) * 3 + c] =
                __builtin_amdgcn_fmed3f(o, 0.f, 255.f) * (1.f / 255.f);
        }
      }
    } else {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double x1 = 0.5 * s1c[c];
      auto th = [&](int b) { return st[WlStats::thrh(c, 0, b)]; };
      double x[4];
      haar_bfly(Ah1[g][c], soft_c(tdot(c, D[0][0], D[0][1], D[0][2]) * x1, th(0)),
                soft_c(tdot(c, D[1][0], D[1][1], D[1][2]) * x1, th(1)),
                soft_c(tdot(c, D[2][0], D[2][1], D[2][2]) * x1, th(2)), x);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i][c] = x[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = i >> 1, s = i & 1;
      double e[3];  // clip [0, 1] (0.14.2), de-normalise, minus the YCbCr offset
#pragma unroll
      for (int c = 0; c < 3; ++c)
        e[c] = __fma_rn(fmin(fmax(v[i][c], 0.0), 1.0), invc[c], mnc[c] - (c == 0 ? 16.0 : 128.0));
      const int y = y0 + 2 * gy + r, xx = x0 + 2 * gx + s;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const double o = __fma_rn(e[2], R[c][2], __fma_rn(e[1], R[c][1], e[0] * R[c][0]));
        // clip [0, 255] after the truncation (v_med3): the same byte for every o
        const uint32_t u = (uint32_t)min(max((int)o, 0), 255);
        if (dw) {
          const int bi = (2 * gx + s) * 3 + c;
          rowp[r][bi >> 2] |= u << (8 * (bi & 3));
        } else if (out_u8) {
          out_u8[(int64_t)img * h * row_stride + (int64_t)y * row_stride + (int64_t)xx * 3 + c] =
              (uint8_t)u;
        }
        if (out_f32)
          out_f32[(((int64_t)img * h + y) * w + xx) * 3 + c] = (float)(fmin(fmax(o, 0.0), 255.0) * (1.0 / 255.0));
      }
    }
    }  // S32
    if (dw && gx == 1) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        uint32_t* p = reinterpret_cast<uint32_t*>(out_u8 + (int64_t)img * h * row_stride +
                                                  (int64_t)(y0 + 2 * gy + r) * row_stride +
                                                  (int64_t)x0 * 3);
#pragma unroll
        for (int j = 0; j < 3; ++j) p[j] = rowp[r][j];
      }
    }
  }
}

// threads per (image, channel): several workgroups per CU overlap phases (512 measured 0.7 %
// faster on the whole bior1.5 op than 256 and 1024)
constexpr int WLM_WG = 512;
#ifndef IDN_WLM_IT  // A/B builds set it
#define IDN_WLM_IT 8
#endif
constexpr int WLM_IT = IDN_WLM_IT;
#ifndef IDN_WLM_HQ  // A/B builds set it
#define IDN_WLM_HQ 6
#endif
constexpr int HQ = IDN_WLM_HQ;  // Haar median: candidate positions per thread and round  // code groups (4 codes, 8 bytes) in flight per lane, passes 1-2
constexpr int WLM_NH = 8;    // histogram copies (32 KB of LDS; 16 measured slower: fewer workgroups per CU)
// BAND: the general path (any wavelet; level-1 dd stored in fp64 by wl_dwt_rb, which also left
// the codes at the start of the channel's input-plane slot): the exact keys of a position are
// read from the band instead of recomputed from the pixels.  L is unused then.  BIOR (with BAND):
// the codes as BAND, the keys recomputed from the input (bior_dd2x2; the band is fp32).
// The channel's sums of squares of every detail band over the analysis' per-tile partials (one
// wave per band, lanes over the tiles in a fixed order: deterministic, and exact for bior1.5 whose
// partials sit on a power-of-two grid) and its BayesShrink thresholds -- wl_sumsq's and
// wl_thresh's work for one channel, at the end of its median workgroup.  The degenerate-image
// flag is only ever raised here (wl_init_stats cleared it), so the three channels' workgroups
// cannot undo one another.
__device__ void wl_sums_thresh(double* __restrict__ st, const double* __restrict__ part_img, int c,
                               const WlLayout& Ls, const WlLayout& Lt, double med, wreal mn,
                               wreal mx) {
  __shared__ double sums[3 * WL_MAXL];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int k = wave; k < 3 * Lt.L; k += WLM_WG / 64) {
    const int l = k / 3, b = k - 3 * l, lev = l + 1;
    const double* p = part_img + (size_t)(c * 3 + b) * (Ls.part_per_img / 9) + Ls.part_tile0[lev];
    double s = 0.0;
    for (int t = lane; t < Ls.tiles[lev]; t += 64) s += p[t];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) sums[k] = s;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const double sigma = med / 0.6744897501960817;
  const bool bad = !(mx > mn) || !(sigma == sigma);  // 0.14.2: NaN everywhere -> U8 0
  const double var = sigma * sigma;
  for (int l = 0; l < Lt.L; ++l)
    for (int b = 0; b < 3; ++b) {
      const double sq = sums[3 * l + b];
      st[WlStats::sumsq(c, l, b, Lt.L)] = sq;
      const double cnt = (double)Lt.H[l + 1] * Lt.W[l + 1];
      const double t = var / sqrt(fmax(sq / cnt - var, 2.220446049250313e-16));
      st[WlStats::thr(c, l, b, Lt.L)] = t;
      if (Lt.L <= 3) st[WlStats::thrh(c, l, b)] = 0.5 * t;
    }
  if (bad) st[WlStats::FLAG] = 1.0;
}

// part (non-null): the channel's sums of squares over the analysis partials (wl_sumsq's work, in
// the partials layout Ls) and its BayesShrink thresholds (wl_thresh's) follow the median in the
// same workgroup -- two launches less per op
template <int L, bool BAND = false, bool BIOR = false>
__global__ __launch_bounds__(WLM_WG) void wl_haar_median(const uint8_t* __restrict__ src,
                                                       const double* __restrict__ in64,
                                                       int64_t row_stride,
                                                       wreal* __restrict__ ws, size_t img_floats,
                                                       double* __restrict__ stats, WlLayout Lt,
                                                       const double* __restrict__ part = nullptr,
                                                       WlLayout Ls = WlLayout{}) {
  constexpr bool MARK = L >= 2;
  const int img = blockIdx.x / 3, c = blockIdx.x % 3;
  const int W1 = Lt.W[1];
  const uint32_t bsz = (uint32_t)Lt.H[1] * (uint32_t)W1;
  const wreal* band_dd = ws + img * img_floats + Lt.off_band[1] + (size_t)c * 4 * bsz + 3 * bsz;
  double* slot = ws + img * img_floats + (size_t)c * Lt.h * Lt.w;
  const uint16_t* codes = BAND ? reinterpret_cast<const uint16_t*>(slot)
                               : reinterpret_cast<const uint16_t*>(band_dd);
  // scratch (the unused input-plane slot of this channel, h*w doubles; after the codes in BAND
  // mode): [0, bsz) keys of the selected bin, then positions of the selected bin and of the next
  double* keys = slot + (BAND ? (bsz + 3) / 4 : 0);
  uint32_t* pos_sel = reinterpret_cast<uint32_t*>(keys + bsz);
  uint32_t* pos_next = pos_sel + bsz;
  double* st = stats + (size_t)img * WL_STATS;
  wreal mn, mx;
  wl_minmax64(st, c, mn, mx);
  const wreal inv = mx - mn, rcp = 1.0 / inv;
  // WLM_NH copies of the histogram (by lane: the codes crowd into few bins, one copy would
  // serialise the LDS atomics); copy k lives at hist[k * WL_FBINS ..]
  __shared__ uint32_t hist[WLM_NH * WL_FBINS];
  __shared__ uint32_t m_s, mn_s, le_s, next_s;
  __shared__ unsigned long long nmin_s, gt_s;
  if (BAND && BIOR && !in64) {
    // the codes the N32 analysis could not certify (wl_dwt_stream): the exact fp64 key's code
    const uint32_t nu = *reinterpret_cast<const uint32_t*>(stats + (size_t)img * WL_STATS + WL_N32U + c);
    if (nu) {
      const uint32_t* lst = reinterpret_cast<const uint32_t*>(slot + (bsz + 3) / 4);
      uint16_t* cw = reinterpret_cast<uint16_t*>(slot);
      const rsrc_t rs = make_rsrc(src + (int64_t)img * Lt.h * row_stride, (uint32_t)((int64_t)Lt.h * row_stride));
      for (uint32_t t = threadIdx.x; t < nu; t += WLM_WG) {
        const uint32_t pos = lst[t];
        const unsigned long long key =
            wl_bior_dd1_eval(wl_bior_dd1_load(rs, Lt.h, Lt.w, row_stride, pos, W1), c, mn, inv, rcp);
        cw[pos] = (uint16_t)(key ? (uint32_t)wl_fbin(key) + 1u : 0u);
      }
      __syncthreads();
    }
  }
  for (int k = threadIdx.x; k < WLM_NH * WL_FBINS; k += WLM_WG) hist[k] = 0u;
  if (threadIdx.x == 0) {
    m_s = 0;
    mn_s = 0;
    le_s = 0;
    next_s = WL_FBINS;
    nmin_s = ~0ull;
    gt_s = ~0ull;
  }
  __syncthreads();
  // codes in 8-byte groups of 4 (the code array is 8-byte aligned), 8 groups in flight per lane:
  // every workgroup of the grid is resident at once, so each phase costs its latency chain
  const uint32_t ngrp = bsz / 4;
  const uint2* cg = reinterpret_cast<const uint2*>(codes);
  auto code_at = [](const uint2& g, int q) -> uint32_t {
    return ((q < 2 ? g.x : g.y) >> (16 * (q & 1))) & 0xFFFFu;
  };
  for (uint32_t g0 = threadIdx.x; g0 < ngrp; g0 += WLM_IT * WLM_WG) {
    uint2 gv[WLM_IT];
#pragma unroll
    for (int u = 0; u < WLM_IT; ++u) {
      const uint32_t g = g0 + (uint32_t)u * WLM_WG;
      gv[u] = g < ngrp ? cg[g] : uint2{0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < WLM_IT; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t cd = code_at(gv[u], q);
        if (cd) atomicAdd(&hist[(threadIdx.x & (WLM_NH - 1)) * WL_FBINS + cd - 1], 1u);
      }
  }
  for (uint32_t k = ngrp * 4 + threadIdx.x; k < bsz; k += WLM_WG) {  // tail codes
    const uint32_t cd = codes[k];
    if (cd) atomicAdd(&hist[(threadIdx.x & (WLM_NH - 1)) * WL_FBINS + cd - 1], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < WL_FBINS; b += WLM_WG) {  // fold the copies into copy 0
    uint32_t v = 0;
#pragma unroll
    for (int cp = 0; cp < WLM_NH; ++cp) v += hist[cp * WL_FBINS + b];
    hist[b] = v;
  }
  __syncthreads();
  uint32_t total = 0;
  const BinSel bs = select_bin(hist, WL_FBINS, 0u, &total, true);
  const int bsel = (int)bs.bin;
  for (int b = threadIdx.x; b < WL_FBINS; b += WLM_WG)
    if (b > bsel && hist[b]) atomicMin(&next_s, (uint32_t)b);
  __syncthreads();
  double med;
  if (total == 0) {
    med = NAN;  // np.median of an empty selection
  } else {
    const uint32_t klo = (total - 1) / 2, khi = total / 2;
    const uint32_t csel = (uint32_t)bsel + 1, cnext = next_s + 1;
    const int lane = threadIdx.x & 63;
    // pass 2: positions of the selected and the next bin.  Each lane counts its hits (selected
    // bin in the low half-word, next bin in the high one), one wave scan places them and one
    // LDS atomic per wave and iteration allocates the slots (per-hit ballots with an atomic each
    // serialise: a 3 % bin hits nearly every wave-wide ballot).
    auto place = [&](uint32_t cnt2, uint32_t& off_sel, uint32_t& off_next) {
      uint32_t inc = cnt2;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)inc, o);
        if (lane >= o) inc += t;
      }
      const uint32_t tot = (uint32_t)__shfl((int)inc, 63);
      uint32_t base_sel = 0, base_next = 0;
      if (lane == 63) {
        if (tot & 0xFFFFu) base_sel = atomicAdd(&m_s, tot & 0xFFFFu);
        if (tot >> 16) base_next = atomicAdd(&mn_s, tot >> 16);
      }
      base_sel = (uint32_t)__shfl((int)base_sel, 63);
      base_next = (uint32_t)__shfl((int)base_next, 63);
      const uint32_t excl = inc - cnt2;
      off_sel = base_sel + (excl & 0xFFFFu);
      off_next = base_next + (excl >> 16);
    };
    for (uint32_t gb = 0; gb < ngrp; gb += WLM_IT * WLM_WG) {  // uniform trip count: the scan needs
      const uint32_t g0 = gb + threadIdx.x;                // every lane of the wave
      uint2 gv[WLM_IT];
#pragma unroll
      for (int u = 0; u < WLM_IT; ++u) {
        const uint32_t g = g0 + (uint32_t)u * WLM_WG;
        gv[u] = g < ngrp ? cg[g] : uint2{0u, 0u};
      }
      uint32_t cnt2 = 0;
#pragma unroll
      for (int u = 0; u < WLM_IT; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t cd = code_at(gv[u], q);
          cnt2 += (cd == csel ? 1u : 0u) + (cd == cnext ? 0x10000u : 0u);
        }
      if (__ballot(cnt2 != 0) == 0) continue;  // wave-uniform
      uint32_t os, on;
      place(cnt2, os, on);
      if (cnt2) {
#pragma unroll
        for (int u = 0; u < WLM_IT; ++u)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t cd = code_at(gv[u], q);
            const uint32_t p = 4 * (g0 + (uint32_t)u * WLM_WG) + (uint32_t)q;
            if (cd == csel) pos_sel[os++] = p;
            if (cd == cnext) pos_next[on++] = p;
          }
      }
    }
    for (uint32_t k0 = ngrp * 4; k0 < bsz; k0 += WLM_WG) {  // tail codes (every lane takes part)
      const uint32_t k = k0 + threadIdx.x;
      const uint32_t cd = k < bsz ? codes[k] : 0u;
      const uint32_t cnt2 = (cd == csel ? 1u : 0u) + (cd == cnext ? 0x10000u : 0u);
      uint32_t os, on;
      place(cnt2, os, on);
      if (cd == csel) pos_sel[os] = k;
      if (cd == cnext) pos_next[on] = k;
    }
    __syncthreads();
    const uint32_t mcnt = m_s, ncnt = mn_s;
    // the selected bin's keys live in LDS when they fit: the level-1 histogram is dead now and
    // the radix passes use only its first 2048 words
    constexpr uint32_t LDS_KEYS = (WLM_NH * WL_FBINS - 2048) / 2;
    double* kb = mcnt <= LDS_KEYS ? reinterpret_cast<double*>(hist + 2048) : keys;
    // the exact keys of the selected bin, recomputed from the input (u8: 8 positions' loads in
    // flight per thread; the recompute is latency-bound otherwise)
    if (BAND && BIOR) {
      if (in64) {
        for (uint32_t t = threadIdx.x; t < mcnt; t += WLM_WG)
          kb[t] = __longlong_as_double((long long)wl_bior_dd1_key64(in64, img, Lt.h, Lt.w,
                                                                     pos_sel[t], W1, c, mn, inv));
      } else {
        const rsrc_t rs = make_rsrc(src + (int64_t)img * Lt.h * row_stride,
                                    (uint32_t)((int64_t)Lt.h * row_stride));
        // BQ positions per thread and round: all positions first (clamped, unconditional: a load
        // under a branch is waited for at once), then all their pixels.  BQ = 6 keeps the kernel
        // at <= 80 VGPRs: three 512-thread workgroups per CU, the whole grid resident at once
        constexpr int BQ = 6;
        for (uint32_t t0 = threadIdx.x; t0 < mcnt; t0 += BQ * WLM_WG) {
          uint32_t pp[BQ];
#pragma unroll
          for (int u = 0; u < BQ; ++u) pp[u] = pos_sel[min(t0 + (uint32_t)u * WLM_WG, mcnt - 1)];
          BiorDdRaw q[BQ];
#pragma unroll
          for (int u = 0; u < BQ; ++u) q[u] = wl_bior_dd1_load(rs, Lt.h, Lt.w, row_stride, pp[u], W1);
#pragma unroll
          for (int u = 0; u < BQ; ++u) {
            const uint32_t t = t0 + (uint32_t)u * WLM_WG;
            if (t < mcnt)
              kb[t] = __longlong_as_double((long long)wl_bior_dd1_eval(q[u], c, mn, inv, rcp));
          }
        }
      }
    } else if (BAND) {
      for (uint32_t t = threadIdx.x; t < mcnt; t += WLM_WG)
        kb[t] = __longlong_as_double((long long)absbits(band_dd[pos_sel[t]]));
    } else if (in64) {
      for (uint32_t t = threadIdx.x; t < mcnt; t += WLM_WG)
        kb[t] = __longlong_as_double((long long)wl_dd1_key<MARK>(
            src, in64, img, Lt.h, Lt.w, row_stride, pos_sel[t], W1, c, mn, inv, rcp));
    } else {
      for (uint32_t t0 = threadIdx.x; t0 < mcnt; t0 += HQ * WLM_WG) {
        // as the bior form: all positions first (clamped, unconditional), then their pixels
        uint32_t pp[HQ];
#pragma unroll
        for (int u = 0; u < HQ; ++u) pp[u] = pos_sel[min(t0 + (uint32_t)u * WLM_WG, mcnt - 1)];
        Dd1Raw q[HQ];
#pragma unroll
        for (int u = 0; u < HQ; ++u) q[u] = wl_dd1_load(src, img, Lt.h, row_stride, pp[u], W1);
#pragma unroll
        for (int u = 0; u < HQ; ++u) {
          const uint32_t t = t0 + (uint32_t)u * WLM_WG;
          if (t < mcnt)
            kb[t] = __longlong_as_double((long long)wl_dd1_eval<MARK>(q[u], c, mn, inv, rcp));
        }
      }
    }
    __syncthreads();
    const uint32_t rank_in = bs.rank;
    RadixState rsx{0ull, 0ull, rank_in};
    if (bsel > 0 && bsel < WL_FBINS - 1) {  // an unclamped bin: exponent and 4 mantissa bits known
      rsx.prefix = ((unsigned long long)(bsel / 16 + (1023 - 61)) << 52) |
                   ((unsigned long long)(bsel % 16) << 48);
      rsx.pmask = 0x7FFFull << 48;
      radix_pass(kb, mcnt, 37, 11, rsx, hist, nullptr);
      radix_pass(kb, mcnt, 26, 11, rsx, hist, nullptr);
      radix_pass(kb, mcnt, 15, 11, rsx, hist, nullptr);
      radix_pass(kb, mcnt, 4, 11, rsx, hist, nullptr);
      radix_pass(kb, mcnt, 0, 4, rsx, hist, nullptr);
    } else {
      radix_pass(kb, mcnt, 52, 11, rsx, hist, nullptr);
      radix_pass(kb, mcnt, 41, 11, rsx, hist, nullptr);
      radix_pass(kb, mcnt, 30, 11, rsx, hist, nullptr);
      radix_pass(kb, mcnt, 19, 11, rsx, hist, nullptr);
      radix_pass(kb, mcnt, 8, 11, rsx, hist, nullptr);
      radix_pass(kb, mcnt, 0, 8, rsx, hist, nullptr);
    }
    const unsigned long long lo_key = rsx.prefix;
    const double vlo = __longlong_as_double((long long)lo_key);
    double vhi = vlo;
    if (khi != klo) {
      if (rank_in + 1 < mcnt) {  // the upper middle rank is in the same bin
        uint32_t le = 0;
        unsigned long long gt = ~0ull;
        for (uint32_t k = threadIdx.x; k < mcnt; k += WLM_WG) {
          const unsigned long long key = absbits(kb[k]);
          if (key <= lo_key) ++le;
          else gt = key < gt ? key : gt;
        }
        for (int o = 32; o > 0; o >>= 1) {
          le += __shfl_xor(le, o);
          const unsigned long long og = (unsigned long long)__shfl_xor((long long)gt, o);
          gt = og < gt ? og : gt;
        }
        if (lane == 0) {
          atomicAdd(&le_s, le);
          atomicMin(&gt_s, gt);
        }
        __syncthreads();
        if (le_s <= rank_in + 1) vhi = __longlong_as_double((long long)gt_s);
      } else {  // it is the smallest key of the next nonempty bin
        unsigned long long nmin = ~0ull;
        for (uint32_t t = threadIdx.x; t < ncnt; t += WLM_WG) {
          unsigned long long key;
          if (BAND && BIOR) {
            if (in64) {
              key = wl_bior_dd1_key64(in64, img, Lt.h, Lt.w, pos_next[t], W1, c, mn, inv);
            } else {
              const rsrc_t rs = make_rsrc(src + (int64_t)img * Lt.h * row_stride,
                                          (uint32_t)((int64_t)Lt.h * row_stride));
              key = wl_bior_dd1_eval(wl_bior_dd1_load(rs, Lt.h, Lt.w, row_stride, pos_next[t], W1),
                                     c, mn, inv, rcp);
            }
          } else if (BAND) {
            key = absbits(band_dd[pos_next[t]]);
          } else {
            key = wl_dd1_key<MARK>(src, in64, img, Lt.h, Lt.w, row_stride, pos_next[t], W1, c, mn,
                                   inv, rcp);
          }
          nmin = key < nmin ? key : nmin;
        }
        for (int o = 32; o > 0; o >>= 1) {
          const unsigned long long on = (unsigned long long)__shfl_xor((long long)nmin, o);
          nmin = on < nmin ? on : nmin;
        }
        if (lane == 0) atomicMin(&nmin_s, nmin);
        __syncthreads();
        vhi = __longlong_as_double((long long)nmin_s);
      }
    }
    med = (vlo + vhi) / 2.0;  // np.median: mean of the two middle values
  }
  if (threadIdx.x == 0) {
    st[WlStats::median(c, Lt.L)] = med;
    st[WlStats::DIAG + c] = (double)total;  // diagnostics
  }
  if (part) wl_sums_thresh(st, part + img * Ls.part_per_img, c, Ls, Lt, med, mn, mx);
}

#include "haar3.hpp"

template <int L>
static void wl_run_haar(const uint8_t* src, const double* in64, uint8_t* out_u8, float* out_f32,
                        const WlLayout& Lt, int64_t row_stride, void* ws, hipStream_t st,
                  const unsigned long long* ycc_keys = nullptr) {
  wreal* wsf = (wreal*)ws;
  double* stats = (double*)((char*)ws + Lt.stats_off);
  double* part = (double*)((char*)ws + Lt.part_off);
  const int n = Lt.n;
  const int nthr = (Lt.h >> L) * (Lt.w >> L) * HaarSplit<L>::NS;
  const int nwg = (nthr + WLH_WG - 1) / WLH_WG;
  if constexpr (L == 3) {
    // round 6 (haar3.hpp): window sample, one statistics read, sigma, one synthesis read
    // (IDN_WAVELET_H3=0: the round-4 passes below); the window kernel also clears its image's
    // statistics block (wl_init_stats' values)
    const int nwg1 = h3_strips(Lt.w) * h3_chunks(Lt.h);
    if (src && !ycc_keys && knob("IDN_WAVELET_H3", 1) && (size_t)(3 * nwg1) <= Lt.part_per_img / 9) {
      hipLaunchKernelGGL(wl_h3_window, dim3(n), dim3(H3_WIN_WG), 0, st, src, Lt.h, Lt.w, row_stride,
                         stats, knob("IDN_WAVELET_H3FB", 0));
      hipLaunchKernelGGL(wl_h3_stats<false>, dim3(nwg1, n), dim3(WLH_WG), 0, st, src, Lt.h, Lt.w,
                         row_stride, wsf, Lt.img_floats, stats, part, Lt.part_per_img);
      hipLaunchKernelGGL(wl_h3_sigma, dim3(n * 3), dim3(WLM_WG), 0, st, src, row_stride, wsf,
                         Lt.img_floats, stats, Lt, (const double*)part, nwg1);
      const bool gen = out_f32 || !out_u8 || ((uintptr_t)out_u8 & 3) != 0;
      if (gen)
        hipLaunchKernelGGL(wl_h3_synth<true>, dim3(h3_strips(Lt.w) * h3s_chunks(Lt.h), n), dim3(WLH_WG), 0, st, src, Lt.h, Lt.w,
                           row_stride, (const double*)stats, out_u8, out_f32);
      else
        hipLaunchKernelGGL(wl_h3_synth<false>, dim3(h3_strips(Lt.w) * h3s_chunks(Lt.h), n), dim3(WLH_WG), 0, st, src, Lt.h,
                           Lt.w, row_stride, (const double*)stats, out_u8, (float*)nullptr);
      return;
    }
  }
  hipLaunchKernelGGL(wl_init_stats, dim3((n * WL_STATS + 255) / 256), dim3(256), 0, st, stats, n,
                     ycc_keys);
  if (!ycc_keys) {
    const int64_t np = (int64_t)Lt.h * Lt.w;
    // a few long-lived workgroups per image: per-wave reduction + atomics are the fixed cost
    int gx = (int)((np / 4 + 255) / 256);
    if (gx > 24) gx = 24;
    hipLaunchKernelGGL(wl_color_minmax, dim3(gx, n), dim3(256), 0, st, src, in64, Lt.h, Lt.w,
                       row_stride, stats);
  }
  int nwg_a;
  if constexpr (L >= 2) {
    if (src && knob("IDN_WAVELET_INTSTATS", 1)) {
      nwg_a = (nthr + WLH_WG * WLS_IT - 1) / (WLH_WG * WLS_IT);
      hipLaunchKernelGGL((wl_haar_stats<L>), dim3(nwg_a, n), dim3(WLH_WG), 0, st, src, Lt.h, Lt.w,
                         row_stride, wsf, Lt.img_floats, Lt.off_band[1], stats, part,
                         Lt.part_per_img);
    } else {
      nwg_a = (nthr + WLH_WG * WLH_IT - 1) / (WLH_WG * WLH_IT);
      hipLaunchKernelGGL((wl_haar_analyze<L>), dim3(nwg_a, n), dim3(WLH_WG), 0, st, src, in64,
                         Lt.h, Lt.w, row_stride, wsf, Lt.img_floats, Lt.off_band[1], stats, part,
                         Lt.part_per_img);
    }
  } else {
    nwg_a = (nthr + WLH_WG * WLH_IT - 1) / (WLH_WG * WLH_IT);
    hipLaunchKernelGGL((wl_haar_analyze<L>), dim3(nwg_a, n), dim3(WLH_WG), 0, st, src, in64, Lt.h,
                       Lt.w, row_stride, wsf, Lt.img_floats, Lt.off_band[1], stats, part,
                       Lt.part_per_img);
  }
  WlLayout Ls = Lt;  // wl_sumsq view of the fused partials: nwg per level, levels back to back
  for (int l = 1; l <= L; ++l) {
    Ls.tiles[l] = nwg_a;
    Ls.part_tile0[l] = (size_t)(l - 1) * nwg_a;
  }
  // the median workgroups also reduce the sums of squares and set the thresholds (wl_sumsq and
  // wl_thresh as separate launches: IDN_WAVELET_FUSETHR=0)
  if (knob("IDN_WAVELET_FUSETHR", 1)) {
    hipLaunchKernelGGL((wl_haar_median<L>), dim3(n * 3), dim3(WLM_WG), 0, st, src, in64, row_stride,
                       wsf, Lt.img_floats, stats, Lt, (const double*)part, Ls);
  } else {
    hipLaunchKernelGGL(wl_sumsq, dim3(n * 3 * L * 3), dim3(256), 0, st, stats, part, Ls);
    hipLaunchKernelGGL((wl_haar_median<L>), dim3(n * 3), dim3(WLM_WG), 0, st, src, in64, row_stride,
                       wsf, Lt.img_floats, stats, Lt, (const double*)nullptr, Ls);
    hipLaunchKernelGGL(wl_thresh, dim3(n), dim3(64), 0, st, stats, Lt);
  }
  if constexpr (L == 3) {
    // round 6: fp32 synthesis with the level-1 groups paired (IDN_WAVELET_H3S=0: the round-4
    // kernel below)
    if (src && knob("IDN_WAVELET_INTSYNTH", 1) && knob("IDN_WAVELET_H3S", 1)) {
      hipLaunchKernelGGL(wl_h3_consts, dim3((3 * n + 63) / 64), dim3(64), 0, st, stats, n);
      const bool gen = out_f32 || !out_u8 || ((uintptr_t)out_u8 & 3) != 0;
      if (gen)
        hipLaunchKernelGGL(wl_h3_synth<true>, dim3(h3_strips(Lt.w) * h3s_chunks(Lt.h), n), dim3(WLH_WG), 0, st, src, Lt.h, Lt.w,
                           row_stride, (const double*)stats, out_u8, out_f32);
      else
        hipLaunchKernelGGL(wl_h3_synth<false>, dim3(h3_strips(Lt.w) * h3s_chunks(Lt.h), n), dim3(WLH_WG), 0, st, src, Lt.h,
                           Lt.w, row_stride, (const double*)stats, out_u8, (float*)nullptr);
      return;
    }
  }
  if constexpr (L >= 2) {
    if (src && knob("IDN_WAVELET_INTSYNTH", 1)) {
      if (knob("IDN_WAVELET_HS32", 1))
        hipLaunchKernelGGL((wl_haar_synth_int<L, true>), dim3(nwg, n), dim3(WLH_WG), 0, st, src,
                           Lt.h, Lt.w, row_stride, stats, out_u8, out_f32);
      else
        hipLaunchKernelGGL((wl_haar_synth_int<L, false>), dim3(nwg, n), dim3(WLH_WG), 0, st, src,
                           Lt.h, Lt.w, row_stride, stats, out_u8, out_f32);
      return;
    }
  }
  hipLaunchKernelGGL((wl_haar_synth<L>), dim3(nwg, n), dim3(WLH_WG), 0, st, src, in64, Lt.h,
                     Lt.w, row_stride, stats, out_u8, out_f32);
}

// the fused path applies: db1, 1 <= L <= 3, both sides divisible by 2^L, room for its partials
static bool wl_haar_ok(int wavelet, const WlLayout& Lt, const uint8_t* src, int64_t row_stride) {
  if (wavelet != IDN_WAVELET_DB1 || Lt.L < 1 || Lt.L > 3 || knob("IDN_WAVELET_FUSED", 1) == 0)
    return false;
  const int B = 1 << Lt.L;
  if (Lt.h % B || Lt.w % B) return false;
  if (src && (((uintptr_t)src & 3) || (row_stride & 3))) return false;  // dword row loads
  const int64_t ns = Lt.L == 3 ? 4 : 1;
  const int64_t nwg = ((int64_t)(Lt.h / B) * (Lt.w / B) * ns + WLH_WG - 1) / WLH_WG;
  return (int64_t)Lt.L * nwg <= (int64_t)(Lt.part_per_img / 9);
}

template <int WV>
static int wl_run(const uint8_t* src, const double* in64, uint8_t* out_u8, float* out_f32,
                  const WlLayout& Lt, int64_t row_stride, void* ws, hipStream_t st,
                  const unsigned long long* ycc_keys = nullptr) {
  wreal* wsf = (wreal*)ws;
  double* stats = (double*)((char*)ws + Lt.stats_off);
  const int n = Lt.n;
  hipLaunchKernelGGL(wl_init_stats, dim3((n * WL_STATS + 255) / 256), dim3(256), 0, st, stats, n,
                     ycc_keys);
  if (!ycc_keys) {
    // u8 input in whole 8x8 blocks with dword-aligned rows: the Haar path's proxy min / max
    // (wl_h3_stats<true>: fp32 proxies, fp64 rescans of the steps near an extreme); else the
    // fp64 chain on every pixel
    if (src && knob("IDN_WAVELET_MMPROXY", 1) && Lt.h % 8 == 0 && Lt.w % 8 == 0 && row_stride % 4 == 0 &&
        ((uintptr_t)src & 3) == 0) {
      hipLaunchKernelGGL(wl_h3_stats<true>, dim3(h3_strips(Lt.w) * h3_chunks_mm(Lt.h), n), dim3(WLH_WG), 0, st,
                         src, Lt.h, Lt.w, row_stride, wsf, Lt.img_floats, stats, (double*)nullptr,
                         (size_t)0);
    } else {
      const int64_t np = (int64_t)Lt.h * Lt.w;
      // a few long-lived workgroups per image: per-wave reduction + atomics are the fixed cost
      int gx = (int)((np / 4 + 255) / 256);
      if (gx > 24) gx = 24;
      hipLaunchKernelGGL(wl_color_minmax, dim3(gx, n), dim3(256), 0, st, src, in64, Lt.h, Lt.w,
                         row_stride, stats);
    }
  }
  double* part = (double*)((char*)ws + Lt.part_off);
  // sigma from level-1 dd codes (wl_haar_median<.., true>) when the channel's input-plane slot
  // holds codes + keys + positions (2.25 band sizes); else the radix select over the band
  const size_t bsz1 = (size_t)Lt.H[1] * Lt.W[1];
  const bool codes = knob("IDN_WAVELET_CODEMED", 1) && (bsz1 + 3) / 4 + 2 * bsz1 <= (size_t)Lt.h * Lt.w;
  const bool fdet = knob("IDN_WAVELET_FDET", 1) != 0;
  // bior1.5 with the code median: the level-1 dd band in fp32 too (the median recomputes its
  // exact values from the input, bior_dd2x2; the synthesis reads it as fp32 either way)
  const bool dd32 = WV == IDN_WAVELET_BIOR15 && codes && fdet && knob("IDN_WAVELET_DD32", 1) != 0;
  // band masks (wl_fband): level 1 / deeper levels, analysis stores and synthesis loads
  auto fm_an = [&](int l) {
    if (!fdet) return 0;
    return (l == 1 ? (dd32 ? 0b1110 : 0b0110) : 0b1110 | WL_FB_AIN) | (l < Lt.L ? 0b0001 : 0);
  };
  auto fm_syn = [&](int l) { return !fdet ? 0 : (l == 1 && !dd32 ? 0b0110 : 0b1110); };
  const int coop = knob("IDN_WAVELET_COOP", 1) ? 1 : 0;
  const int a32 = knob("IDN_WAVELET_A32", 3);
  for (int l = 1; l <= Lt.L; ++l) {
    const size_t in_off = l == 1 ? 0 : Lt.off_band[l - 1];
    if (WV == IDN_WAVELET_BIOR15) {
      const int sw = ws_sw(Lt.W[l]);
      const int strips = Lt.tiles_x[l], bands = Lt.bands[l], groups = (Lt.H[l] + WS_G - 1) / WS_G;
      const dim3 grid((unsigned)(strips * bands), 1, (unsigned)n);
      const dim3 blk((unsigned)((2 * sw + 8 + 63) / 64 * 64));
      const int Hi = Lt.H[l - 1], Wi = Lt.W[l - 1], emit = (l == 1 && codes) ? 1 : 0;
      // IDN_WAVELET_A32 bit 0: level 1's lowpass path in fp32; bit 1: deeper levels in fp32;
      // bit 2 (with bit 0, u8 input and the code median): level 1's normalisation and highpass
      // in fp32 too, the codes from exact integer keys (wl_dwt_stream's N32; sigma bit-identical
      // by test, but 1041 vs 849 us per 256 images: gfx950 issues fp64 FMA at the fp32 rate, and
      // the key staging adds instructions and registers -- profiles/r06/wavelet/n32_ab.txt)
#define IDN_WS_(SRC, TL, TH, FMC, CC, EMIT)                                                        \
  hipLaunchKernelGGL((wl_dwt_stream<SRC, TL, TH, FMC, CC>), grid, blk, 0, st, wsf, Lt.img_floats,  \
                     stats, in_off, Hi, Wi, Lt.off_band[l], Lt.H[l], Lt.W[l], sw, strips, bands,   \
                     groups, src, in64, row_stride, part, Lt.part_per_img, Lt.part_tile0[l], EMIT, \
                     fm_an(l), Lt.sq_grid[l])
      // the product's band masks as compile-time constants (bit 4 = WL_FB_AIN is read by the
      // launcher only); anything else (tuning forms) through the runtime-mask instance
#define IDN_WS(SRC, TL, TH, EMIT)                                                                  \
  do {                                                                                             \
    const int fmb = fm_an(l) & 0b1111;                                                             \
    if ((SRC == 0 || SRC == 1) && fmb == 0b1111 && (EMIT) == 1)                                    \
      IDN_WS_(SRC, TL, TH, 0b1111, 1, EMIT);                                                       \
    else if (SRC == 0 && fmb == 0b1110 && (EMIT) == 1) IDN_WS_(SRC, TL, TH, 0b1110, 1, EMIT);      \
    else if (SRC == 0 && fmb == 0b0111 && (EMIT) == 1) IDN_WS_(SRC, TL, TH, 0b0111, 1, EMIT);      \
    else if (SRC == 0 && fmb == 0b0110 && (EMIT) == 1) IDN_WS_(SRC, TL, TH, 0b0110, 1, EMIT);      \
    else if (SRC == 3 && fmb == 0b1111) IDN_WS_(SRC, TL, TH, 0b1111, 0, EMIT);                     \
    else if (SRC == 3 && fmb == 0b1110) IDN_WS_(SRC, TL, TH, 0b1110, 0, EMIT);                     \
    else IDN_WS_(SRC, TL, TH, -1, -1, EMIT);                                                       \
  } while (0)
      const bool f1 = (a32 & 1) != 0, fd = (a32 & 2) != 0;
      if (l > 1 && (fm_an(l) & WL_FB_AIN)) {
        if (fd) IDN_WS(3, float, float, 0);
        else IDN_WS(3, wreal, wreal, 0);
      } else if (l > 1) {
        if (fd) IDN_WS(2, float, float, 0);
        else IDN_WS(2, wreal, wreal, 0);
      } else if (in64) {
        if (f1) IDN_WS(1, float, wreal, emit);
        else IDN_WS(1, wreal, wreal, emit);
      } else if (f1 && (a32 & 4) && emit && dd32) {
        // the whole level-1 analysis in fp32, codes from the exact integer keys (N32; A/B form)
        IDN_WS(0, float, float, emit);
      } else {
        if (f1) IDN_WS(0, float, wreal, emit);
        else IDN_WS(0, wreal, wreal, emit);
      }
#undef IDN_WS
#undef IDN_WS_
    } else if (l > 1)
      hipLaunchKernelGGL((wl_dwt_rb<WV, 2>), dim3(Lt.tiles[l], 1, n), dim3(256), 0, st, wsf, Lt.img_floats, stats,
                         in_off, Lt.H[l - 1], Lt.W[l - 1], Lt.off_band[l], Lt.H[l], Lt.W[l],
                         Lt.tiles_x[l], src, in64, row_stride, part, Lt.part_per_img,
                         Lt.part_tile0[l], 0, fm_an(l), coop);
    else if (in64)
      hipLaunchKernelGGL((wl_dwt_rb<WV, 1>), dim3(Lt.tiles[1], 1, n), dim3(256), 0, st, wsf, Lt.img_floats, stats,
                         in_off, Lt.H[0], Lt.W[0], Lt.off_band[1], Lt.H[1], Lt.W[1],
                         Lt.tiles_x[1], src, in64, row_stride, part, Lt.part_per_img,
                         Lt.part_tile0[1], codes ? 1 : 0, fm_an(1), coop);
    else
      hipLaunchKernelGGL((wl_dwt_rb<WV, 0>), dim3(Lt.tiles[1], 1, n), dim3(256), 0, st, wsf, Lt.img_floats, stats,
                         in_off, Lt.H[0], Lt.W[0], Lt.off_band[1], Lt.H[1], Lt.W[1],
                         Lt.tiles_x[1], src, in64, row_stride, part, Lt.part_per_img,
                         Lt.part_tile0[1], codes ? 1 : 0, fm_an(1), coop);
  }
  // the code medians also reduce the sums of squares and set the thresholds (see wl_haar_median)
  const bool fuse = codes && knob("IDN_WAVELET_FUSETHR", 1);
  const double* part_f = fuse ? (const double*)part : nullptr;
  if (!fuse)
    hipLaunchKernelGGL(wl_sumsq, dim3(n * 3 * Lt.L * 3), dim3(256), 0, st, stats, part, Lt);
  if (codes && dd32)
    hipLaunchKernelGGL((wl_haar_median<1, true, true>), dim3(n * 3), dim3(WLM_WG), 0, st, src, in64,
                       row_stride, wsf, Lt.img_floats, stats, Lt, part_f, Lt);
  else if (codes)
    hipLaunchKernelGGL((wl_haar_median<1, true>), dim3(n * 3), dim3(WLM_WG), 0, st, src, in64,
                       row_stride, wsf, Lt.img_floats, stats, Lt, part_f, Lt);
  else
    hipLaunchKernelGGL(wl_median, dim3(n * 3), dim3(1024), 0, st, wsf, Lt.img_floats, stats, Lt);
  if (!fuse) hipLaunchKernelGGL(wl_thresh, dim3(n), dim3(64), 0, st, stats, Lt);
  // bior1.5 synthesis form per level (bit 0: level 1, bit 1: deeper levels): streaming
  // (wl_synth_stream) or tiled (wl_synth / wl_synth_final)
  const int sstream = WV == IDN_WAVELET_BIOR15 ? knob("IDN_WAVELET_SSTREAM", 3) : 0;
  // streaming levels in fp32 arithmetic (wl_synth_stream<.., float>); a level >= 2 that is then
  // stores its reconstruction as fp32, so the level below reads its 'aa' band as fp32 (bit 0)
  const bool s32 = knob("IDN_WAVELET_S32", 1) != 0;
  // fp32 level 1 with all three channels per thread (wl_synth_final3)
  const bool s3 = knob("IDN_WAVELET_S3", 1) != 0;
  // ... and at the deeper levels whose output is at least this wide (0: every level; measured
  // 2.93 -> 2.85 ms per 256 images against wl_synth_stream<false, float> at levels >= 2, and no
  // better with a width floor of 200 or 384: profiles/r03/wavelet/s3d_ab.txt)
  const int s3d = knob("IDN_WAVELET_S3D", 0);
  auto str = [&](int l) { return (sstream & (l == 1 ? 1 : 2)) != 0; };
  auto fm_syn2 = [&](int l) { return fm_syn(l) | (l < Lt.L && str(l + 1) && s32 ? 0b0001 : 0); };
  if (sstream) {
    for (int l = Lt.L; l >= 1; --l) {
      if (!str(l)) {
        if (l >= 2) {
          const int tx = (Lt.W[l - 1] + ST_O - 1) / ST_O, ty = (Lt.H[l - 1] + ST_O - 1) / ST_O;
          hipLaunchKernelGGL((wl_synth<WV>), dim3(tx * ty, n * 3), dim3(256), 0, st, wsf,
                             Lt.img_floats, stats, l, Lt.L, Lt.off_band[l], Lt.H[l], Lt.W[l],
                             Lt.off_band[l - 1], Lt.H[l - 1], Lt.W[l - 1],
                             (size_t)4 * Lt.H[l - 1] * Lt.W[l - 1], tx, fm_syn2(l));
        } else {
          const int tx = (Lt.w + ST_O - 1) / ST_O, ty = (Lt.h + ST_O - 1) / ST_O;
          hipLaunchKernelGGL((wl_synth_final<WV>), dim3(tx * ty, n), dim3(256), 0, st, wsf,
                             Lt.img_floats, stats, Lt.L, Lt.off_band[1], Lt.H[1], Lt.W[1], Lt.h,
                             Lt.w, tx, out_u8, row_stride, out_f32, fm_syn2(1));
        }
        continue;
      }
      const int Hout = Lt.H[l - 1], Wout = Lt.W[l - 1];
      const int strips = ss_strips(Wout), sw = ss_sw(Wout);
      const int bands = ss_bands_occ(
          n, (Hout + 1) / 2, strips,
          reinterpret_cast<const void*>(&wl_synth_stream<false, float>), SS_MAXT);
      const dim3 grid((unsigned)(strips * bands), 1, (unsigned)n), blk(SS_MAXT);
      const int fm2 = fm_syn2(l);
      if (l >= 2 && s32 && s3 && Wout >= s3d && (fm2 == 0b1111 || fm2 == 0b1110)) {
        const int strips3 = s3_strips(Wout), sw3 = s3_sw(Wout);
        const int bands3 = ss_bands_occ(
            n, (Hout + 1) / 2, strips3,
            reinterpret_cast<const void*>(&wl_synth_final3<0b1111, false>), S3_T);
        const dim3 grid3((unsigned)(strips3 * bands3), 1, (unsigned)n);
        if (fm2 == 0b1111)
          hipLaunchKernelGGL((wl_synth_final3<0b1111, false>), grid3, dim3(S3_T), 0, st, wsf,
                             Lt.img_floats, stats, Lt.L, Lt.off_band[l], Lt.H[l], Lt.W[l], Hout,
                             Wout, sw3, strips3, bands3, (uint8_t*)nullptr, row_stride,
                             (float*)nullptr, l, Lt.off_band[l - 1], (size_t)4 * Hout * Wout);
        else
          hipLaunchKernelGGL((wl_synth_final3<0b1110, false>), grid3, dim3(S3_T), 0, st, wsf,
                             Lt.img_floats, stats, Lt.L, Lt.off_band[l], Lt.H[l], Lt.W[l], Hout,
                             Wout, sw3, strips3, bands3, (uint8_t*)nullptr, row_stride,
                             (float*)nullptr, l, Lt.off_band[l - 1], (size_t)4 * Hout * Wout);
      } else if (l >= 2) {
        if (s32)
          hipLaunchKernelGGL((wl_synth_stream<false, float>), grid, blk, 0, st, wsf, Lt.img_floats,
                             stats, l, Lt.L, Lt.off_band[l], Lt.H[l], Lt.W[l], Lt.off_band[l - 1],
                             Hout, Wout, (size_t)4 * Hout * Wout, fm_syn2(l), sw, strips, bands,
                             (uint8_t*)nullptr, row_stride, (float*)nullptr);
        else
          hipLaunchKernelGGL((wl_synth_stream<false>), grid, blk, 0, st, wsf, Lt.img_floats, stats,
                             l, Lt.L, Lt.off_band[l], Lt.H[l], Lt.W[l], Lt.off_band[l - 1], Hout,
                             Wout, (size_t)4 * Hout * Wout, fm_syn2(l), sw, strips, bands,
                             (uint8_t*)nullptr, row_stride, (float*)nullptr);
      } else if (s32 && s3 && (fm_syn2(1) & 0b0110) == 0b0110) {
        const int strips3 = s3_strips(Wout), sw3 = s3_sw(Wout);
        const int bands3 = ss_bands_occ(n, (Hout + 1) / 2, strips3,
                                        reinterpret_cast<const void*>(&wl_synth_final3<0b0111>), S3_T);
        const dim3 grid3((unsigned)(strips3 * bands3), 1, (unsigned)n);
        if (fm_syn2(1) == 0b1111)
          hipLaunchKernelGGL((wl_synth_final3<0b1111>), grid3, dim3(S3_T), 0, st, wsf,
                             Lt.img_floats, stats, Lt.L, Lt.off_band[1], Lt.H[1], Lt.W[1], Lt.h,
                             Lt.w, sw3, strips3, bands3, out_u8, row_stride, out_f32);
        else if (fm_syn2(1) == 0b1110)
          hipLaunchKernelGGL((wl_synth_final3<0b1110>), grid3, dim3(S3_T), 0, st, wsf,
                             Lt.img_floats, stats, Lt.L, Lt.off_band[1], Lt.H[1], Lt.W[1], Lt.h,
                             Lt.w, sw3, strips3, bands3, out_u8, row_stride, out_f32);
        else if (fm_syn2(1) == 0b0111)
          hipLaunchKernelGGL((wl_synth_final3<0b0111>), grid3, dim3(S3_T), 0, st, wsf,
                             Lt.img_floats, stats, Lt.L, Lt.off_band[1], Lt.H[1], Lt.W[1], Lt.h,
                             Lt.w, sw3, strips3, bands3, out_u8, row_stride, out_f32);
        else
          hipLaunchKernelGGL((wl_synth_final3<0b0110>), grid3, dim3(S3_T), 0, st, wsf,
                             Lt.img_floats, stats, Lt.L, Lt.off_band[1], Lt.H[1], Lt.W[1], Lt.h,
                             Lt.w, sw3, strips3, bands3, out_u8, row_stride, out_f32);
      } else if (s32) {
        hipLaunchKernelGGL((wl_synth_stream<true, float>), grid, blk, 0, st, wsf, Lt.img_floats,
                           stats, 1, Lt.L, Lt.off_band[1], Lt.H[1], Lt.W[1], (size_t)0, Lt.h, Lt.w,
                           (size_t)0, fm_syn2(1), sw, strips, bands, out_u8, row_stride, out_f32);
      } else {
        hipLaunchKernelGGL((wl_synth_stream<true>), grid, blk, 0, st, wsf, Lt.img_floats, stats, 1,
                           Lt.L, Lt.off_band[1], Lt.H[1], Lt.W[1], (size_t)0, Lt.h, Lt.w, (size_t)0,
                           fm_syn2(1), sw, strips, bands, out_u8, row_stride, out_f32);
      }
    }
    return IDN_OK;
  }
  for (int l = Lt.L; l >= 2; --l) {
    // the level-(l-1) 'aa' slot (consumed by the analysis already) receives the reconstruction
    const int tx = (Lt.W[l - 1] + ST_O - 1) / ST_O, ty = (Lt.H[l - 1] + ST_O - 1) / ST_O;
    hipLaunchKernelGGL((wl_synth<WV>), dim3(tx * ty, n * 3), dim3(256), 0, st, wsf, Lt.img_floats,
                       stats, l, Lt.L, Lt.off_band[l], Lt.H[l], Lt.W[l], Lt.off_band[l - 1],
                       Lt.H[l - 1], Lt.W[l - 1], (size_t)4 * Lt.H[l - 1] * Lt.W[l - 1], tx, fm_syn(l));
  }
  {
    const int tx = (Lt.w + ST_O - 1) / ST_O, ty = (Lt.h + ST_O - 1) / ST_O;
    hipLaunchKernelGGL((wl_synth_final<WV>), dim3(tx * ty, n), dim3(256), 0, st, wsf,
                       Lt.img_floats, stats, Lt.L, Lt.off_band[1], Lt.H[1], Lt.W[1], Lt.h, Lt.w,
                       tx, out_u8, row_stride, out_f32, fm_syn(1));
  }
  return IDN_OK;
}

}  // namespace idn

extern "C" size_t idn_wavelet_workspace_size(int n, int h, int w, int wavelet, int levels) {
  using namespace idn;
  if (n <= 0 || h <= 0 || w <= 0 || (wavelet != IDN_WAVELET_DB1 && wavelet != IDN_WAVELET_BIOR15))
    return 0;
  return wl_layout(n, h, w, wavelet, levels).bytes;
}

extern "C" size_t idn_wavelet_stats_offset(int n, int h, int w, int wavelet, int levels) {
  using namespace idn;
  if (n <= 0 || h <= 0 || w <= 0 || (wavelet != IDN_WAVELET_DB1 && wavelet != IDN_WAVELET_BIOR15))
    return 0;
  return wl_layout(n, h, w, wavelet, levels).stats_off;
}

namespace idn {
static int wavelet_impl(const uint8_t* src, const double* in_f64,
                        const unsigned long long* ycc_keys, uint8_t* out_u8, float* out_f32, int n,
                        int h, int w, int64_t row_stride, int wavelet, int levels, void* workspace,
                        size_t ws_bytes, void* stream) {
  IDN_CHECK_ARG(src || in_f64, "idn_wavelet_denoise_u8: no input");
  IDN_CHECK_ARG(out_u8 || out_f32, "idn_wavelet_denoise_u8: no output");
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0, "idn_wavelet_denoise_u8: bad shape");
  IDN_CHECK_ARG((int64_t)h * w < ((int64_t)1 << 31), "idn_wavelet_denoise_u8: image too large");
  IDN_CHECK_ARG(row_stride >= (int64_t)w * 3, "idn_wavelet_denoise_u8: row_stride < w*3");
  IDN_CHECK_ARG(wavelet == IDN_WAVELET_DB1 || wavelet == IDN_WAVELET_BIOR15,
                "idn_wavelet_denoise_u8: unknown wavelet %d", wavelet);
  if (n == 0) return IDN_OK;
  const WlLayout Lt = wl_layout(n, h, w, wavelet, levels);
  IDN_CHECK_ARG(Lt.L >= 1 && Lt.L <= WL_MAXL, "idn_wavelet_denoise_u8: levels %d out of range", Lt.L);
  // pywt needs every level's input at least one sample long; skimage warns but proceeds
  for (int l = 1; l <= Lt.L; ++l)
    IDN_CHECK_ARG(Lt.H[l - 1] >= 1 && Lt.W[l - 1] >= 1, "idn_wavelet_denoise_u8: image too small");
  if (!workspace || ws_bytes < Lt.bytes)
    return set_error(IDN_EWORKSPACE, "idn_wavelet_denoise_u8: needs %zu workspace bytes (got %zu)",
                     Lt.bytes, ws_bytes);
  hipStream_t st = as_stream(stream);
  const unsigned long long* K = ycc_keys;
  if (wl_haar_ok(wavelet, Lt, src, row_stride)) {
    if (Lt.L == 1) wl_run_haar<1>(src, in_f64, out_u8, out_f32, Lt, row_stride, workspace, st, K);
    else if (Lt.L == 2) wl_run_haar<2>(src, in_f64, out_u8, out_f32, Lt, row_stride, workspace, st, K);
    else wl_run_haar<3>(src, in_f64, out_u8, out_f32, Lt, row_stride, workspace, st, K);
  } else if (wavelet == IDN_WAVELET_DB1) {
    wl_run<IDN_WAVELET_DB1>(src, in_f64, out_u8, out_f32, Lt, row_stride, workspace, st, K);
  } else {
    wl_run<IDN_WAVELET_BIOR15>(src, in_f64, out_u8, out_f32, Lt, row_stride, workspace, st, K);
  }
  IDN_CHECK_LAUNCH("idn_wavelet_denoise_u8");
  return IDN_OK;
}
}  // namespace idn

extern "C" int idn_wavelet_denoise_u8(const uint8_t* src, const double* in_f64, uint8_t* out_u8,
                                      float* out_f32, int n, int h, int w, int64_t row_stride,
                                      int wavelet, int levels, void* workspace, size_t ws_bytes,
                                      void* stream) {
  return idn::wavelet_impl(src, in_f64, nullptr, out_u8, out_f32, n, h, w, row_stride, wavelet,
                           levels, workspace, ws_bytes, stream);
}

extern "C" int idn_wavelet_denoise_ycc(const double* in_f64, const uint64_t* ycc_keys,
                                       uint8_t* out_u8, float* out_f32, int n, int h, int w,
                                       int wavelet, int levels, void* workspace, size_t ws_bytes,
                                       void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(in_f64 && ycc_keys, "idn_wavelet_denoise_ycc: null input or keys");
  return wavelet_impl(nullptr, in_f64, reinterpret_cast<const unsigned long long*>(ycc_keys),
                      out_u8, out_f32, n, h, w, (int64_t)w * 3, wavelet, levels, workspace,
                      ws_bytes, stream);
}
