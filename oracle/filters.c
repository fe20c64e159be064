/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, imported by or called from the product
 * path (image-denoising_amd/).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it, and only as the checker / the timed CPU baseline.
 *
 * Plain-C restatement of the OpenCV 3.4.2 8-bit filters the reference calls on its hot path
 * (OpenCV is pinned at requirements.txt:89,121,141 and is NOT importable in this image, so these
 * are restated from the library's published algorithm):
 *
 *   cv2.GaussianBlur(u8,(k,k),0)  lib/model/test.py:224, lib/roi_data_layer/minibatch.py:119,1636
 *   cv2.blur(u8,(3,3))            lib/model/test.py:241,1767, minibatch.py:136,1640
 *   cv2.medianBlur(u8,k)          lib/model/test.py:259, minibatch.py:153,1644
 *   cv2.bilateralFilter(u8,d,sc,ss,BORDER_CONSTANT)  lib/model/test.py:278, minibatch.py:172,1658
 *
 * Pinning: the integer filters are cross-checked against scipy.ndimage (tests/test_oracle.py:
 * correlate(mode='mirror') == BORDER_REFLECT_101, median_filter(mode='nearest') ==
 * BORDER_REPLICATE).  Bilateral has no independent implementation in this image: parity vs
 * cv2 is UNPINNED; it is checked against an fp64 numpy restatement only.
 *
 * Images: n x h x w x c uint8, row pitch `rs` bytes, image pitch h*rs.  OpenMP over rows.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int refl101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}
static int clampi(int i, int n) { return i < 0 ? 0 : (i >= n ? n - 1 : i); }

/* GaussianBlur, sigma=0, ksize<=7: OpenCV's fixed small kernels ([1 2 1]/4, [1 4 6 4 1]/16);
 * 8U result = round-half-up of the exact dyadic sum (fixed-point path). */
void oracle_gaussian_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                        int64_t rs, int k) {
  static const int k3[3] = {1, 2, 1};
  static const int k5[5] = {1, 4, 6, 4, 1};
  const int* a = (k == 3) ? k3 : k5;
  const int R = k / 2;
  const int shift = (k == 3) ? 4 : 8;
  for (int img = 0; img < n; ++img) {
    const uint8_t* s = src + (int64_t)img * h * rs;
    uint8_t* d = dst + (int64_t)img * h * rs;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x)
        for (int ch = 0; ch < c; ++ch) {
          int S = 0;
          for (int i = -R; i <= R; ++i) {
            const uint8_t* row = s + (int64_t)refl101(y + i, h) * rs;
            for (int j = -R; j <= R; ++j)
              S += a[i + R] * a[j + R] * row[(int64_t)refl101(x + j, w) * c + ch];
          }
          d[(int64_t)y * rs + (int64_t)x * c + ch] = (uint8_t)((S + (1 << (shift - 1))) >> shift);
        }
  }
}

/* blur (normalised box), BORDER_REFLECT_101; u8 = round(S/k^2) (never a tie for k=3). */
void oracle_box_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c, int64_t rs,
                   int k) {
  const int R = k / 2;
  const int kk = k * k;
  for (int img = 0; img < n; ++img) {
    const uint8_t* s = src + (int64_t)img * h * rs;
    uint8_t* d = dst + (int64_t)img * h * rs;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x)
        for (int ch = 0; ch < c; ++ch) {
          int S = 0;
          for (int i = -R; i <= R; ++i) {
            const uint8_t* row = s + (int64_t)refl101(y + i, h) * rs;
            for (int j = -R; j <= R; ++j) S += row[(int64_t)refl101(x + j, w) * c + ch];
          }
          d[(int64_t)y * rs + (int64_t)x * c + ch] = (uint8_t)((2 * S + kk) / (2 * kk));
        }
  }
}

/* medianBlur 8U: exact median of the k x k window per channel, BORDER_REPLICATE. */
void oracle_median_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c, int64_t rs,
                      int k) {
  const int R = k / 2;
  const int kk = k * k;
  for (int img = 0; img < n; ++img) {
    const uint8_t* s = src + (int64_t)img * h * rs;
    uint8_t* d = dst + (int64_t)img * h * rs;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x)
        for (int ch = 0; ch < c; ++ch) {
          int hist[256];
          memset(hist, 0, sizeof(hist));
          for (int i = -R; i <= R; ++i) {
            const uint8_t* row = s + (int64_t)clampi(y + i, h) * rs;
            for (int j = -R; j <= R; ++j) hist[row[(int64_t)clampi(x + j, w) * c + ch]]++;
          }
          int acc = 0, v = 0;
          for (v = 0; v < 256; ++v) {
            acc += hist[v];
            if (acc > kk / 2) break;
          }
          d[(int64_t)y * rs + (int64_t)x * c + ch] = (uint8_t)v;
        }
  }
}

/* bilateralFilter_8u (OpenCV 3.4.2 imgproc/smooth.cpp): radius = d/2 (d<=0: round(1.5*ss)),
 * taps with sqrt(i^2+j^2) <= radius, float LUTs from double exp, border = constant 0,
 * float accumulation, out = cvRound(sum * (1.f/wsum)).  Scalar tap order (row-major i, j). */
void oracle_bilateral_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                         int64_t rs, int d, double sigma_color, double sigma_space) {
  if (sigma_color <= 0) sigma_color = 1;
  if (sigma_space <= 0) sigma_space = 1;
  const double gcc = -0.5 / (sigma_color * sigma_color);
  const double gsc = -0.5 / (sigma_space * sigma_space);
  int radius = (d <= 0) ? (int)lrint(sigma_space * 1.5) : d / 2;
  if (radius < 1) radius = 1;
  const int dd = 2 * radius + 1;
  float* cw = (float*)malloc(sizeof(float) * 256 * c);
  float* sw = (float*)malloc(sizeof(float) * dd * dd);
  int* oy = (int*)malloc(sizeof(int) * dd * dd);
  int* ox = (int*)malloc(sizeof(int) * dd * dd);
  for (int i = 0; i < 256 * c; ++i) cw[i] = (float)exp((double)i * i * gcc);
  int maxk = 0;
  for (int i = -radius; i <= radius; ++i)
    for (int j = -radius; j <= radius; ++j) {
      double r = sqrt((double)i * i + (double)j * j);
      if (r > radius) continue;
      sw[maxk] = (float)exp(r * r * gsc);
      oy[maxk] = i;
      ox[maxk] = j;
      ++maxk;
    }
  for (int img = 0; img < n; ++img) {
    const uint8_t* s = src + (int64_t)img * h * rs;
    uint8_t* dp = dst + (int64_t)img * h * rs;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        const uint8_t* p0 = s + (int64_t)y * rs + (int64_t)x * c;
        float sum[4] = {0, 0, 0, 0}, wsum = 0;
        for (int t = 0; t < maxk; ++t) {
          const int yy = y + oy[t], xx = x + ox[t];
          int v[4] = {0, 0, 0, 0};
          if (yy >= 0 && yy < h && xx >= 0 && xx < w) {
            const uint8_t* p = s + (int64_t)yy * rs + (int64_t)xx * c;
            for (int ch = 0; ch < c; ++ch) v[ch] = p[ch];
          }
          int diff = 0;
          for (int ch = 0; ch < c; ++ch) diff += abs(v[ch] - (int)p0[ch]);
          const float wt = sw[t] * cw[diff];
          for (int ch = 0; ch < c; ++ch) sum[ch] += (float)v[ch] * wt;
          wsum += wt;
        }
        const float inv = 1.f / wsum;
        for (int ch = 0; ch < c; ++ch) {
          float r = sum[ch] * inv;
          int q = (int)lrintf(r); /* cvRound: round half to even */
          dp[(int64_t)y * rs + (int64_t)x * c + ch] = (uint8_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
        }
      }
  }
  free(cw);
  free(sw);
  free(oy);
  free(ox);
}

/* bilateral pre-round float values (n*h*w*c floats) for tolerance checks */
void oracle_bilateral_f32(const uint8_t* src, float* out, int n, int h, int w, int c, int64_t rs,
                          int d, double sigma_color, double sigma_space) {
  if (sigma_color <= 0) sigma_color = 1;
  if (sigma_space <= 0) sigma_space = 1;
  const double gcc = -0.5 / (sigma_color * sigma_color);
  const double gsc = -0.5 / (sigma_space * sigma_space);
  int radius = (d <= 0) ? (int)lrint(sigma_space * 1.5) : d / 2;
  if (radius < 1) radius = 1;
  for (int img = 0; img < n; ++img) {
    const uint8_t* s = src + (int64_t)img * h * rs;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        const uint8_t* p0 = s + (int64_t)y * rs + (int64_t)x * c;
        double sum[4] = {0, 0, 0, 0}, wsum = 0;
        for (int i = -radius; i <= radius; ++i)
          for (int j = -radius; j <= radius; ++j) {
            double r = sqrt((double)i * i + (double)j * j);
            if (r > radius) continue;
            const int yy = y + i, xx = x + j;
            int v[4] = {0, 0, 0, 0};
            if (yy >= 0 && yy < h && xx >= 0 && xx < w) {
              const uint8_t* p = s + (int64_t)yy * rs + (int64_t)xx * c;
              for (int ch = 0; ch < c; ++ch) v[ch] = p[ch];
            }
            int diff = 0;
            for (int ch = 0; ch < c; ++ch) diff += abs(v[ch] - (int)p0[ch]);
            const double wt =
                (double)(float)exp(r * r * gsc) * (double)(float)exp((double)diff * diff * gcc);
            for (int ch = 0; ch < c; ++ch) sum[ch] += v[ch] * wt;
            wsum += wt;
          }
        float* o = out + (((int64_t)img * h + y) * w + x) * c;
        for (int ch = 0; ch < c; ++ch) o[ch] = (float)(sum[ch] / wsum);
      }
  }
}

/* numpy `arr @ M.T` for (n,3) x (3,3) float64 as OpenBLAS's dgemm kernels evaluate it on x86-64
 * with FMA (an fma chain over k, checked bit-for-bit against numpy 1.26 / 2.2 in this image), with
 * skimage's offsets: out = fma(x2', M[k][2], fma(x1', M[k][1], x0' * M[k][0])) + post[k], where
 * x' = x - pre (rgb2ycbcr: pre = 0, post = [16,128,128]; ycbcr2rgb: pre = [16,128,128], post = 0).
 * Used by oracle/wavelet.py so the oracle does not depend on the host BLAS kernel. */
void oracle_matmul3_fma(const double* in, double* out, int64_t n, const double* M,
                        const double* pre, const double* post) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const double x0 = in[3 * i] - pre[0], x1 = in[3 * i + 1] - pre[1], x2 = in[3 * i + 2] - pre[2];
    for (int k = 0; k < 3; ++k) {
      const double* m = M + 3 * k;
      const double d = fma(x2, m[2], fma(x1, m[1], x0 * m[0]));
      out[3 * i + k] = d + post[k];
    }
  }
}
