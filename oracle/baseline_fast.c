/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  The CPU baseline bench.py times (cpu_baseline leg), never
 * linked into or called from the product path.
 *
 * A fast host restatement of cv2.GaussianBlur(u8, (5,5), 0) / (3,3) (lib/model/test.py:224,
 * lib/roi_data_layer/minibatch.py:119,1636-1639), written the way OpenCV's own 8-bit path works
 * so the baseline is a fair stand-in for the reference's cv2 CPU path (cv2 is not installable
 * here):  separable, a horizontal pass into 16-bit row sums, a vertical pass over a 5-row ring of
 * them, all 16-bit lanes the compiler vectorises (built for x86-64-v3: AVX2),
 * OpenMP over (image, row strip).  Results are bit-exact with oracle_gaussian_u8 (filters.c):
 * the 5x5 sum fits 16 bits (16 * 16 * 255 + 128 = 65408).  BORDER_REFLECT_101.
 */
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

/* horizontal [1 4 6 4 1] (K=5) or [1 2 1] (K=3) of one interleaved row into 16-bit sums */
static void hpass(const uint8_t* restrict row, uint16_t* restrict out, int w, int c, int K) {
  const int n = w * c, R = K / 2, b = R * c;
  for (int x = 0; x < n; ++x) {
    if (x >= b && x < n - b) break;
    const int px = x / c, ch = x % c;
    unsigned s = 0;
    for (int j = -R; j <= R; ++j) {
      const unsigned v = row[refl101(px + j, w) * c + ch];
      const unsigned wt = K == 5 ? (j == 0 ? 6u : (j == 1 || j == -1) ? 4u : 1u)
                                 : (j == 0 ? 2u : 1u);
      s += wt * v;
    }
    out[x] = (uint16_t)s;
  }
  if (K == 5) {
    for (int x = b; x < n - b; ++x)
      out[x] = (uint16_t)(row[x - 2 * c] + row[x + 2 * c] + 4 * (row[x - c] + row[x + c]) +
                          6 * row[x]);
  } else {
    for (int x = b; x < n - b; ++x) out[x] = (uint16_t)(row[x - c] + row[x + c] + 2 * row[x]);
  }
  for (int x = (n - b > b ? n - b : b); x < n; ++x) {
    const int px = x / c, ch = x % c;
    unsigned s = 0;
    for (int j = -R; j <= R; ++j) {
      const unsigned v = row[refl101(px + j, w) * c + ch];
      const unsigned wt = K == 5 ? (j == 0 ? 6u : (j == 1 || j == -1) ? 4u : 1u)
                                 : (j == 0 ? 2u : 1u);
      s += wt * v;
    }
    out[x] = (uint16_t)s;
  }
}

static void vpass5(const uint16_t* restrict a, const uint16_t* restrict b,
                   const uint16_t* restrict m, const uint16_t* restrict d,
                   const uint16_t* restrict e, uint8_t* restrict out, int n) {
  for (int x = 0; x < n; ++x)
    out[x] = (uint8_t)((uint16_t)(a[x] + e[x] + 4 * (b[x] + d[x]) + 6 * m[x] + 128) >> 8);
}

static void vpass3(const uint16_t* restrict a, const uint16_t* restrict m,
                   const uint16_t* restrict e, uint8_t* restrict out, int n) {
  for (int x = 0; x < n; ++x) out[x] = (uint8_t)((uint16_t)(a[x] + e[x] + 2 * m[x] + 8) >> 4);
}

void baseline_gaussian_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                          int64_t rs, int K) {
  const int R = K / 2;
  const int strips = (h + 31) / 32;
  const int nrow = w * c;
#pragma omp parallel
  {
    uint16_t* ring = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)nrow * 5);
    int ring_y[5];
#pragma omp for schedule(static)
    for (int64_t job = 0; job < (int64_t)n * strips; ++job) {
      const int img = (int)(job / strips), st = (int)(job % strips);
      const uint8_t* s = src + (int64_t)img * h * rs;
      uint8_t* d = dst + (int64_t)img * h * rs;
      for (int k = 0; k < 5; ++k) ring_y[k] = -1 << 30;
      const int y0 = st * 32, y1 = y0 + 32 < h ? y0 + 32 : h;
      for (int y = y0; y < y1; ++y) {
        const uint16_t* rows[5];
        for (int i = -R; i <= R; ++i) {
          const int yy = refl101(y + i, h);
          const int slot = ((yy % 5) + 5) % 5;
          if (ring_y[slot] != yy) {
            hpass(s + (int64_t)yy * rs, ring + (size_t)slot * nrow, w, c, K);
            ring_y[slot] = yy;
          }
          rows[i + R] = ring + (size_t)slot * nrow;
        }
        if (K == 5)
          vpass5(rows[0], rows[1], rows[2], rows[3], rows[4], d + (int64_t)y * rs, nrow);
        else
          vpass3(rows[0], rows[1], rows[2], d + (int64_t)y * rs, nrow);
      }
    }
    free(ring);
  }
}
