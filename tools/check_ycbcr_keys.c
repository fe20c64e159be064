/* Checks the integer keys wl_color_minmax (csrc/wavelet.hip) ranks u8 pixels by: for each of Y, Cb,
 * Cr, over all 2^24 (r, g, b) triples, a smaller key 1000 x (skimage's decimal coefficients . rgb)
 * always means a smaller fp64 value of the kernel's chain fma(b, c2, fma(g, c1, r * c0)) + offset on
 * x / 255, and counts the key ties whose fp64 values differ (the kernel evaluates those).
 *   gcc -O2 -ffp-contract=off tools/check_ycbcr_keys.c -lm && ./a.out      (prints bad=0 per channel) */
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <stdint.h>
typedef struct { int32_t k; double f; } E;
static int cmp(const void* a, const void* b) {
  const E* x = a; const E* y = b;
  if (x->k != y->k) return x->k < y->k ? -1 : 1;
  return x->f < y->f ? -1 : (x->f > y->f);
}
int main(void) {
  const double C[3][3] = {{65.481, 128.553, 24.966}, {-37.797, -74.203, 112.0}, {112.0, -93.786, -18.214}};
  const int32_t K[3][3] = {{65481, 128553, 24966}, {-37797, -74203, 112000}, {112000, -93786, -18214}};
  const double off[3] = {16.0, 128.0, 128.0};
  E* e = malloc(sizeof(E) << 24);
  for (int c = 0; c < 3; ++c) {
    size_t i = 0;
    for (int r = 0; r < 256; ++r) for (int g = 0; g < 256; ++g) for (int b = 0; b < 256; ++b) {
      const double x0 = (double)r * (1.0 / 255.0), x1 = (double)g * (1.0 / 255.0), x2 = (double)b * (1.0 / 255.0);
      const double f = fma(x2, C[c][2], fma(x1, C[c][1], x0 * C[c][0])) + off[c];
      e[i].k = K[c][0] * r + K[c][1] * g + K[c][2] * b; e[i].f = f; ++i;
    }
    qsort(e, i, sizeof(E), cmp);
    long bad = 0, ties = 0, tiediff = 0;
    double prevmax = -1e300; int32_t prevk = e[0].k - 1;
    for (size_t j = 0; j < i; ) {
      size_t j2 = j; double mn = e[j].f, mx = e[j].f;
      while (j2 < i && e[j2].k == e[j].k) { if (e[j2].f < mn) mn = e[j2].f; if (e[j2].f > mx) mx = e[j2].f; ++j2; }
      if (j2 - j > 1) { ties++; if (mn != mx) tiediff++; }
      if (!(mn > prevmax)) bad++;
      prevmax = mx; j = j2;
    }
    printf("c=%d keys ordered strictly: bad=%ld  tie groups=%ld  tie groups with different f=%ld\n", c, bad, ties, tiediff);
  }
  return 0;
}
