// Empirical check behind wavelet.hip haar_row4_c (verification aid, not product code): the
// Markstein-corrected quotient q1 = fma(fma(-q0, b, a), r, q0), q0 = a*r, r = 1/b equals the IEEE
// quotient a/b for every u8 triple's normalised YCbCr value over 24 channel ranges.
//   gcc -O2 -ffp-contract=off -o /tmp/check_div tools/check_div.c -lm && /tmp/check_div
#include <stdio.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
static double dot3(double x0, double x1, double x2, double m0, double m1, double m2) {
  return fma(x2, m2, fma(x1, m1, x0 * m0));
}
int main(void) {
  srand(7);
  long bad = 0, tot = 0;
  const double M[3][3] = {{65.481, 128.553, 24.966}, {-37.797, -74.203, 112.0}, {112.0, -93.786, -18.214}};
  const double add[3] = {16.0, 128.0, 128.0};
  for (int trial = 0; trial < 24; ++trial) {
    int c = trial % 3;
    // plausible channel min / max
    double mn = add[c] - 40 + (rand() % 4000) / 100.0, mx = mn + 20 + (rand() % 20000) / 100.0;
    if (trial % 4 == 0) { mn = 16.0; mx = 235.0; }
    const double b = mx - mn, r = 1.0 / b;
    for (int v0 = 0; v0 < 256; ++v0)
      for (int v1 = 0; v1 < 256; ++v1)
        for (int v2 = 0; v2 < 256; v2 += (trial < 6 ? 1 : 3)) {
          const double y = dot3(v0 * (1.0 / 255.0), v1 * (1.0 / 255.0), v2 * (1.0 / 255.0), M[c][0], M[c][1], M[c][2]) + add[c];
          const double a = y - mn;
          const double q = a / b;
          const double q0 = a * r;
          const double q1 = fma(fma(-q0, b, a), r, q0);
          tot++;
          if (q1 != q) { if (bad < 5) printf("mismatch a=%.17g b=%.17g q=%.17g q1=%.17g\n", a, b, q, q1); bad++; }
        }
  }
  printf("checked %ld, mismatches %ld\n", tot, bad);
  return bad != 0;
}
