// Table-driven fp64 pieces of the float64 noise stream's Box-Muller (noise.hip normal2_f64).  The
// stream draws 53-bit integers a, b per pair: u1 = (a + 1) 2^-53 in (0, 1], u2 = b 2^-53 in [0, 1),
// z0 = sqrt(-2 ln u1) cos(2 pi u2), z1 = sqrt(-2 ln u1) sin(2 pi u2).  The library log /
// sincospi took ~130 fp64 operations per pair (the kernel was fp64-issue-bound); with the
// integers in hand both reduce exactly and need short polynomials only:
//   ln u1   = e ln2 + ln c_k + log1p(r), x = a + 1 = 2^e m, m in [1, 2), k = the top 7 fraction
//             bits of m, r = m / c_k - 1 formed as fma(m, 1/c_k, -1) with the tabled reciprocal
//             (|r| < 2^-7.5), log1p by its series to r^8, ln c_k tabled as a double-double
//   2 pi u2 = 2 pi k / 256 + d, k = b >> 45, d = (b mod 2^45) 2pi 2^-53 in [0, 2pi / 256): the
//             tabled (sin, cos) of the sector and the series of sin d, cos d - 1 (to d^9 / d^10),
//             combined as sin K + (sin K (cos d - 1) + cos K sin d) (and cos alike)
// Both within ~2 ulp of the correctly rounded values (tools/check_f64_math.cpp measures it over
// 10^7 draws against long double); only u1 within a few ulp of 1 loses relative precision in
// ln u1 (absolute error < 1e-19 there).  Tables: 128 (reciprocal, ln hi, ln lo), 256 (sin, cos).
#pragma once

#include <math.h>
#include <stdint.h>

#ifndef __HIPCC__
#define IDN_F64M_FN inline
#define IDN_F64M_TAB static const
#else
#define IDN_F64M_FN __host__ __device__ __forceinline__
#define IDN_F64M_TAB __device__ __constant__
#endif

namespace idn {
namespace f64m {

#include "f64_math_tables.inc"  // LN_TAB[4 * 128], SC_TAB[2 * 256]
constexpr int LN_TAB_N = 4 * 128, SC_TAB_N = 2 * 256;

constexpr double LN2_HI = 0x1.62e42fefa3800p-1;  // 11 trailing zero bits: e * LN2_HI is exact
constexpr double LN2_LO = 0x1.ef35793c76730p-45;

// log1p(r) for |r| <= 2^-7.5: the series to r^8 (the next term < 2^-70)
IDN_F64M_FN double log1p_small(double r) {
  const double r2 = r * r;
  return fma(r2, fma(r, fma(r, fma(r, fma(r, fma(r, fma(r, -1.0 / 8, 1.0 / 7), -1.0 / 6), 1.0 / 5),
                                  -1.0 / 4), 1.0 / 3), -0.5), r);
}

// ln(x 2^-53) for an integer 1 <= x <= 2^53; lt = LN_TAB or a copy of it (the kernels stage the
// tables in LDS: per-lane gathers from global memory cost more than the fp64 work they save)
IDN_F64M_FN double ln_u53(uint64_t x, const double* lt) {
  if (x >= (1ull << 53) - (1ull << 45)) {
    // u1 within 2^-8 of 1: ln u1 = log1p(u1 - 1) with u1 - 1 exact (the table form's e ln2 +
    // ln c_k cancel to |ln u1| there, losing up to 16 bits)
    return log1p_small((double)((int64_t)x - (int64_t)(1ull << 53)) * 0x1p-53);
  }
  const int lz = __builtin_clzll(x);
  const int e = 63 - lz;                       // x = 2^e m
  const uint64_t mant = x << lz;               // m with its leading 1 at bit 63
  const int k = (int)((mant >> 56) & 0x7F);    // top 7 fraction bits
  // m as a double in [1, 2): exact (x has at most 53 significant bits)
  const double m = (double)(mant >> 11) * 0x1p-52;
  const double p = log1p_small(fma(m, lt[4 * k], -1.0));
  const double ee = (double)(e - 53);
  const double hi = fma(ee, LN2_HI, lt[4 * k + 1]);  // exact product, one rounding of the sum
  return hi + (fma(ee, LN2_LO, lt[4 * k + 2]) + p);
}

// (sin, cos) of 2 pi b 2^-53 for an integer 0 <= b < 2^53; st = SC_TAB or a copy of it
IDN_F64M_FN void sincos2pi_u53(uint64_t b, const double* st, double* s, double* c) {
  const int k = (int)(b >> 45);
  const double d = (double)(b & ((1ull << 45) - 1)) * 0x1.921fb54442d18p-51;  // 2 pi 2^-53
  const double d2 = d * d;
  // sin d = d + d^3 (-1/6 + d^2 (1/120 + d^2 (-1/5040 + d^2 / 362880)))
  const double sd = fma(d * d2, fma(d2, fma(d2, fma(d2, 1.0 / 362880, -1.0 / 5040), 1.0 / 120),
                                    -1.0 / 6), d);
  // cos d - 1 = d^2 (-1/2 + d^2 (1/24 + d^2 (-1/720 + d^2 (1/40320 - d^2 / 3628800))))
  const double cd = d2 * fma(d2, fma(d2, fma(d2, fma(d2, -1.0 / 3628800, 1.0 / 40320), -1.0 / 720),
                                     1.0 / 24), -0.5);
  const double sk = st[2 * k], ck = st[2 * k + 1];
  *s = sk + fma(sk, cd, ck * sd);
  *c = ck + fma(ck, cd, -(sk * sd));
}

}  // namespace f64m
}  // namespace idn
