// skimage rgb2ycbcr's fp64 dot products and the order-preserving u64 keys of their min / max
// (shared by the wavelet's colour range, wavelet.hip, and the float64 noise kernel that reduces
// that range while it writes the image, noise.hip).
#pragma once

#include "idn_common.hpp"

namespace idn {

// skimage rgb2ycbcr: arr @ ycbcr_from_rgb.T + [16, 128, 128].  numpy's matmul (OpenBLAS dgemm) rounds
// each dot product as an fma chain over k; reproduced exactly, because the set of exactly-zero finest
// detail coefficients (and so sigma) depends on the last bit of Y (oracle/filters.c, same chain).
__device__ __forceinline__ double dot3(double x0, double x1, double x2, double m0, double m1, double m2) {
  return __fma_rn(x2, m2, __fma_rn(x1, m1, __dmul_rn(x0, m0)));
}
__device__ __forceinline__ void ycc_dots(double x0, double x1, double x2, double (&d)[3]) {
  d[0] = dot3(x0, x1, x2, 65.481, 128.553, 24.966);
  d[1] = dot3(x0, x1, x2, -37.797, -74.203, 112.0);
  d[2] = dot3(x0, x1, x2, 112.0, -93.786, -18.214);
}
// ycbcr64's offsets, added once after a min / max reduction of the dot products: x -> round(x + k)
// is monotone, so the min / max of the rounded sums is the rounded sum of the dots' min / max
__device__ __forceinline__ double ycc_offset(int c) { return c == 0 ? 16.0 : 128.0; }

// fp64 min / max as order-preserving u64 keys (negative values flip all bits, positive ones the
// sign bit), so unsigned atomics order any doubles -- f64 inputs outside [0, 1] give negative Cb/Cr
__device__ __forceinline__ unsigned long long dkey(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double dkey_inv(unsigned long long k) {
  return __longlong_as_double((long long)((k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k));
}
__device__ __forceinline__ void atomicMinD(double* p, double v) {
  atomicMin(reinterpret_cast<unsigned long long*>(p), dkey(v));
}
__device__ __forceinline__ void atomicMaxD(double* p, double v) {
  atomicMax(reinterpret_cast<unsigned long long*>(p), dkey(v));
}

}  // namespace idn
