// Shared device/host helpers for the idn HIP kernels (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <stdlib.h>

#include "../../include/idn.h"

namespace idn {

// ---- error plumbing (thread-local message, negative status) --------------------------------
int set_error(int status, const char* fmt, ...);
// shared argument validation of the u8 -> u8 filters (defined in stencil_u8.hip)
int check_filter_args(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                      int64_t row_stride, const char* name);
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

#define IDN_CHECK_ARG(cond, ...)                                         \
  do {                                                                   \
    if (!(cond)) return ::idn::set_error(IDN_EINVAL, __VA_ARGS__);       \
  } while (0)

#define IDN_CHECK_LAUNCH(name)                                                          \
  do {                                                                                  \
    hipError_t e_ = hipGetLastError();                                                  \
    if (e_ != hipSuccess)                                                               \
      return ::idn::set_error(IDN_EHIP, "%s: launch failed: %s", name, hipGetErrorString(e_)); \
  } while (0)

// ---- buffer resource descriptors (T8/T20): per-image range-checked loads -----------------
// Out-of-range loads return 0 and never fault, so border lanes may over-read safely.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef uint32_t v3u __attribute__((ext_vector_type(3)));

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  // readfirstlane the inputs so the compiler can prove the descriptor wave-uniform
  uint64_t p = reinterpret_cast<uint64_t>(base);
  uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p));
  uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p >> 32));
  uint32_t nb = __builtin_amdgcn_readfirstlane(bytes);
  void* q = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, 0, nb, 0x00020000);
}

// Tuning knobs (host).  The product library (idn/libidn_hip.so) is built without
// IDN_TUNING_BUILD: every knob is its compile-time default and the library reads no environment
// variable (tests/test_abi.py checks its undefined symbols).  The tools-only variant
// (idn/libidn_hip_tuning.so, idn._build.build(tuning=True)) reads them from the environment for
// A/B measurements and the cross-form tests, which load it explicitly (idn._lib.variant).
#ifdef IDN_TUNING_BUILD
inline int knob(const char* name, int dflt) {
  const char* v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}
#else
constexpr int knob(const char*, int dflt) { return dflt; }
#endif

// compute units of the current device (host; cached per device)
inline int cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    cached[dev] = cus;
  }
  return cached[dev];
}

// ---- small integer helpers ------------------------------------------------------------------
// OpenCV BORDER_REFLECT_101 index (cv::borderInterpolate; repeats for overshoot >= len)
__host__ __device__ __forceinline__ int reflect101(int i, int len) {
  if (len == 1) return 0;
  while (i < 0 || i >= len) {
    if (i < 0) i = -i;
    if (i >= len) i = 2 * len - 2 - i;
  }
  return i;
}
__host__ __device__ __forceinline__ int clampi(int i, int lo, int hi) {
  return i < lo ? lo : (i > hi ? hi : i);
}

// ---- Philox4x32-10 (Salmon et al., SC'11) --------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

// a ^ b ^ c: one v_bitop3_b32 (truth table 0x96) on gfx950
__host__ __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

__host__ __device__ __forceinline__ void philox_round(u32x4& c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  // one 32x32->64 product per word (v_mad_u64_u32 on the device instead of mul_hi + mul_lo)
  const uint64_t p0 = (uint64_t)M0 * c.x, p1 = (uint64_t)M1 * c.z;
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  c = u32x4{xor3(hi1, c.y, k0), lo1, xor3(hi0, c.w, k1), lo0};
}

// ROUNDS = 10 is Random123's default; Salmon et al. (SC'11, Table 2) report Philox4x32 with 7
// rounds already passing TestU01 BigCrush, and the Gaussian flat stream uses 7 (noise_apply.hpp)
template <int ROUNDS = 10>
__host__ __device__ __forceinline__ u32x4 philox4x32(u32x4 ctr, uint64_t key) {
  uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    philox_round(ctr, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return ctr;
}

// uniform double in (0, 1) from 53 random bits (never 0 -> safe for log)
__device__ __forceinline__ double u01_open(uint32_t a, uint32_t b) {
  uint64_t v = ((uint64_t)(a >> 5) << 26) | (b >> 6);  // 53 bits
  return ((double)v + 0.5) * (1.0 / 9007199254740992.0);
}
// uniform double in [0, 1) (numpy random_sample semantics)
__device__ __forceinline__ double u01_closed_open(uint32_t a, uint32_t b) {
  uint64_t v = ((uint64_t)(a >> 5) << 26) | (b >> 6);
  return (double)v * (1.0 / 9007199254740992.0);
}

// Workgroup renumbering for the 8 XCDs (dispatch places workgroup b on XCD b % 8): the returned
// ids of each XCD's workgroups form one contiguous run, so neighbouring work items (halo rows, the
// partial 128-byte lines at a strip's edges) run on the same XCD and meet in its L2
__device__ __forceinline__ int xcd_contiguous_block(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

}  // namespace idn
