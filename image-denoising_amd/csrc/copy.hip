// Flat device copy: the copy ceiling the bench line reports beside the stencil (SURVEY §8d asks
// for "a measured copy-kernel peak" next to the roofline fraction).  Not on the reference path:
// the nearest reference operation is the numpy array copy cv2.resize makes at scale 1.0
// (lib/utils/blob.py:44-45).
//
// One 256-thread workgroup moves one contiguous 32 KB chunk: all 8 16-byte loads per lane are in
// flight before the first store (the burst pattern of the stencil's tile fetch).  The chunk's
// buffer descriptor range-checks the tail, so any byte count is accepted.
//   policy 0: default cache policy on loads and stores
//   policy 1: nontemporal loads and stores (aux = 2): the fastest copy measured on MI355X
//             (6.27 TB/s vs 5.5-5.7 default, profiles/r01b/copyceil.txt)
#include "idn_common.hpp"

namespace idn {

constexpr int COPY_NL = 8;
constexpr uint32_t COPY_CHUNK = COPY_NL * 256u * 16u;  // 32 KB

template <int AUX>
__global__ __launch_bounds__(256) void copy_burst_kernel(const uint8_t* __restrict__ src,
                                                         uint8_t* __restrict__ dst, int64_t nbytes) {
  const int64_t base = (int64_t)blockIdx.x * COPY_CHUNK;
  const int64_t left = nbytes - base;
  const uint32_t range = left < (int64_t)COPY_CHUNK ? (uint32_t)left : COPY_CHUNK;
  const rsrc_t rs = make_rsrc(src + base, range);
  const rsrc_t rd = make_rsrc(dst + base, range);
  v4u v[COPY_NL];
#pragma unroll
  for (int i = 0; i < COPY_NL; ++i)
    v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, 16u * (256u * i + threadIdx.x), 0, AUX);
#pragma unroll
  for (int i = 0; i < COPY_NL; ++i)
    __builtin_amdgcn_raw_buffer_store_b128(v[i], rd, 16u * (256u * i + threadIdx.x), 0, AUX);
}

}  // namespace idn

extern "C" int idn_copy_u8(const uint8_t* src, uint8_t* dst, int64_t nbytes, int policy,
                           void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(src && dst, "idn_copy_u8: null pointer");
  IDN_CHECK_ARG(nbytes >= 0, "idn_copy_u8: negative size");
  IDN_CHECK_ARG(policy == 0 || policy == 1, "idn_copy_u8: policy must be 0 or 1");
  IDN_CHECK_ARG(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0,
                "idn_copy_u8: pointers must be 16-byte aligned");
  IDN_CHECK_ARG(nbytes % 16 == 0, "idn_copy_u8: size must be a multiple of 16");
  if (nbytes == 0) return IDN_OK;
  const int64_t blocks = (nbytes + COPY_CHUNK - 1) / COPY_CHUNK;
  IDN_CHECK_ARG(blocks < (int64_t)0x7FFFFFFF, "idn_copy_u8: size too large");
  if (policy == 1)
    hipLaunchKernelGGL((copy_burst_kernel<2>), dim3((unsigned)blocks), dim3(256), 0,
                       as_stream(stream), src, dst, nbytes);
  else
    hipLaunchKernelGGL((copy_burst_kernel<0>), dim3((unsigned)blocks), dim3(256), 0,
                       as_stream(stream), src, dst, nbytes);
  IDN_CHECK_LAUNCH("idn_copy_u8");
  return IDN_OK;
}
