// Copy-ceiling probe (tuning aid, not product code): what a u8->u8 pass over the bench's
// 256 x 600 x 3000-byte batch (460.8 MB read + 460.8 MB written) can reach on this chip, with
// the same back-to-back launch pattern as bench.py.
//   hipcc --offload-arch=gfx950 -O3 -o tools/copyceil tools/copyceil.hip && tools/copyceil
//   gstride<U,AUXL,AUXS>  grid-stride dwordx4 copy, U loads in flight per thread
//   burst<NL,AUXL,AUXS>   one 256-thread workgroup copies one contiguous NL*4 KB chunk, all loads
//                         issued before the first store (the stencil tile form's pattern)
//   read / write          read-only (xor-reduced) and write-only passes over one buffer
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>
#include <algorithm>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, n, 0x00020000);
}

template <int U, int AUXL, int AUXS>
__global__ __launch_bounds__(256) void gstride(const v4u* __restrict__ s, v4u* __restrict__ d,
                                               size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(&s[i + u * stride]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (AUXS) __builtin_nontemporal_store(v[u], &d[i + u * stride]);
      else d[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) d[i] = s[i];
}

// chunk = NL * 256 * 16 bytes per workgroup; buffer-addressed so the tail is range-checked
template <int NL, int AUXL, int AUXS>
__global__ __launch_bounds__(256) void burst(const uint8_t* __restrict__ s, uint8_t* __restrict__ d,
                                             uint32_t nbytes_img, int chunks_per_img) {
  const int img = blockIdx.x / chunks_per_img, ch = blockIdx.x % chunks_per_img;
  auto rs = rsrc(s + (size_t)img * nbytes_img, nbytes_img);
  auto rd = rsrc(d + (size_t)img * nbytes_img, nbytes_img);
  const uint32_t base = (uint32_t)ch * NL * 4096u;
  v4u v[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i)
    v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, base + 16u * (256u * i + threadIdx.x), 0, AUXL);
#pragma unroll
  for (int i = 0; i < NL; ++i)
    __builtin_amdgcn_raw_buffer_store_b128(v[i], rd, base + 16u * (256u * i + threadIdx.x), 0, AUXS);
}

__global__ __launch_bounds__(256) void readonly(const v4u* __restrict__ s, v4u* __restrict__ sink,
                                                size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  v4u acc = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) acc ^= s[i];
  if (acc.x == 0x12345678u) sink[0] = acc;
}
__global__ __launch_bounds__(256) void writeonly(v4u* __restrict__ d, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const v4u z = {1, 2, 3, 4};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) d[i] = z;
}

int main() {
  const size_t IMG = 600 * 3000, N = 256, bytes = IMG * N;
  uint8_t *a, *b;
  hipMalloc(&a, bytes + 4096);
  hipMalloc(&b, bytes + 4096);
  hipMemset(a, 7, bytes);
  hipMemset(b, 0, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](const char* name, double moved, auto fn) {
    for (int i = 0; i < 10; ++i) fn();
    hipDeviceSynchronize();
    std::vector<float> t;
    for (int i = 0; i < 60; ++i) {
      hipEventRecord(e0);
      fn();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      t.push_back(ms);
    }
    double avg = 0;
    for (float x : t) avg += x;
    avg /= t.size();
    std::sort(t.begin(), t.end());
    printf("%-34s avg %7.4f ms  med %7.4f  min %7.4f  -> %7.1f GB/s avg  %7.1f med\n", name, avg,
           t[t.size() / 2], t[0], moved / (avg * 1e-3) / 1e9, moved / (t[t.size() / 2] * 1e-3) / 1e9);
    fflush(stdout);
  };
  const size_t n16 = bytes / 16;
  char nm[96];
  for (int grid : {2048, 4096, 8192, 16384}) {
    snprintf(nm, sizeof nm, "gstride U4 grid=%d", grid);
    timeit(nm, 2.0 * bytes, [&] { gstride<4, 0, 0><<<grid, 256>>>((const v4u*)a, (v4u*)b, n16); });
    snprintf(nm, sizeof nm, "gstride U4 nt-store grid=%d", grid);
    timeit(nm, 2.0 * bytes, [&] { gstride<4, 0, 1><<<grid, 256>>>((const v4u*)a, (v4u*)b, n16); });
  }
  for (int grid : {4096, 8192}) {
    snprintf(nm, sizeof nm, "gstride U8 grid=%d", grid);
    timeit(nm, 2.0 * bytes, [&] { gstride<8, 0, 0><<<grid, 256>>>((const v4u*)a, (v4u*)b, n16); });
  }
  {
    // 1.8 MB per image: chunk sizes that divide it (or nearly; the tail is range-checked)
    const uint32_t ib = (uint32_t)IMG;
#define BURST(NLV, AL, AS)                                                                      \
  {                                                                                             \
    const int cpi = (int)((ib + NLV * 4096 - 1) / (NLV * 4096));                                \
    snprintf(nm, sizeof nm, "burst NL=%d aux=%d/%d", NLV, AL, AS);                               \
    timeit(nm, 2.0 * bytes, [&] { burst<NLV, AL, AS><<<(unsigned)(N * cpi), 256>>>(a, b, ib, cpi); }); \
  }
    BURST(4, 0, 0) BURST(6, 0, 0) BURST(8, 0, 0) BURST(12, 0, 0) BURST(16, 0, 0)
    BURST(8, 0, 2) BURST(8, 2, 0) BURST(8, 2, 2) BURST(8, 1, 0) BURST(8, 0, 1)
#undef BURST
  }
  for (int grid : {4096, 8192}) {
    snprintf(nm, sizeof nm, "read-only grid=%d", grid);
    timeit(nm, 1.0 * bytes, [&] { readonly<<<grid, 256>>>((const v4u*)a, (v4u*)b, n16); });
    snprintf(nm, sizeof nm, "write-only grid=%d", grid);
    timeit(nm, 1.0 * bytes, [&] { writeonly<<<grid, 256>>>((v4u*)b, n16); });
  }
  hipFree(a);
  hipFree(b);
  return 0;
}
