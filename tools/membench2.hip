// HBM copy-ceiling probe (tuning aid, not product code): which copy form sustains the most
// bandwidth on this MI355X for a 2 x 461 MB u8 batch (the bench workload's footprint).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/membench2 tools/membench2.hip && /tmp/membench2
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// grid-stride, U loads in flight per lane, optional nontemporal load/store
template <int U, int NTL, int NTS>
__global__ __launch_bounds__(256) void gs_copy(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NTL ? __builtin_nontemporal_load(&s[i + u * stride]) : s[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NTS) __builtin_nontemporal_store(v[u], &d[i + u * stride]);
      else d[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) d[i] = s[i];
}

// block-contiguous chunks: workgroup b copies [b*CH, (b+1)*CH) 16-B units, U per lane in flight
template <int U, int NTS>
__global__ __launch_bounds__(256) void chunk_copy(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n,
                                                  size_t chunk) {
  const size_t b0 = blockIdx.x * chunk, b1 = b0 + chunk < n ? b0 + chunk : n;
  for (size_t i = b0 + threadIdx.x; i < b1; i += U * 256) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * 256 < b1) v[u] = s[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * 256 < b1) {
        if (NTS) __builtin_nontemporal_store(v[u], &d[i + u * 256]);
        else d[i + u * 256] = v[u];
      }
  }
}

// buffer load/store with cache-policy aux bits on the store (0 = default, 1 = glc/sc0,
// 2 = slc/nt, 3 = both)
template <int U, int AUX>
__global__ __launch_bounds__(256) void buf_copy(const uint8_t* __restrict__ s, uint8_t* __restrict__ d,
                                                uint32_t bytes_per_block) {
  const size_t base = (size_t)blockIdx.x * bytes_per_block;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(s + base), 0, bytes_per_block, 0x00020000);
  __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(d + base), 0, bytes_per_block, 0x00020000);
  for (uint32_t o = threadIdx.x * 16; o < bytes_per_block; o += U * 4096) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, o + u * 4096, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, o + u * 4096, 0, AUX);
  }
}

__global__ __launch_bounds__(256) void read_only(const v4u* __restrict__ s, uint32_t* out, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    v4u v = s[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void write_only(v4u* __restrict__ d, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) d[i] = v4u{1, 2, 3, (uint32_t)i};
}

int main() {
  const size_t bytes = (size_t)256 * 600 * 1000 * 3;  // 460.8 MB
  uint8_t *a, *b;
  uint32_t* o;
  hipMalloc(&a, bytes + 4096);
  hipMalloc(&b, bytes + 4096);
  hipMalloc(&o, 64);
  hipMemset(a, 7, bytes + 4096);
  hipMemset(b, 0, bytes + 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](const char* name, double moved, auto fn) {
    for (int i = 0; i < 3; ++i) fn();
    hipEventRecord(e0);
    const int it = 20;
    for (int i = 0; i < it; ++i) fn();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= it;
    printf("%-36s %8.4f ms  %8.1f GB/s\n", name, ms, moved / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  const size_t n16 = bytes / 16;
  char nm[96];
  timeit("hipMemcpyDtoD", 2.0 * bytes, [&] { hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); });
  for (int grid : {1024, 2048, 4096, 8192, 16384, 32768}) {
    snprintf(nm, 96, "gs U1 grid=%d", grid);
    timeit(nm, 2.0 * bytes, [&] { gs_copy<1, 0, 0><<<grid, 256>>>((const v4u*)a, (v4u*)b, n16); });
    snprintf(nm, 96, "gs U4 grid=%d", grid);
    timeit(nm, 2.0 * bytes, [&] { gs_copy<4, 0, 0><<<grid, 256>>>((const v4u*)a, (v4u*)b, n16); });
    snprintf(nm, 96, "gs U4 ntstore grid=%d", grid);
    timeit(nm, 2.0 * bytes, [&] { gs_copy<4, 0, 1><<<grid, 256>>>((const v4u*)a, (v4u*)b, n16); });
    snprintf(nm, 96, "gs U4 ntload+store grid=%d", grid);
    timeit(nm, 2.0 * bytes, [&] { gs_copy<4, 1, 1><<<grid, 256>>>((const v4u*)a, (v4u*)b, n16); });
  }
  for (size_t chunk_kb : {16, 64, 256, 1024}) {
    const size_t chunk = chunk_kb * 1024 / 16;
    const int grid = (int)((n16 + chunk - 1) / chunk);
    snprintf(nm, 96, "chunk %zuKB U4", chunk_kb);
    timeit(nm, 2.0 * bytes, [&] { chunk_copy<4, 0><<<grid, 256>>>((const v4u*)a, (v4u*)b, n16, chunk); });
    snprintf(nm, 96, "chunk %zuKB U4 ntstore", chunk_kb);
    timeit(nm, 2.0 * bytes, [&] { chunk_copy<4, 1><<<grid, 256>>>((const v4u*)a, (v4u*)b, n16, chunk); });
    snprintf(nm, 96, "chunk %zuKB U8", chunk_kb);
    timeit(nm, 2.0 * bytes, [&] { chunk_copy<8, 0><<<grid, 256>>>((const v4u*)a, (v4u*)b, n16, chunk); });
  }
  for (uint32_t kb : {64, 256}) {
    const uint32_t bpb = kb * 1024;
    const int grid = (int)(bytes / bpb);
    snprintf(nm, 96, "buf %uKB U4 aux0", kb);
    timeit(nm, 2.0 * grid * (double)bpb, [&] { buf_copy<4, 0><<<grid, 256>>>(a, b, bpb); });
    snprintf(nm, 96, "buf %uKB U4 aux1", kb);
    timeit(nm, 2.0 * grid * (double)bpb, [&] { buf_copy<4, 1><<<grid, 256>>>(a, b, bpb); });
    snprintf(nm, 96, "buf %uKB U4 aux2", kb);
    timeit(nm, 2.0 * grid * (double)bpb, [&] { buf_copy<4, 2><<<grid, 256>>>(a, b, bpb); });
    snprintf(nm, 96, "buf %uKB U4 aux3", kb);
    timeit(nm, 2.0 * grid * (double)bpb, [&] { buf_copy<4, 3><<<grid, 256>>>(a, b, bpb); });
  }
  for (int grid : {4096, 16384}) {
    snprintf(nm, 96, "read_only grid=%d", grid);
    timeit(nm, 1.0 * bytes, [&] { read_only<<<grid, 256>>>((const v4u*)a, o, n16); });
    snprintf(nm, 96, "write_only grid=%d", grid);
    timeit(nm, 1.0 * bytes, [&] { write_only<<<grid, 256>>>((v4u*)b, n16); });
  }
  return 0;
}
