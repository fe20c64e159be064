// Memory-ceiling microbenchmark for the stencil access pattern (tuning aid, not product code).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/membench tools/membench.hip && /tmp/membench
// Prints GB/s (read + write bytes / time) for:
//   copy16      flat grid-stride dwordx4 copy, 16-B aligned
//   copy16_off8 the same with src/dst shifted by 8 bytes
//   stripe      the wave-stripe pattern of stencil_u8_fast (segments of 1000 B, lanes at -8,
//               PF rows in flight, bands) doing an identity copy: the structure's own ceiling
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void copy16(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    d[i] = s[i];
}

__global__ __launch_bounds__(256) void copy16_unroll(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    v4u a = s[i], b = s[i + stride], c = s[i + 2 * stride], e = s[i + 3 * stride];
    d[i] = a; d[i + stride] = b; d[i + 2 * stride] = c; d[i + 3 * stride] = e;
  }
  for (; i < n; i += stride) d[i] = s[i];
}

template <int PF>
__global__ __launch_bounds__(256) void stripe(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                              int h, int rb, int nseg, int seg_len, int bands,
                                              int band_rows, int total, int order) {
  const int lane = threadIdx.x & 63;
  const int item = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (item >= total) return;
  const int seg = item % nseg, t = item / nseg;
  const int nimg = total / (nseg * bands);
  const int band = order ? t / nimg : t % bands, img = order ? t % nimg : t / bands;
  const uint32_t ib = (uint32_t)h * rb;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(src + (size_t)img * ib), 0, ib, 0x00020000);
  __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(dst + (size_t)img * ib), 0, ib, 0x00020000);
  const int q = seg * seg_len - 8 + 16 * lane;
  const uint32_t off = q < 0 ? 0u : (uint32_t)q;
  const int y0 = band * band_rows, y1 = min(y0 + band_rows, h);
  v4u Lq[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) Lq[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)min(y0 + i, h - 1) * rb + off, 0, 0);
  const bool st = lane > 0 && lane < 63;
  for (int y = y0; y < y1; y += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      v4u v = Lq[u];
      Lq[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)min(y + u + PF, h - 1) * rb + off, 0, 0);
      if (y + u < y1 && st) __builtin_amdgcn_raw_buffer_store_b128(v, rd, (uint32_t)(y + u) * rb + off, 0, 0);
    }
  }
}

// one workgroup of NT threads covers whole rows (thread t: bytes [16t, 16t+16) of the row)
template <int PF, int NT>
__global__ __launch_bounds__(NT) void rowwg(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                            int h, int rb, int bands, int band_rows, int total) {
  const int item = blockIdx.x;
  if (item >= total) return;
  const int band = item % bands, img = item / bands;
  const uint32_t ib = (uint32_t)h * rb;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(src + (size_t)img * ib), 0, ib, 0x00020000);
  __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(dst + (size_t)img * ib), 0, ib, 0x00020000);
  const uint32_t off = 16u * threadIdx.x;
  const bool act = (int)off < rb;
  const int y0 = band * band_rows, y1 = min(y0 + band_rows, h);
  v4u Lq[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) Lq[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)min(y0 + i, h - 1) * rb + off, 0, 0);
  for (int y = y0; y < y1; y += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      v4u v = Lq[u];
      Lq[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)min(y + u + PF, h - 1) * rb + off, 0, 0);
      if (y + u < y1 && act) __builtin_amdgcn_raw_buffer_store_b128(v, rd, (uint32_t)(y + u) * rb + off, 0, 0);
    }
  }
}

// one wave = one full row (3 contiguous 1 KB load/store instructions per row); a workgroup of 4
// waves = 4 consecutive bands of one image; HALO extra rows read per band (stencil halo);
// XCD=1 remaps blocks so that consecutive band groups run on the same XCD.
template <int PF, int HALO, int XCD>
__global__ __launch_bounds__(256) void rowwave(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                               int h, int rb, int bands, int band_rows, int total) {
  int blk = blockIdx.x;
  if (XCD) {
    const int nb = gridDim.x, q = nb / 8, r = nb % 8, x = blk % 8;
    blk = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + blk / 8;
  }
  const int item = __builtin_amdgcn_readfirstlane(blk * 4 + (threadIdx.x >> 6));
  if (item >= total) return;
  const int lane = threadIdx.x & 63;
  const int band = item % bands, img = item / bands;
  const uint32_t ib = (uint32_t)h * rb;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(src + (size_t)img * ib), 0, ib, 0x00020000);
  __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(dst + (size_t)img * ib), 0, ib, 0x00020000);
  const uint32_t off = 16u * lane;
  const int y0 = band * band_rows, y1 = min(y0 + band_rows, h);
  const int ya = max(y0 - HALO / 2, 0), yb = min(y1 + HALO / 2, h);
  v4u Lq[PF][3];
#pragma unroll
  for (int i = 0; i < PF; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      Lq[i][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)min(ya + i, h - 1) * rb + off + 1024 * j, 0, 0);
  v4u acc[3] = {};
  for (int y = ya; y < yb; y += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        v4u v = Lq[u][j];
        Lq[u][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)min(y + u + PF, h - 1) * rb + off + 1024 * j, 0, 0);
        acc[j] ^= v;
        const int yy = y + u;
        if (yy >= y0 && yy < y1 && (int)(off + 1024 * j) < rb)
          __builtin_amdgcn_raw_buffer_store_b128(acc[j], rd, (uint32_t)yy * rb + off + 1024 * j, 0, 0);
      }
    }
  }
}

int main() {
  const int N = 256, H = 600, W = 1000, C = 3;
  const size_t bytes = (size_t)N * H * W * C;
  uint8_t *a, *b;
  hipMalloc(&a, bytes + 64);
  hipMalloc(&b, bytes + 64);
  hipMemset(a, 7, bytes + 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](const char* name, auto fn) {
    for (int i = 0; i < 3; ++i) fn();
    hipEventRecord(e0);
    const int it = 20;
    for (int i = 0; i < it; ++i) fn();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= it;
    printf("%-28s %8.4f ms  %8.1f GB/s\n", name, ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
  };
  const size_t n16 = bytes / 16;
  for (int grid : {2048, 4096, 8192, 16384}) {
    char nm[64];
    snprintf(nm, 64, "copy16 grid=%d", grid);
    timeit(nm, [&] { copy16<<<grid, 256>>>((const v4u*)a, (v4u*)b, n16); });
    snprintf(nm, 64, "copy16_unroll grid=%d", grid);
    timeit(nm, [&] { copy16_unroll<<<grid, 256>>>((const v4u*)a, (v4u*)b, n16); });
    snprintf(nm, 64, "copy16_off8 grid=%d", grid);
    timeit(nm, [&] { copy16<<<grid, 256>>>((const v4u*)(a + 8), (v4u*)(b + 8), n16 - 1); });
  }
  const int rb = W * C;
  for (int br : {4, 8, 16, 32}) {
    const int bands = (H + br - 1) / br;
    const int total = N * bands;
    const int nb = (total + 3) / 4;
    char nm[64];
    snprintf(nm, 64, "rowwave PF2 H0 band=%d", br);
    timeit(nm, [&] { rowwave<2, 0, 0><<<nb, 256>>>(a, b, H, rb, bands, br, total); });
    snprintf(nm, 64, "rowwave PF2 H4 band=%d", br);
    timeit(nm, [&] { rowwave<2, 4, 0><<<nb, 256>>>(a, b, H, rb, bands, br, total); });
    snprintf(nm, 64, "rowwave PF2 H4 xcd band=%d", br);
    timeit(nm, [&] { rowwave<2, 4, 1><<<nb, 256>>>(a, b, H, rb, bands, br, total); });
    snprintf(nm, 64, "rowwave PF4 H4 xcd band=%d", br);
    timeit(nm, [&] { rowwave<4, 4, 1><<<nb, 256>>>(a, b, H, rb, bands, br, total); });
    snprintf(nm, 64, "rowwave PF1 H4 xcd band=%d", br);
    timeit(nm, [&] { rowwave<1, 4, 1><<<nb, 256>>>(a, b, H, rb, bands, br, total); });
  }
  return 0;
}
