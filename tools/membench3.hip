// Tile-shape probe for the stencil (tuning aid, not product code): identity copies of a
// 256 x 600 x 3000-byte batch where each workgroup owns a band of T output rows and also reads H
// halo rows, loading everything up front ("burst") before storing.
//   rowburst   3 waves x 1000-byte row segments (the stencil's lane layout)
//   flatburst  256 threads sweep the band's bytes contiguously, 16 B per lane per instruction
//   chunk      plain 16 KB contiguous chunk copy (reference)
//   hipcc --offload-arch=gfx950 -O3 -o tools/membench3 tools/membench3.hip && tools/membench3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int H_ = 600, RB = 3000, N_ = 256;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, n, 0x00020000);
}

template <int T, int HALO, int AUX>
__global__ __launch_bounds__(192) void rowburst(const uint8_t* __restrict__ s, uint8_t* __restrict__ d,
                                                int bands) {
  const int b = blockIdx.x, img = b / bands, band = b % bands;
  const int lane = threadIdx.x & 63, seg = threadIdx.x >> 6;
  const uint32_t ib = (uint32_t)H_ * RB;
  auto rs = rsrc(s + (size_t)img * ib, ib);
  auto rd = rsrc(d + (size_t)img * ib, ib);
  const int col = seg * 1000 + 16 * lane;
  const bool act = 16 * lane < 1000;
  const int y0 = band * T;
  v4u v[T + HALO];
#pragma unroll
  for (int i = 0; i < T + HALO; ++i) {
    int y = y0 - HALO / 2 + i;
    y = y < 0 ? 0 : (y >= H_ ? H_ - 1 : y);
    v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(y * RB + col), 0, 0);
  }
  v4u acc = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < HALO / 2; ++i) acc ^= v[i] ^ v[T + HALO - 1 - i];
#pragma unroll
  for (int i = 0; i < T; ++i) {
    const int y = y0 + i;
    if (act && y < H_)
      __builtin_amdgcn_raw_buffer_store_b128(v[HALO / 2 + i] ^ (acc & 0u), rd, (uint32_t)(y * RB + col), 0, AUX);
  }
}

template <int T, int HALO, int AUX>
__global__ __launch_bounds__(256) void flatburst(const uint8_t* __restrict__ s, uint8_t* __restrict__ d,
                                                 int bands) {
  constexpr int NL = ((T + HALO) * RB + 4095) / 4096;
  const int b = blockIdx.x, img = b / bands, band = b % bands;
  const uint32_t ib = (uint32_t)H_ * RB;
  auto rs = rsrc(s + (size_t)img * ib, ib);
  auto rd = rsrc(d + (size_t)img * ib, ib);
  const int y0 = band * T;
  const int ys = y0 - HALO / 2 < 0 ? 0 : y0 - HALO / 2;
  const uint32_t base = (uint32_t)ys * RB;
  v4u v[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, base + 4096u * i + 16u * threadIdx.x, 0, 0);
  const uint32_t lo = (uint32_t)y0 * RB, hi = (uint32_t)(y0 + T < H_ ? y0 + T : H_) * RB;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const uint32_t o = base + 4096u * i + 16u * threadIdx.x;
    if (o >= lo && o + 16 <= hi) __builtin_amdgcn_raw_buffer_store_b128(v[i], rd, o, 0, AUX);
  }
}

// flat load of the band (+halo) into LDS, then 3 waves store their 1000-byte row segments
// (exact: lane 62 writes its low 8 bytes only) -- the LDS-staged stencil's traffic shape
template <int T, int HALO, int AUX, int WGT>
__global__ __launch_bounds__(256) void flat_lds_row(const uint8_t* __restrict__ s, uint8_t* __restrict__ d,
                                                    int bands) {
  constexpr int NB = (T + HALO) * RB;
  constexpr int NL = (NB + 16 * WGT - 1) / (16 * WGT);
  __shared__ __attribute__((aligned(16))) uint8_t tile[NL * 16 * WGT];
  const int b = blockIdx.x, img = b / bands, band = b % bands;
  const uint32_t ib = (uint32_t)H_ * RB;
  auto rs = rsrc(s + (size_t)img * ib, ib);
  auto rd = rsrc(d + (size_t)img * ib, ib);
  const int y0 = band * T;
  const int ys = y0 - HALO / 2 < 0 ? 0 : y0 - HALO / 2;
  const uint32_t base = (uint32_t)ys * RB;
  v4u v[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i)
    v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, base + 16u * (WGT * i + threadIdx.x), 0, 0);
#pragma unroll
  for (int i = 0; i < NL; ++i) *(v4u*)&tile[16 * (WGT * i + threadIdx.x)] = v[i];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave < 3) {
    const int col = wave * 1000 + 16 * lane;
    for (int r = 0; r < T; ++r) {
      const int y = y0 + r;
      if (y >= H_) break;
      const uint32_t t = (uint32_t)(y - ys) * RB + col;
      if (16 * lane + 16 <= 1000) {
        v4u x = *(const v4u*)&tile[t];
        __builtin_amdgcn_raw_buffer_store_b128(x, rd, (uint32_t)y * RB + col, 0, AUX);
      } else if (16 * lane < 1000) {
        typedef uint32_t v2 __attribute__((ext_vector_type(2)));
        v2 x = *(const v2*)&tile[t];
        __builtin_amdgcn_raw_buffer_store_b64(x, rd, (uint32_t)y * RB + col, 0, AUX);
      }
    }
  }
}

template <int AUX>
__global__ __launch_bounds__(256) void chunk(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, uint32_t per) {
  const size_t base = (size_t)blockIdx.x * per;
  auto rs = rsrc(s + base, per);
  auto rd = rsrc(d + base, per);
  v4u v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, 4096u * i + 16u * threadIdx.x, 0, 0);
#pragma unroll
  for (int i = 0; i < 4; ++i) __builtin_amdgcn_raw_buffer_store_b128(v[i], rd, 4096u * i + 16u * threadIdx.x, 0, AUX);
}

int main() {
  const size_t bytes = (size_t)N_ * H_ * RB;
  uint8_t *a, *b;
  hipMalloc(&a, bytes + 65536);
  hipMalloc(&b, bytes + 65536);
  hipMemset(a, 7, bytes + 65536);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](const char* name, auto fn) {
    for (int i = 0; i < 3; ++i) fn();
    float best = 1e9, tot = 0;
    for (int r = 0; r < 5; ++r) {
      hipEventRecord(e0);
      for (int i = 0; i < 10; ++i) fn();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      ms /= 10;
      tot += ms;
      best = ms < best ? ms : best;
    }
    printf("%-28s avg %7.4f ms  min %7.4f ms  %7.1f GB/s(avg)\n", name, tot / 5, best,
           2.0 * bytes / (tot / 5 * 1e-3) / 1e9);
    fflush(stdout);
  };
  timeit("chunk16K", [&] { chunk<0><<<bytes / 16384, 256>>>(a, b, 16384); });
  timeit("chunk16K nt", [&] { chunk<2><<<bytes / 16384, 256>>>(a, b, 16384); });
#define ROW(T, HL)                                                                        \
  {                                                                                       \
    const int bands = (H_ + T - 1) / T;                                                   \
    timeit("rowburst T" #T " H" #HL, [&] { rowburst<T, HL, 0><<<N_ * bands, 192>>>(a, b, bands); }); \
    timeit("rowburst T" #T " H" #HL " nt", [&] { rowburst<T, HL, 2><<<N_ * bands, 192>>>(a, b, bands); }); \
    timeit("flatburst T" #T " H" #HL, [&] { flatburst<T, HL, 0><<<N_ * bands, 256>>>(a, b, bands); }); \
    timeit("flatburst T" #T " H" #HL " nt", [&] { flatburst<T, HL, 2><<<N_ * bands, 256>>>(a, b, bands); }); \
    timeit("flat_lds_row T" #T " H" #HL, [&] { flat_lds_row<T, HL, 0, 256><<<N_ * bands, 256>>>(a, b, bands); }); \
    timeit("flat_lds_row T" #T " H" #HL " nt", [&] { flat_lds_row<T, HL, 2, 256><<<N_ * bands, 256>>>(a, b, bands); }); \
    timeit("flat_lds_row192 T" #T " H" #HL, [&] { flat_lds_row<T, HL, 0, 192><<<N_ * bands, 192>>>(a, b, bands); }); \
  }
  ROW(6, 4) ROW(11, 4) ROW(16, 4)
  return 0;
}
