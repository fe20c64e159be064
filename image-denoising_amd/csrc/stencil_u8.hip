// Separable 8-bit stencils on interleaved HxWxC images for gfx950:
//   cv2.GaussianBlur(u8, (3,3)|(5,5), 0)   and   cv2.blur(u8, (3,3)),  BORDER_REFLECT_101.
//
// Reference call sites: lib/model/test.py:224,241,1767; lib/roi_data_layer/minibatch.py:119,136,
// 1636-1643.  OpenCV 3.4.2 semantics restated in oracle/filters.c.
//
// Lane layout (shared with the median, stripe.hpp): a row of RB = W*C bytes is cut into
// segments of <= 1008 output bytes; a wave owns one segment, lane l the 16-byte chunk
// [seg_start - 8 + 16 l, +16).  The horizontal halo comes from the neighbouring lanes by DPP
// wave shifts, so each byte is fetched once per row; row/segment edges rebuild the reflected
// bytes in registers.
//
// Arithmetic (vertical first): each input row is split once into even/odd u16 lanes
// (x & 0x00FF00FF, v_perm), the K vertical taps run on the lane's own 16 bytes from a K-deep
// register ring (v_mad_u32_u24 for the 6x tap), then the horizontal taps run once per OUTPUT row
// on the vertical sums, whose 2C-byte halos arrive by DPP (v_pk_mad_u16 for the 6x tap).  The
// Gaussian weights and the +128 rounding bias are arranged so the cv2 result lands in the high
// byte of each u16 lane (one v_perm packs 4 bytes); the box mean uses (S*7280 + 33200) >> 16.
//
// Memory forms:
//   stencil_u8_lds  (default, compact rows <= 3024 B)  one 3-wave workgroup per band of NB rows:
//                   the band's NB + K - 1 input rows are fetched flat into LDS (16 B per lane,
//                   contiguous lanes, all loads in flight), then each wave walks its segment
//                   out of LDS.  ~5.7 TB/s on the 600x1000 batch (profiles/).
//   stencil_u8_vf   (strided rows) the same arithmetic loading each row segment from HBM
//   stencil_u8_generic  one thread per pixel for shapes the lane layout does not accept
#include "stripe.hpp"

#include <type_traits>

namespace idn {

// OP_IDENT5: tuning-build probe -- the pitched tile's data movement with the taps reduced to a copy
// of the centre byte
enum StencilOp { OP_GAUSS3 = 0, OP_GAUSS5 = 1, OP_BOX3 = 2, OP_IDENT5 = 3 };

template <int OP> struct Stencil;
template <> struct Stencil<OP_GAUSS3> { static constexpr int K = 3; };
template <> struct Stencil<OP_GAUSS5> { static constexpr int K = 5; };
template <> struct Stencil<OP_BOX3> { static constexpr int K = 3; };

// ---- vertical-first fast path --------------------------------------------------------------
// Halo rows of a band cost only their unpack (8 ops); the horizontal pass runs per output row.
// Borders: the lead lane's reflected bytes are rebuilt on the raw row (lead_fix) before the
// unpack; the tail reflections are rebuilt on the u16 vertical sums (reflection commutes with the
// separable sums).

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_mad16(uint32_t a, uint32_t k, uint32_t c) {
  const u16x2 r = __builtin_bit_cast(u16x2, a) * __builtin_bit_cast(u16x2, k) +
                  __builtin_bit_cast(u16x2, c);
  return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint32_t mad24(uint32_t a, uint32_t k, uint32_t c) {
  return __umul24(a, k) + c;
}

// vertical taps over ring rows r0..r(K-1) (oldest first); raw u16 lanes <= 255
template <int OP>
__device__ __forceinline__ uint32_t vtap(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3,
                                         uint32_t r4) {
  if constexpr (OP == OP_GAUSS5) {
    // [1 4 6 4 1] + 8 per lane (x16 horizontal weight = the +128 rounding bias): <= 4088
    const uint32_t t = ((r1 + r3) << 2) + 0x00080008u;
    return r0 + r4 + mad24(r2, 6u, t);
  } else if constexpr (OP == OP_GAUSS3) {
    return r0 + r2 + (r1 << 1);  // [1 2 1]: <= 1020
  } else {
    return r0 + r1 + r2;  // <= 765
  }
}

// horizontal taps at window byte P of the vertical sums, finished to the output byte:
// GAUSS: result in the high byte of each u16 lane; BOX: the rounded mean in byte 2 of each of
// two dwords (lo lane, hi lane)
template <int C, int OP>
__device__ __forceinline__ uint32_t htap(const VWin& V, int P) {
  if constexpr (OP == OP_GAUSS5) {
    const uint32_t t = (V.at(P - C) + V.at(P + C)) << 2;
    return V.at(P - 2 * C) + V.at(P + 2 * C) + pk_mad16(V.at(P), 0x00060006u, t);
  } else if constexpr (OP == OP_GAUSS3) {
    // 16 * [1 2 1] + 128: (16 S + 128) >> 8 == (S + 8) >> 4
    const uint32_t x = V.at(P - C) + V.at(P + C) + (V.at(P) << 1);
    return (x << 4) + 0x00800080u;
  } else {
    return V.at(P - C) + V.at(P) + V.at(P + C);  // <= 2295
  }
}

template <int OP>
__device__ __forceinline__ v4u finish(const uint32_t (&A)[8]) {
  uint32_t o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if constexpr (OP == OP_BOX3) {
      // round(S/9) == (S*455 + 2075) >> 12 == (S*7280 + 33200) >> 16 (byte 2), S <= 2295
      const uint32_t e = A[2 * k], od = A[2 * k + 1];
      const uint32_t el = mad24(e & 0xFFFFu, 7280u, 33200u), eh = mad24(e >> 16, 7280u, 33200u);
      const uint32_t ol = mad24(od & 0xFFFFu, 7280u, 33200u), oh = mad24(od >> 16, 7280u, 33200u);
      // bytes: (el.b2, ol.b2, eh.b2, oh.b2)
      const uint32_t lo = __builtin_amdgcn_perm(ol, el, 0x0C0C0602u);  // el.b2 | ol.b2 << 8
      const uint32_t hi = __builtin_amdgcn_perm(oh, eh, 0x06020C0Cu);  // eh.b2 << 16 | oh.b2 << 24
      o[k] = lo | hi;
    } else {
      o[k] = __builtin_amdgcn_perm(A[2 * k + 1], A[2 * k], 0x07030501u);
    }
  }
  v4u r = {o[0], o[1], o[2], o[3]};
  return r;
}

// NB > 0: burst form.  The band is exactly NB rows (the launcher sizes it so), all NB + 2R input
// rows are loaded up front (PF = NB + 2R) and the body is straight-line code.  NB == 0: long
// bands, a PF-deep load queue and a U-row unrolled loop (U a multiple of K and PF).
template <int C, int OP, int PF, int NT, int NB>
__global__ __launch_bounds__(256) void stencil_u8_vf(const uint8_t* __restrict__ src,
                                                     uint8_t* __restrict__ dst, int h, int rb,
                                                     uint32_t row_stride, int nseg, int seg_len,
                                                     int bands, int band_rows, int total_items,
                                                     int map) {
  constexpr int K = Stencil<OP>::K;
  constexpr int R = K / 2;
  constexpr int U = NB ? NB : (K == 5) ? 5 : 6;
  static_assert(NB ? PF == NB + 2 * R : (U % K == 0 && U % PF == 0), "queue / unroll shape");
  static_assert(R * C <= 8, "one-side halo must fit in two neighbour dwords");

  const int lane = threadIdx.x & 63;
  const int item = stripe_item(map, nseg);
  if (item >= total_items) return;
  const StripeGeom g = stripe_geom(item, lane, rb, nseg, seg_len, bands);

  const uint32_t img_bytes = (uint32_t)h * row_stride;
  const rsrc_t rs = make_rsrc(src + (size_t)g.img * img_bytes, img_bytes);
  const rsrc_t rd = make_rsrc(dst + (size_t)g.img * img_bytes, img_bytes);
  const uint32_t ld_off = g.lead ? 0u : (uint32_t)g.q;

  const int y0 = g.band * band_rows;
  const int y1 = min(y0 + band_rows, h);
  if (y0 >= y1) return;
  const int nin = (y1 - y0) + 2 * R;
  auto load_row = [&](int r) -> v4u {
    const int y = reflect101_1(y0 - R + min(r, nin - 1), h);
    return __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)y * row_stride + ld_off, 0,
                                                  (NT & 1) ? 2 : 0);
  };
  const StoreOffs so = store_offs(g);

  v4u Lq[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) Lq[i] = load_row(i);

  uint32_t Rg[K][8];  // ring of unpacked input rows; row r lives in slot r % K

  // input row r: take it from the queue, refill the queue, rebuild the lead lane, unpack
  auto take_row = [&](int r, int slot_q, int slot_k, bool refill) {
    v4u Lv = Lq[slot_q];
    if (refill) Lq[slot_q] = load_row(r + PF);
    if (g.lead) {  // chunk = row bytes -8..7: rebuild the reflected 8 bytes
      const uint32_t L[4] = {Lv.x, Lv.y, Lv.z, Lv.w};
      Lv = v4u{lead_fix<C, BORDER_REFLECT101>(L, -8), lead_fix<C, BORDER_REFLECT101>(L, -4),
               L[0], L[1]};
    }
    unpack_row(Lv, Rg[slot_k]);
  };
  // output row from the ring whose newest row sits in slot `nw`
  auto out_row = [&](int nw, uint32_t row_off) {
    uint32_t Vs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (K == 5) {
        Vs[j] = vtap<OP>(Rg[(nw + 1) % K][j], Rg[(nw + 2) % K][j], Rg[(nw + 3) % K][j],
                         Rg[(nw + 4) % K][j], Rg[nw][j]);
      } else {
        Vs[j] = vtap<OP>(Rg[(nw + 1) % K][j], Rg[(nw + 2) % K][j], Rg[nw][j], 0u, 0u);
      }
    }
    VWin V;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      V.SE[2 + j] = Vs[j];
      V.SO[2 + j] = Vs[4 + j];
    }
    if constexpr (R * C > 4) {  // halos: R*C bytes each side
      V.SE[0] = from_prev_lane(Vs[2]);
      V.SO[0] = from_prev_lane(Vs[6]);
      V.SE[7] = from_next_lane(Vs[1]);
      V.SO[7] = from_next_lane(Vs[5]);
    } else {
      V.SE[0] = V.SO[0] = V.SE[7] = V.SO[7] = 0u;
    }
    V.SE[1] = from_prev_lane(Vs[3]);
    V.SO[1] = from_prev_lane(Vs[7]);
    V.SE[6] = from_next_lane(Vs[0]);
    V.SO[6] = from_next_lane(Vs[4]);
    if (g.fix_t0) vwin_tail_fix<C>(V, 24);
    if (g.fix_t8) vwin_tail_fix<C>(V, 16);
    uint32_t A[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      A[2 * k] = htap<C, OP>(V, 4 * k + 8);
      A[2 * k + 1] = htap<C, OP>(V, 4 * k + 9);
    }
    stripe_store_nb<NT>(finish<OP>(A), rd, so, row_off);
  };

  // prologue: the 2R rows above the band only fill the ring
#pragma unroll
  for (int r = 0; r < 2 * R; ++r) take_row(r, r % PF, r % K, !NB);

  if constexpr (NB) {
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int r = 2 * R + u;
      take_row(r, r % PF, r % K, false);
      const int y = y0 + u;
      out_row(r % K, y < y1 ? (uint32_t)y * row_stride : OOB_OFF);
    }
  } else {
    const int nout = y1 - y0;
    const int ngroups = (nout + U - 1) / U;
    for (int gi = 0; gi < ngroups; ++gi) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = 2 * R + gi * U + u;  // slots (2R + u) % K / % PF are static
        take_row(r, (2 * R + u) % PF, (2 * R + u) % K, true);
        const int y = y0 + gi * U + u;
        out_row((2 * R + u) % K, y < y1 ? (uint32_t)y * row_stride : OOB_OFF);
      }
    }
  }
}

// ---- shared per-row body of the LDS forms ------------------------------------------------------
// One output row from the register ring of K unpacked input rows whose newest row sits in slot
// `nw`: vertical taps, DPP halos, tail reflections, horizontal taps, pack, store.
template <int C, int OP>
__device__ __forceinline__ v4u ring_row(const uint32_t (&Rg)[Stencil<OP>::K][8], int nw,
                                        const StripeGeom& g) {
  constexpr int K = Stencil<OP>::K;
  constexpr int R = K / 2;
  uint32_t Vs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if constexpr (K == 5) {
      Vs[j] = vtap<OP>(Rg[(nw + 1) % K][j], Rg[(nw + 2) % K][j], Rg[(nw + 3) % K][j],
                       Rg[(nw + 4) % K][j], Rg[nw][j]);
    } else {
      Vs[j] = vtap<OP>(Rg[(nw + 1) % K][j], Rg[(nw + 2) % K][j], Rg[nw][j], 0u, 0u);
    }
  }
  VWin V;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    V.SE[2 + j] = Vs[j];
    V.SO[2 + j] = Vs[4 + j];
  }
  if constexpr (R * C > 4) {
    V.SE[0] = from_prev_lane(Vs[2]);
    V.SO[0] = from_prev_lane(Vs[6]);
    V.SE[7] = from_next_lane(Vs[1]);
    V.SO[7] = from_next_lane(Vs[5]);
  } else {
    V.SE[0] = V.SO[0] = V.SE[7] = V.SO[7] = 0u;
  }
  V.SE[1] = from_prev_lane(Vs[3]);
  V.SO[1] = from_prev_lane(Vs[7]);
  V.SE[6] = from_next_lane(Vs[0]);
  V.SO[6] = from_next_lane(Vs[4]);
  if (g.tail) {  // scalar branch: the other segments' waves skip the masked tail fix-ups
    if (g.fix_t0) vwin_tail_fix<C>(V, 24);
    if (g.fix_t8) vwin_tail_fix<C>(V, 16);
  }
  uint32_t A[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    A[2 * k] = htap<C, OP>(V, 4 * k + 8);
    A[2 * k + 1] = htap<C, OP>(V, 4 * k + 9);
  }
  return finish<OP>(A);
}
template <int C, int OP, int NT>
__device__ __forceinline__ void ring_out_row(const uint32_t (&Rg)[Stencil<OP>::K][8], int nw,
                                             const StripeGeom& g, rsrc_t rd, const StoreOffs& so,
                                             uint32_t row_off) {
  stripe_store_nb<NT>(ring_row<C, OP>(Rg, nw, g), rd, so, row_off);
}

// the lane's 16-byte chunk of one row staged in LDS at byte `o`, lead lane rebuilt, unpacked
template <int C>
__device__ __forceinline__ void lds_take_row(const uint8_t* tile, uint32_t o, bool lead,
                                             uint32_t (&U)[8]) {
  const v2u a = *reinterpret_cast<const v2u*>(&tile[o]);
  const v2u b = *reinterpret_cast<const v2u*>(&tile[o + 8]);
  v4u Lv = v4u{a.x, a.y, b.x, b.y};
  if (lead) {
    const uint32_t L[4] = {Lv.x, Lv.y, Lv.z, Lv.w};
    Lv = v4u{lead_fix<C, BORDER_REFLECT101>(L, -8), lead_fix<C, BORDER_REFLECT101>(L, -4), L[0],
             L[1]};
  }
  unpack_row(Lv, U);
}

enum TileEpi { EPI_U8 = 0, EPI_BLOB = 1 };

// Blob epilogue (EPI_BLOB): blob = float32(float64(v) - PIXEL_MEANS[ch]) (lib/utils/blob.py:35-36:
// numpy's float64 subtract, then the float32 store) is a 3 x 256 table, held in LDS interleaved as
// lut[3 v + ch] (lanes reading the same byte value of different channels hit different banks).
// The filtered row segment is staged in LDS (one 16-byte write per lane) and re-read as dwords, so
// store k of a lane writes the four floats of row bytes seg_start + 256 k + 4 lane .. + 3: every
// 16-byte store instruction of a wave writes 1 KiB of contiguous blob (the last 960 B), with no
// partial-chunk stores.
constexpr int BLOB_LUT = 768;          // floats
constexpr int BLOB_STAGE = 3 * 1024;   // bytes: one 1 KiB row-segment stage per wave
template <int AUX = 0>
__device__ __forceinline__ void blob_row_store(const v4u& o, uint32_t* __restrict__ stage,
                                               const float* __restrict__ lut, int lane,
                                               const StripeGeom& g, const uint32_t (&c4)[3],
                                               rsrc_t rd, bool row_ok, uint32_t row_byte) {
  // WAR: the previous row's reads of this wave's stage are issued before this write
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  reinterpret_cast<v4u*>(stage)[lane] = o;  // stage byte 16 lane = row byte q
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = g.seg_start + 256 * k + 4 * lane;  // row byte of the store's first float
    const bool ok = row_ok && e < g.seg_end;         // seg_end - seg_start is a multiple of 8
    const uint32_t w = stage[min(2 + 64 * k + lane, 255)];
    float f[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t v = (w >> (8 * j)) & 0xFFu;
      f[j] = *reinterpret_cast<const float*>(reinterpret_cast<const uint8_t*>(lut) +
                                             (v * 12u + c4[(k + j) % 3]));
    }
    __builtin_amdgcn_raw_buffer_store_b128(
        v4u{__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]),
            __float_as_uint(f[3])},
        rd, ok ? 4u * (row_byte + (uint32_t)e) : OOB_OFF, 0, AUX);
  }
}

// ---- LDS-tiled form --------------------------------------------------------------------------
// One workgroup = one band of NB output rows of one image, nseg waves (<= 3: rows <= 3024 bytes).
// The band's NB + 2R input rows are contiguous in HBM (row_stride == row bytes), so the whole
// tile is fetched flat -- 16 B per lane, consecutive lanes on consecutive addresses, all loads in
// flight at once -- and staged in LDS; the waves then walk their row segments out of LDS with
// the vertical-first arithmetic above and store their output rows directly.  Measured on this
// chip the flat tile fetch sustains ~5.8 TB/s copy-equivalent where per-segment row loads stop
// near 5.2 (tools/membench3.hip).
#ifndef IDN_STENCIL_NB  // band height of the u8 stencils' LDS tile (A/B builds set it)
#define IDN_STENCIL_NB 6
#endif
constexpr int TILE_WGT = 192;     // 3 waves
constexpr int TILE_RBMAX = 3024;  // 3 segments of 1008 bytes
template <int NB, int K>
struct TileShape {
  static constexpr int ROWS = NB + K - 1;
  static constexpr int BYTES = ROWS * TILE_RBMAX + 16;           // + alignment shift
  static constexpr int NL = (BYTES + 16 * TILE_WGT - 1) / (16 * TILE_WGT);
  // exact footprint (the fetch never writes past the tile's bytes): one more resident
  // workgroup per CU for some band heights than a whole number of fetch rounds would allow
  static constexpr int LDS = (BYTES + 15) / 16 * 16;
};

template <int C, int OP, int NB, int EPI = EPI_U8, int NTS = 0, int DMA = 0>
__global__ __launch_bounds__(TILE_WGT) void stencil_u8_lds(const uint8_t* __restrict__ src,
                                                          uint8_t* __restrict__ dst, int h, int rb,
                                                          int nseg, int seg_len, int bands,
                                                          int total_items,
                                                          float* __restrict__ blob = nullptr,
                                                          double mb = 0.0, double mg = 0.0,
                                                          double mr = 0.0) {
  constexpr int K = Stencil<OP>::K;
  constexpr int R = K / 2;
  using TS = TileShape<NB, K>;
  constexpr int EXTRA = EPI == EPI_BLOB ? BLOB_LUT * 4 + BLOB_STAGE : 0;
  __shared__ __attribute__((aligned(16))) uint8_t smem[TS::LDS + EXTRA];
  uint8_t* const tile = smem;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-contiguous block order: a band's neighbours (which fetch its halo rows) run on the same
  // XCD, so the halo re-reads hit that XCD's L2
  const int blk = xcd_contiguous_block(blockIdx.x, gridDim.x);
  // waves beyond nseg (rows narrower than 3 segments) only help fetch the tile
  const int item = blk * nseg + min(wave, nseg - 1);
  const StripeGeom g = stripe_geom(item, lane, rb, nseg, seg_len, bands);
  const uint32_t img_bytes = (uint32_t)h * (uint32_t)rb;
  const rsrc_t rs = make_rsrc(src + (size_t)g.img * img_bytes, img_bytes);
  const rsrc_t rd = EPI != EPI_BLOB ? make_rsrc(dst + (size_t)g.img * img_bytes, img_bytes)
                                  : make_rsrc(blob + (size_t)g.img * img_bytes, 4u * img_bytes);

  const int y0 = g.band * NB;
  const int y1 = min(y0 + NB, h);
  const int ys = max(y0 - R, 0), ye = min(y1 + R, h);
  const uint32_t base = (uint32_t)ys * (uint32_t)rb;
  const uint32_t base_al = base & ~15u, shift = base - base_al;
  const uint32_t nbytes = (uint32_t)ye * (uint32_t)rb - base_al;
  if constexpr (EPI == EPI_BLOB) {  // the blob table (published by the tile's barrier)
    float* lut = reinterpret_cast<float*>(smem + TS::LDS);
    for (int i = threadIdx.x; i < BLOB_LUT; i += TILE_WGT) {
      const int v = i / 3, ch = i - 3 * v;
      lut[i] = (float)__dsub_rn((double)v, ch == 0 ? mb : ch == 1 ? mg : mr);
    }
  }

  // flat fetch of the tile into LDS (out-of-image lanes read 0 and are not written).  Full bands
  // (every chunk but the last round's inside the tile): one lane offset, the round in the scalar
  // offset, no per-load compare / select and no guarded LDS stores but the last round's (~30
  // fewer VALU per band: the filter runs at the power cap, so VALU is time)
  {
    v4u v[TS::NL];
    const bool full = __builtin_amdgcn_readfirstlane(
        (int)(nbytes >= (uint32_t)(16 * TILE_WGT * (TS::NL - 1))));
    if (DMA && full) {  // (full: every chunk but the last round's inside the tile)
      // LDS-DMA: global_load_lds_dwordx4 writes each wave's 1 KiB straight into the tile (the
      // destination is wave base + 16 lane, as the flat layout wants), no VGPR round trip and no
      // ds_write.  Every wave must see every other wave's rows after the barrier, so each wave
      // waits for its own DMA (vmcnt(0)) before it: the workgroup fence does not promise that
      // wait on gfx9 (LLVM emits it here today, s_waitcnt vmcnt(0) lgkmcnt(0) before s_barrier;
      // stated explicitly so it cannot silently go away)
      const uint8_t* gsrc = src + (size_t)g.img * img_bytes + base_al + 16u * threadIdx.x;
      const int wv64 = 64 * wave;
#pragma unroll
      for (int i = 0; i < TS::NL - 1; ++i)
        __builtin_amdgcn_global_load_lds(
            (const void*)(gsrc + 16 * TILE_WGT * i),
            (__attribute__((address_space(3))) void*)(tile + 16 * (TILE_WGT * i + wv64)), 16, 0, 0);
      const uint32_t o = 16u * (uint32_t)(TILE_WGT * (TS::NL - 1) + threadIdx.x);
      if (o < nbytes)
        __builtin_amdgcn_global_load_lds(
            (const void*)(gsrc + 16 * TILE_WGT * (TS::NL - 1)),
            (__attribute__((address_space(3))) void*)(tile + 16 * (TILE_WGT * (TS::NL - 1) + wv64)),
            16, 0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (full) {
      const uint32_t vo = base_al + 16u * threadIdx.x;
#pragma unroll
      for (int i = 0; i < TS::NL - 1; ++i)
        v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 16 * TILE_WGT * i, 0);
      const uint32_t o = 16u * (uint32_t)(TILE_WGT * (TS::NL - 1) + threadIdx.x);
      v[TS::NL - 1] = __builtin_amdgcn_raw_buffer_load_b128(rs, o < nbytes ? base_al + o : OOB_OFF,
                                                            0, 0);
#pragma unroll
      for (int i = 0; i < TS::NL - 1; ++i)
        *reinterpret_cast<v4u*>(&tile[16u * (uint32_t)(TILE_WGT * i + threadIdx.x)]) = v[i];
      if (o < nbytes) *reinterpret_cast<v4u*>(&tile[o]) = v[TS::NL - 1];
    } else {
#pragma unroll
      for (int i = 0; i < TS::NL; ++i) {
        const uint32_t o = 16u * (uint32_t)(TILE_WGT * i + threadIdx.x);
        v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, o < nbytes ? base_al + o : OOB_OFF, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < TS::NL; ++i) {
        const uint32_t o = 16u * (uint32_t)(TILE_WGT * i + threadIdx.x);
        if (o < nbytes) *reinterpret_cast<v4u*>(&tile[o]) = v[i];
      }
    }
  }
  __syncthreads();
  const bool active = !(wave >= nseg || item >= total_items || y0 >= y1);  // wave-uniform
  if (!active) return;

  const uint32_t ld_off = g.lead ? 0u : (uint32_t)g.q;
  const int nin = (y1 - y0) + 2 * R;
  const StoreOffs so = store_offs(g);
  uint32_t Rg[K][8];
  auto take_row = [&](int r) {
    const int y = reflect101_1(y0 - R + min(r, nin - 1), h);
    lds_take_row<C>(tile, (uint32_t)(y - ys) * (uint32_t)rb + shift + ld_off, g.lead, Rg[r % K]);
  };
  // blob: byte offsets into lut[3 v + ch] of the channels of this lane's store bytes
  // (row byte seg_start + 256 k + 4 lane + j has channel (c0 + k + j) % 3: 256 = 1 mod 3)
  uint32_t c4[3] = {0u, 0u, 0u};
  if constexpr (EPI == EPI_BLOB) {
    const int c0 = (g.seg_start + 4 * lane) % 3;
#pragma unroll
    for (int t = 0; t < 3; ++t) c4[t] = 4u * (uint32_t)((c0 + t) % 3);
  }
#pragma unroll
  for (int r = 0; r < 2 * R; ++r) take_row(r);
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const int r = 2 * R + u;
    take_row(r);
    const int y = y0 + u;
    const uint32_t row_off = y < y1 ? (uint32_t)y * (uint32_t)rb : OOB_OFF;
    if constexpr (EPI == EPI_BLOB) {
      blob_row_store(ring_row<C, OP>(Rg, r % K, g),
                     reinterpret_cast<uint32_t*>(smem + TS::LDS + BLOB_LUT * 4 + 1024 * wave),
                     reinterpret_cast<const float*>(smem + TS::LDS), lane, g, c4, rd, y < y1,
                     (uint32_t)y * (uint32_t)rb);
    } else {
      ring_out_row<C, OP, NTS ? 2 : 0>(Rg, r % K, g, rd, so, row_off);
    }
  }
}


// ---- pitched LDS tile (round 5) ----------------------------------------------------------------
// The band's NB + 2R input rows are fetched by LDS-DMA into tile rows of PT_PITCH = 3072 bytes, one
// fetch round (3 waves x 64 lanes x 16 B) per row: tile row j holds image row
// reflect101(y0 - R + j) -- the reflected rows of the first / last band are fetched like any other,
// so every band runs the same straight-line body -- and row byte x sits at tile byte 8 + x.  Lane
// l's 16-byte chunk [seg_start - 8 + 16 l, +16) then starts at tile byte seg_start + 16 l: with
// 1008-byte segments every chunk is one aligned, conflict-free ds_read_b128 at a compile-time
// offset (the flat tile's 3000-byte rows put every other row at 8 mod 16: two 8-byte reads, half
// of its LDS cycles bank conflicts).  The fetch lanes' global offsets are row * rb + 16 t - 8, so
// it takes rows of 16 k + 8 bytes (the 600x1000x3 batch: 3000 B); others keep the flat tile.
//
// Per output row the arithmetic runs on u16 lanes holding ADJACENT bytes (b, b+1) (the flat tile's
// (b, b+2) pairs need 8 DPP halo moves and 14 funnel shifts per row; adjacent pairs 6 and 11), and
// the border reflections are rebuilt on the vertical sums of the row's first and last lane only
// (wave-uniform branches): no per-input-row fix-up, no per-row address arithmetic.
//
// NTP: cache policy of the tile fetch -- 0 default, 1 nontemporal for the band's private rows
// [2R, NB) (no other band's tile reads them) and default for the shared halo rows, 2 nontemporal
// for every row, 3 nontemporal for rows [0, NB) (the leading halo: the band above read it
// first), 4 for rows [2R, NB + 2R) (the trailing halo).  NTS: nontemporal stores.
constexpr int PT_WGT = 192;
constexpr int PT_PITCH = 16 * PT_WGT;  // 3072
constexpr int PT_SEG = 1008;           // 63 output chunks per wave
constexpr int PT_RBMAX = 3 * PT_SEG;   // 3024
// The product's band height and cache policy (profiles/r05/stencil/): 9-row bands (13 tile rows,
// 39 KB: four workgroups per CU), nontemporal loads for the band's private rows and nontemporal
// stores -- 6.1-6.2 TB/s against 5.6 for 6-row bands at the default policy (which was the flat
// tile's best); nontemporal stores alone, nontemporal halo rows, sc1 stores, 8 / 10 / 12 / 16-row
// bands and two waves per segment all measured slower
#ifndef IDN_STENCIL_PT_NB  // band height of the pitched tile (A/B builds set it)
#define IDN_STENCIL_PT_NB 9
#endif
#ifndef IDN_STENCIL_PT_NTP  // the product's tile-fetch policy (see stencil_u8_pt)
#define IDN_STENCIL_PT_NTP 1
#endif
#ifndef IDN_STENCIL_PT_NTS  // the product's store policy
#define IDN_STENCIL_PT_NTS 1
#endif
// the fused blob epilogue's (12 B written per 3 B read): 6-row bands at the default policy,
// 5.61 TB/s against 5.56-5.57 for the flat tile; the nontemporal policies cost 3-8 % here
// (profiles/r05/stencil/r05g)
#ifndef IDN_STENCIL_PT_NB_BLOB
#define IDN_STENCIL_PT_NB_BLOB 6
#endif
#ifndef IDN_STENCIL_PT_NTP_BLOB
#define IDN_STENCIL_PT_NTP_BLOB 0
#endif
#ifndef IDN_STENCIL_PT_NTS_BLOB
#define IDN_STENCIL_PT_NTS_BLOB 0
#endif


// window of vertical sums as adjacent-byte u16 pairs: W[i] = window bytes (2i, 2i+1) (lo, hi lane);
// window byte 0 = chunk byte -8
struct PWin {
  uint32_t W[16];
  __device__ __forceinline__ uint32_t at(int b) const {  // window bytes (b, b+1) as a u16 pair
    return (b & 1) ? __builtin_amdgcn_alignbyte(W[(b + 1) >> 1], W[b >> 1], 2) : W[b >> 1];
  }
};

// byte s of the window's pair registers as (register, half)
__device__ __forceinline__ uint32_t pw_pair(const PWin& V, int slo, int shi) {
  if ((slo & 1) == 0 && shi == slo + 1) return V.W[slo >> 1];
  return pick16(V.W[slo >> 1], slo & 1, V.W[shi >> 1], shi & 1);
}

// source window byte of window byte w for BORDER_REFLECT_101 at the row start (row byte 0 = window
// byte 16, the row's first lane) or at the row end (row byte rb = window byte `base`)
template <int C>
__host__ __device__ constexpr int pw_lead_src(int w) {
  const int rho = w - 16;  // < 0
  const int pix = (rho - (C - 1)) / C;  // floor(rho / C)
  const int ch = rho - pix * C;
  return 16 + (-pix) * C + ch;
}
template <int C>
__host__ __device__ constexpr int pw_tail_src(int base, int w) {
  const int k = w - base;  // >= 0
  return base - 2 * C - (k / C) * C + (k % C);
}

// rebuild the window bytes [16 - HB, 16) (lead) of `V` from row bytes 0.. (only lane 0 of the
// row's first wave takes them)
template <int C, int HB>
__device__ __forceinline__ void pw_lead_fix(PWin& V, bool lane_is_lead) {
  constexpr int I0 = (16 - HB) >> 1;
  uint32_t nw[8 - I0];
#pragma unroll
  for (int i = I0; i < 8; ++i) {
    const int lo = 2 * i < 16 - HB ? 2 * i : pw_lead_src<C>(2 * i);
    nw[i - I0] = pw_pair(V, lo, pw_lead_src<C>(2 * i + 1));
  }
#pragma unroll
  for (int i = I0; i < 8; ++i) V.W[i] = lane_is_lead ? nw[i - I0] : V.W[i];
}
// rebuild window bytes [base, base + HB) past the row end (base = 16 or 24) on the lanes `fix`
template <int C, int HB>
__device__ __forceinline__ void pw_tail_fix(PWin& V, int base, bool fix) {
  const int i0 = base >> 1, i1 = (base + HB + 1) >> 1;  // registers [i0, i1)
  uint32_t nw[(HB + 1) / 2 + 1];
#pragma unroll
  for (int i = i0; i < i1; ++i) {
    const int hi = 2 * i + 1 < base + HB ? pw_tail_src<C>(base, 2 * i + 1) : 2 * i + 1;
    nw[i - i0] = pw_pair(V, pw_tail_src<C>(base, 2 * i), hi);
  }
#pragma unroll
  for (int i = i0; i < i1; ++i) V.W[i] = fix ? nw[i - i0] : V.W[i];
}

// horizontal taps of the output pair at window bytes (P, P+1); GAUSS / IDENT: the result in the
// high byte of each u16 lane (the +128 rounding bias rides in the vertical sums); BOX: the sum
template <int C, int OP>
__device__ __forceinline__ uint32_t ptap(const PWin& V, int P) {
  if constexpr (OP == OP_GAUSS5) {
    const uint32_t t = (V.at(P - C) + V.at(P + C)) << 2;
    return V.at(P - 2 * C) + V.at(P + 2 * C) + pk_mad16(V.at(P), 0x00060006u, t);
  } else if constexpr (OP == OP_GAUSS3) {
    const uint32_t x = V.at(P - C) + V.at(P + C) + (V.at(P) << 1);
    return (x << 4) + 0x00800080u;
  } else if constexpr (OP == OP_BOX3) {
    return V.at(P - C) + V.at(P) + V.at(P + C);  // <= 2295
  } else {
    return V.at(P);  // identity probe (tuning build): centre byte
  }
}

// 8 horizontal results (output pairs (2j, 2j+1) of the chunk) -> the 16 output bytes
template <int OP>
__device__ __forceinline__ v4u pfinish(const uint32_t (&A)[8]) {
  uint32_t o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if constexpr (OP == OP_BOX3) {
      // round(S/9) == (S*7280 + 33200) >> 16 (byte 2), S <= 2295; bytes 4k..4k+3 from the lanes
      // (A[2k].lo, A[2k].hi, A[2k+1].lo, A[2k+1].hi)
      const uint32_t a = A[2 * k], b = A[2 * k + 1];
      const uint32_t r0 = mad24(a & 0xFFFFu, 7280u, 33200u), r1 = mad24(a >> 16, 7280u, 33200u);
      const uint32_t r2 = mad24(b & 0xFFFFu, 7280u, 33200u), r3 = mad24(b >> 16, 7280u, 33200u);
      const uint32_t lo = __builtin_amdgcn_perm(r1, r0, 0x0C0C0602u);  // r0.b2 | r1.b2 << 8
      const uint32_t hi = __builtin_amdgcn_perm(r3, r2, 0x06020C0Cu);  // r2.b2 << 16 | r3.b2 << 24
      o[k] = lo | hi;
    } else {
      o[k] = __builtin_amdgcn_perm(A[2 * k + 1], A[2 * k], 0x07050301u);
    }
  }
  return v4u{o[0], o[1], o[2], o[3]};
}

// one input row chunk -> 8 adjacent-byte u16 pairs (chunk bytes 2j, 2j+1)
__device__ __forceinline__ void unpack_pairs(const v4u& x, uint32_t (&U)[8]) {
  const uint32_t d[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    U[2 * j] = __builtin_amdgcn_perm(0u, d[j], 0x0C010C00u);
    U[2 * j + 1] = __builtin_amdgcn_perm(0u, d[j], 0x0C030C02u);
  }
}

template <int OP> struct PStencil { static constexpr int K = Stencil<OP>::K; };
template <> struct PStencil<OP_IDENT5> { static constexpr int K = 5; };

// LEAD: the wave owns the row's first segment (lane 0 rebuilds the left reflection); TAIL: the
// row's last (lane `fix` rebuilds the right one: rows of 16 k + 8 bytes end at a chunk end)
template <int C, int OP, bool LEAD, bool TAIL>
__device__ __forceinline__ v4u pring_row(const uint32_t (&Rg)[PStencil<OP>::K][8], int nw,
                                         bool lane0, bool fix) {
  constexpr int K = PStencil<OP>::K;
  constexpr int R = K / 2;
  constexpr int HB = R * C;  // halo bytes per side
  uint32_t Vs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t r0 = Rg[(nw + 1) % K][j], r1 = Rg[(nw + 2) % K][j];
    if constexpr (OP == OP_GAUSS5) {
      Vs[j] = vtap<OP>(r0, r1, Rg[(nw + 3) % K][j], Rg[(nw + 4) % K][j], Rg[nw][j]);
    } else if constexpr (OP == OP_IDENT5) {
      Vs[j] = Rg[(nw + 3) % K][j] << 8;  // identity: the centre row
    } else {
      Vs[j] = vtap<OP>(r0, r1, Rg[nw][j], 0u, 0u);
    }
  }
  PWin V;
#pragma unroll
  for (int j = 0; j < 8; ++j) V.W[4 + j] = Vs[j];
  // halos: window bytes [8 - HB, 8) from the previous lane's chunk, [24, 24 + HB) from the next's
#pragma unroll
  for (int i = (8 - HB) >> 1; i < 4; ++i) V.W[i] = from_prev_lane(Vs[i + 4]);
#pragma unroll
  for (int i = 0; 2 * i < HB; ++i) V.W[12 + i] = from_next_lane(Vs[i]);
  if constexpr (LEAD) pw_lead_fix<C, HB>(V, lane0);
  if constexpr (TAIL) pw_tail_fix<C, HB>(V, 24, fix);
  uint32_t A[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) A[j] = ptap<C, OP>(V, 8 + 2 * j);
  return pfinish<OP>(A);
}

// the compute phase of one wave: the segment's chunk of each tile row, NB output rows
template <int C, int OP, int NB, int SAUX, bool LEAD, bool TAIL, int EPI = EPI_U8>
__device__ __forceinline__ void pt_body(const uint8_t* tile, rsrc_t rs, rsrc_t rd, int h, int rb,
                                        int seg_start, int y0, int lane, uint8_t* extra = nullptr) {
  constexpr int K = PStencil<OP>::K;
  constexpr int R = K / 2;
  const int seg_end = min(seg_start + PT_SEG, rb);
  const int q = seg_start - 8 + 16 * lane;  // the lane's chunk: row bytes [q, q + 16)
  const bool lane0 = lane == 0;
  const bool fix = q + 16 == rb;  // (TAIL) the row ends at this lane's chunk end
  // stores: lanes 1..62 16 B, lane 0 its chunk's high 8 B, lane 63 its low 8 B (nothing at or
  // past the row end); the row offset rides in the scalar offset
  const int o_lo = max(q, seg_start), o_hi = min(q + 16, seg_end);
  const int kind = (o_hi <= o_lo) ? 0 : (o_lo == q && o_hi == q + 16) ? 1 : (o_lo == q) ? 2 : 3;
  const uint32_t full = kind == 1 ? (uint32_t)q : OOB_OFF;
  const bool hi = kind == 3;
  const uint32_t half = kind == 2 ? (uint32_t)q : (kind == 3 ? (uint32_t)q + 8u : OOB_OFF);
  constexpr int aux = SAUX;

  // image row 0 (tile row R of the first band): the fetch slot of row bytes [-8, 8) lies partly
  // before the image and reads as zeros, so lane 0 takes row bytes 0..7 from a load of its own
  const bool first_band = LEAD && y0 == 0;  // wave-uniform
  v2u row0 = {0u, 0u};
  if (first_band) row0 = __builtin_amdgcn_raw_buffer_load_b64(rs, lane == 0 ? 0u : OOB_OFF, 0, 0);
  const uint8_t* rd_base = tile + seg_start + 16 * lane;
  uint32_t Rg[K][8];
  auto take = [&](int j) {
    v4u Lv = *reinterpret_cast<const v4u*>(rd_base + j * PT_PITCH);
    if (j == R && first_band) {
      Lv.z = lane == 0 ? row0.x : Lv.z;
      Lv.w = lane == 0 ? row0.y : Lv.w;
    }
    unpack_pairs(Lv, Rg[j % K]);
  };
#pragma unroll
  for (int j = 0; j < 2 * R; ++j) take(j);
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const int j = 2 * R + u;
    take(j);
    const v4u o = pring_row<C, OP, LEAD, TAIL>(Rg, j % K, lane0, fix);
    const int y = y0 + u;
    if constexpr (EPI == EPI_BLOB) {
      // the blob row through the wave's LDS stage (float stores of 1 KiB per wave-instruction)
      StripeGeom g;
      g.seg_start = seg_start;
      g.seg_end = seg_end;
      const int c0 = (seg_start + 4 * lane) % 3;
      uint32_t c4[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) c4[t] = 4u * (uint32_t)((c0 + t) % 3);
      const int wave = seg_start / PT_SEG;
      blob_row_store<aux>(o, reinterpret_cast<uint32_t*>(extra + BLOB_LUT * 4 + 1024 * wave),
                          reinterpret_cast<const float*>(extra), lane, g, c4, rd, y < h,
                          (uint32_t)y * (uint32_t)rb);
    } else if (y < h) {  // wave-uniform
      const uint32_t row_off = (uint32_t)y * (uint32_t)rb;
      __builtin_amdgcn_raw_buffer_store_b128(o, rd, full, row_off, aux);
      __builtin_amdgcn_raw_buffer_store_b64(hi ? v2u{o.z, o.w} : v2u{o.x, o.y}, rd, half, row_off,
                                            aux);
    }
  }
}

// LAUX / SAUX: the cache-policy bits of the selected tile rows' loads / of the stores (2 = nt;
// tuning builds try the sc bits too)
// EPI_BLOB: the fused blob epilogue (idn_gaussian_blob_f32): dst is the float32 blob, the
// 3 x 256 table of blob values is built from (mb, mg, mr) before the tile barrier
template <int C, int OP, int NB, int NTP, int SAUX, int LAUX = 2, int EPI = EPI_U8>
__global__ __launch_bounds__(PT_WGT) void stencil_u8_pt(const uint8_t* __restrict__ src,
                                                        uint8_t* __restrict__ dst, int h, int rb,
                                                        int nseg, int bands, double mb = 0.0,
                                                        double mg = 0.0, double mr = 0.0) {
  constexpr int K = PStencil<OP>::K;
  constexpr int R = K / 2;
  constexpr int ROWS = NB + 2 * R;
  constexpr int EXTRA = EPI == EPI_BLOB ? BLOB_LUT * 4 + BLOB_STAGE : 0;
  __shared__ __attribute__((aligned(16))) uint8_t tile[ROWS * PT_PITCH + EXTRA];
  uint8_t* const extra = tile + ROWS * PT_PITCH;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-contiguous block order: a band's neighbours (which fetch its halo rows) run on the same
  // XCD, so the halo re-reads hit that XCD's L2
  const int blk = xcd_contiguous_block(blockIdx.x, gridDim.x);
  const int img = blk / bands, band = blk - img * bands;
  const uint32_t img_bytes = (uint32_t)h * (uint32_t)rb;
  const rsrc_t rs = make_rsrc(src + (size_t)img * img_bytes, img_bytes);
  const int y0 = band * NB;

  // fetch: round j -> tile row j = image row reflect101(y0 - R + j) (rows past the band's last
  // needed row clamp to a valid row); lane slot t holds row bytes [16 t - 8, 16 t + 8): the
  // row's first slot reads the previous row's last 8 bytes with the row's first 8 (image row 0:
  // offset -8 wraps, the whole slot is out of range and reads zeros -- pt_body reloads its row
  // bytes 0..7), slots starting at or past the row end are not fetched
  {
    const int x = 16 * (int)threadIdx.x - 8;
    const uint32_t vx = x < rb ? (uint32_t)x : OOB_OFF;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      const int yy = reflect101_1(min(y0 - R + j, h - 1 + R), h);
      auto* lds = (__attribute__((address_space(3))) void*)(tile + j * PT_PITCH + 1024 * wave);
      const uint32_t vo = vx + (uint32_t)yy * (uint32_t)rb;
      if (NTP == 2 || (NTP == 1 && j >= 2 * R && j < NB) || (NTP == 3 && j < NB) ||
          (NTP == 4 && j >= 2 * R))  // folded after unrolling
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, lds, 16, vo, 0, 0, LAUX);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, lds, 16, vo, 0, 0, 0);
    }
    if constexpr (EPI == EPI_BLOB) {  // the blob table (published by the tile's barrier)
      float* lut = reinterpret_cast<float*>(extra);
      for (int i = threadIdx.x; i < BLOB_LUT; i += PT_WGT) {
        const int v = i / 3, ch = i - 3 * v;
        lut[i] = (float)__dsub_rn((double)v, ch == 0 ? mb : ch == 1 ? mg : mr);
      }
    }
    // every wave waits for its own DMA before the barrier (the workgroup fence does not promise
    // that wait for LDS-DMA on gfx9)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (wave >= nseg) return;  // rows narrower than 3 segments: the extra waves only fetched

  const int seg_start = wave * PT_SEG;
  const bool lead = wave == 0, tail = min(seg_start + PT_SEG, rb) == rb;
  const rsrc_t rd = EPI == EPI_BLOB
                        ? make_rsrc(reinterpret_cast<float*>(dst) + (size_t)img * img_bytes,
                                    4u * img_bytes)
                        : make_rsrc(dst + (size_t)img * img_bytes, img_bytes);
  if (lead && tail)
    pt_body<C, OP, NB, SAUX, true, true, EPI>(tile, rs, rd, h, rb, seg_start, y0, lane, extra);
  else if (lead)
    pt_body<C, OP, NB, SAUX, true, false, EPI>(tile, rs, rd, h, rb, seg_start, y0, lane, extra);
  else if (tail)
    pt_body<C, OP, NB, SAUX, false, true, EPI>(tile, rs, rd, h, rb, seg_start, y0, lane, extra);
  else
    pt_body<C, OP, NB, SAUX, false, false, EPI>(tile, rs, rd, h, rb, seg_start, y0, lane, extra);
}

// ---- generic path ------------------------------------------------------------------------
template <int OP>
__global__ __launch_bounds__(256) void stencil_u8_generic(const uint8_t* __restrict__ src,
                                                          uint8_t* __restrict__ dst, int n, int h,
                                                          int w, int c, int64_t row_stride) {
  constexpr int K = Stencil<OP>::K;
  constexpr int R = K / 2;
  const int64_t npix = (int64_t)n * h * w;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npix;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(p % w);
    const int64_t t = p / w;
    const int y = (int)(t % h);
    const int img = (int)(t / h);
    const uint8_t* s = src + (int64_t)img * h * row_stride;
    uint8_t* d = dst + (int64_t)img * h * row_stride + (int64_t)y * row_stride + (int64_t)x * c;
    for (int ch = 0; ch < c; ++ch) {
      uint32_t S = 0;
#pragma unroll
      for (int i = -R; i <= R; ++i) {
        const uint8_t* sr = s + (int64_t)reflect101(y + i, h) * row_stride;
#pragma unroll
        for (int j = -R; j <= R; ++j) {
          uint32_t v = sr[(int64_t)reflect101(x + j, w) * c + ch];
          uint32_t wgt;
          if constexpr (OP == OP_GAUSS5) {
            constexpr uint32_t a[5] = {1, 4, 6, 4, 1};
            wgt = a[i + R] * a[j + R];
          } else if constexpr (OP == OP_GAUSS3) {
            constexpr uint32_t a[3] = {1, 2, 1};
            wgt = a[i + R] * a[j + R];
          } else {
            wgt = 1;
          }
          S += wgt * v;
        }
      }
      uint32_t out;
      if constexpr (OP == OP_GAUSS5) out = (S + 128) >> 8;
      else if constexpr (OP == OP_GAUSS3) out = (S + 8) >> 4;
      else out = (2 * S + 9) / 18;
      d[ch] = (uint8_t)out;
    }
  }
}

// ---- float64 path (the reference's quirk branches filter the float64 output of random_noise) ----
// cv2.GaussianBlur / cv2.blur on CV_64F: separable double filter, BORDER_REFLECT_101, no rounding.
template <int OP>
__device__ __forceinline__ double f64_tap(int i) {
  if constexpr (OP == OP_GAUSS5) {
    constexpr double a[5] = {0.0625, 0.25, 0.375, 0.25, 0.0625};
    return a[i];
  } else if constexpr (OP == OP_GAUSS3) {
    constexpr double a[3] = {0.25, 0.5, 0.25};
    return a[i];
  } else {
    return 1.0;
  }
}

// Summation order follows OpenCV's 64F engines so results agree to the last ulp for the Gaussian:
// RowFilter<double> sums taps left to right; SymmColumnFilter<double> forms
// ky0*c + ky1*(r+1 + r-1) + ky2*(r+2 + r-2).  cv2.blur's 64F path uses running row/column sums
// (RowSum/ColumnSum), which this direct 3x3 sum matches only to a few ulp.
template <int OP>
__global__ __launch_bounds__(256) void stencil_f64(const double* __restrict__ src,
                                                   double* __restrict__ dst, int n, int h, int w,
                                                   int c) {
  constexpr int K = Stencil<OP>::K;
  constexpr int R = K / 2;
  const int64_t total = (int64_t)n * h * w * c;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int ch = (int)(e % c);
    int64_t t = e / c;
    const int x = (int)(t % w);
    t /= w;
    const int y = (int)(t % h);
    const int img = (int)(t / h);
    const double* s = src + (int64_t)img * h * w * c;
    double rs[K];
#pragma unroll
    for (int i = -R; i <= R; ++i) {
      const double* row = s + (int64_t)reflect101(y + i, h) * w * c;
      double racc = f64_tap<OP>(0) * row[(int64_t)reflect101(x - R, w) * c + ch];
#pragma unroll
      for (int j = -R + 1; j <= R; ++j)
        racc = __dadd_rn(racc, __dmul_rn(f64_tap<OP>(j + R), row[(int64_t)reflect101(x + j, w) * c + ch]));
      rs[i + R] = racc;
    }
    double acc;
    if constexpr (OP == OP_BOX3) {
      acc = __dadd_rn(__dadd_rn(rs[0], rs[1]), rs[2]) * (1.0 / 9.0);
    } else {
      acc = __dmul_rn(f64_tap<OP>(R), rs[R]);
#pragma unroll
      for (int k = 1; k <= R; ++k)
        acc = __dadd_rn(acc, __dmul_rn(f64_tap<OP>(R + k), __dadd_rn(rs[R + k], rs[R - k])));
    }
    dst[e] = acc;
  }
}

template <int OP>
static int launch_f64(const double* src, double* dst, int n, int h, int w, int c, hipStream_t st,
                      const char* name) {
  const int64_t total = (int64_t)n * h * w * c;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL((stencil_f64<OP>), dim3((unsigned)blocks), dim3(256), 0, st, src, dst, n, h, w, c);
  IDN_CHECK_LAUNCH(name);
  return IDN_OK;
}

// pitched-tile launch for the cache policy: ntp (which tile rows take the LAUX bits), the store
// bits (nts: 1 = nt) -- the product library's are compile-time; the tuning build also takes raw
// bit values IDN_STENCIL_SAUX / IDN_STENCIL_LAUX for a few combinations
template <int OP, int NB>
static int launch_pt(dim3 grid, hipStream_t st, const uint8_t* src, uint8_t* dst, int h, int rb,
                     int nseg, int bands, int ntp, int nts) {
  const dim3 block(PT_WGT);
#define IDN_PT(P, S, L) \
  hipLaunchKernelGGL((stencil_u8_pt<3, OP, NB, P, S, L>), grid, block, 0, st, src, dst, h, rb, \
                     nseg, bands)
#ifdef IDN_TUNING_BUILD
  const int saux = knob("IDN_STENCIL_SAUX", nts ? 2 : 0), laux = knob("IDN_STENCIL_LAUX", 2);
  if (ntp == 1 && saux == 2 && laux == 2) { IDN_PT(1, 2, 2); return IDN_OK; }
  if (ntp == 1 && saux == 16 && laux == 2) { IDN_PT(1, 16, 2); return IDN_OK; }
  if (ntp == 1 && saux == 18 && laux == 2) { IDN_PT(1, 18, 2); return IDN_OK; }
  if (ntp == 1 && saux == 17 && laux == 2) { IDN_PT(1, 17, 2); return IDN_OK; }
  if (ntp == 1 && saux == 2 && laux == 16) { IDN_PT(1, 2, 16); return IDN_OK; }
  if (ntp == 1 && saux == 2 && laux == 18) { IDN_PT(1, 2, 18); return IDN_OK; }
  if (ntp == 1 && saux == 0) { IDN_PT(1, 0, 2); return IDN_OK; }
  if (ntp == 4 && saux == 2) { IDN_PT(4, 2, 2); return IDN_OK; }
  if (ntp == 2 && saux == 2) { IDN_PT(2, 2, 2); return IDN_OK; }
  if (ntp == 0 && saux == 2) { IDN_PT(0, 2, 2); return IDN_OK; }
  if (ntp == 0 && saux == 0) { IDN_PT(0, 0, 2); return IDN_OK; }
  return set_error(IDN_EUNSUPPORTED, "tuning: no pitched-tile instance for NTP %d SAUX %d LAUX %d",
                   ntp, saux, laux);
#else
  (void)ntp;
  (void)nts;
  IDN_PT(IDN_STENCIL_PT_NTP, IDN_STENCIL_PT_NTS ? 2 : 0, 2);
  return IDN_OK;
#endif
#undef IDN_PT
}

// the fused blob form of the pitched tile (ntp / nts as launch_pt; the product's are compile-time)
template <int OP, int NB>
static int launch_pt_blob(dim3 grid, hipStream_t st, const uint8_t* src, float* blob, int h, int rb,
                          int nseg, int bands, int ntp, int nts, const double* mean) {
  const dim3 block(PT_WGT);
#define IDN_PTB(P, S) \
  hipLaunchKernelGGL((stencil_u8_pt<3, OP, NB, P, S, 2, EPI_BLOB>), grid, block, 0, st, src, \
                     reinterpret_cast<uint8_t*>(blob), h, rb, nseg, bands, mean[0], mean[1], mean[2])
#ifdef IDN_TUNING_BUILD
  if (ntp == 1 && nts) { IDN_PTB(1, 2); return IDN_OK; }
  if (ntp == 1) { IDN_PTB(1, 0); return IDN_OK; }
  if (ntp == 0 && nts) { IDN_PTB(0, 2); return IDN_OK; }
  if (ntp == 0) { IDN_PTB(0, 0); return IDN_OK; }
  return set_error(IDN_EUNSUPPORTED, "tuning: no blob pitched-tile instance for NTP %d NTS %d", ntp,
                   nts);
#else
  (void)ntp;
  (void)nts;
  IDN_PTB(IDN_STENCIL_PT_NTP_BLOB, IDN_STENCIL_PT_NTS_BLOB ? 2 : 0);
  return IDN_OK;
#endif
#undef IDN_PTB
}

// ---- host launchers --------------------------------------------------------------------------
// compact rows <= 3024 B: the LDS tile with 6-row bands (10 / 8 input rows in LDS, 30 / 24 KB per
// workgroup, up to 5-6 workgroups per CU; band heights 4-11 measured, tools/sweep_stencil.py);
// strided or wide rows: the stripe form from HBM; anything else the generic per-pixel kernel
template <int OP>
static int launch_stencil(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                          int64_t row_stride, hipStream_t st, const char* name) {
  constexpr int K = Stencil<OP>::K;
  constexpr int R = K / 2;
  const int64_t rb = (int64_t)w * c;
  const int form = knob("IDN_STENCIL_FORM", 1);
  if (form == 1 && stripe_ok(c, rb, row_stride, h, src, dst) && row_stride == rb &&
      rb <= PT_RBMAX && rb % 16 == 8 && h > 2 * R) {
    // pitched tile (rows of 16 k + 8 bytes, the 600x1000x3 batch)
    constexpr int NB = IDN_STENCIL_PT_NB;
    const int nseg = (int)((rb + PT_SEG - 1) / PT_SEG);
    const int bands = (h + NB - 1) / NB;
    const int64_t blocks = (int64_t)n * bands;
    IDN_CHECK_ARG(blocks < (int64_t)0x7FFFFFFF, "%s: batch too large", name);
    const dim3 grid((unsigned)blocks);
    const int ntp = knob("IDN_STENCIL_NTP", IDN_STENCIL_PT_NTP),
              nts = knob("IDN_STENCIL_NTS", IDN_STENCIL_PT_NTS);
    int rc;
    if (OP == OP_GAUSS5 && knob("IDN_STENCIL_IDENT", 0))  // tuning probe: data movement only
      rc = launch_pt<OP_IDENT5, NB>(grid, st, src, dst, h, (int)rb, nseg, bands, ntp, nts);
    else
      rc = launch_pt<OP, NB>(grid, st, src, dst, h, (int)rb, nseg, bands, ntp, nts);
    if (rc) return rc;
  } else if (stripe_ok(c, rb, row_stride, h, src, dst) && row_stride == rb && rb <= TILE_RBMAX &&
      h > 2 * R) {
    const int nseg = (int)((rb + 1007) / 1008);
    const int seg_len = (int)(((rb + nseg - 1) / nseg + 7) / 8 * 8);
    constexpr int NB = IDN_STENCIL_NB;
    const int bands = (h + NB - 1) / NB;
    const int64_t total = (int64_t)n * bands * nseg;
    IDN_CHECK_ARG(total < (int64_t)0x7FFFFFFF, "%s: batch too large", name);
    // nontemporal stores: a tuning-build A/B (IDN_STENCIL_NTS); the product keeps the default
    // tuning-build A/B: nontemporal stores (IDN_STENCIL_NTS, measured slower), register-staged
    // tile fetch (IDN_STENCIL_GLDS=0; the product fetches the tile by LDS-DMA)
    if (knob("IDN_STENCIL_NTS", 0))
      hipLaunchKernelGGL((stencil_u8_lds<3, OP, NB, EPI_U8, 1>), dim3((unsigned)((int64_t)n * bands)),
                         dim3(TILE_WGT), 0, st, src, dst, h, (int)rb, nseg, seg_len, bands,
                         (int)total);
    else if (knob("IDN_STENCIL_GLDS", 1))
      hipLaunchKernelGGL((stencil_u8_lds<3, OP, NB, EPI_U8, 0, 1>), dim3((unsigned)((int64_t)n * bands)),
                         dim3(TILE_WGT), 0, st, src, dst, h, (int)rb, nseg, seg_len, bands,
                         (int)total);
    else
      hipLaunchKernelGGL((stencil_u8_lds<3, OP, NB>), dim3((unsigned)((int64_t)n * bands)),
                         dim3(TILE_WGT), 0, st, src, dst, h, (int)rb, nseg, seg_len, bands,
                         (int)total);
  } else if (stripe_ok(c, rb, row_stride, h, src, dst)) {
    // strided or wide rows: stripe form.  Rows of <= 4 segments: short bands, one workgroup per
    // band, all band rows loaded up front; wider rows: long bands of independent waves.
    constexpr int PF = (K == 5) ? 5 : 6;
    constexpr int NBS = 6;
    const bool burst = (rb + 1007) / 1008 <= 4;
    const StripePlan p = plan_stripe(n, h, rb, K, burst ? 1 : PF, 5120, burst ? 1 : 0, NBS,
                                     burst ? NBS : 0);
    IDN_CHECK_ARG(p.total < (int64_t)0x7FFFFFFF, "%s: batch too large", name);
    const dim3 grid(p.grid), block(p.block);
    if (burst)
      hipLaunchKernelGGL((stencil_u8_vf<3, OP, NBS + K - 1, 0, NBS>), grid, block, 0, st, src, dst,
                         h, (int)rb, (uint32_t)row_stride, p.nseg, p.seg_len, p.bands, p.band_rows,
                         (int)p.total, p.map);
    else
      hipLaunchKernelGGL((stencil_u8_vf<3, OP, PF, 0, 0>), grid, block, 0, st, src, dst, h,
                         (int)rb, (uint32_t)row_stride, p.nseg, p.seg_len, p.bands, p.band_rows,
                         (int)p.total, p.map);
  } else {
    const int64_t npix = (int64_t)n * h * w;
    int64_t blocks = (npix + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL((stencil_u8_generic<OP>), dim3((unsigned)blocks), dim3(256), 0, st, src,
                       dst, n, h, w, c, row_stride);
  }
  IDN_CHECK_LAUNCH(name);
  return IDN_OK;
}

int check_filter_args(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                        int64_t row_stride, const char* name) {
  IDN_CHECK_ARG(src && dst, "%s: null pointer", name);
  IDN_CHECK_ARG(src != dst, "%s: in-place filtering is not supported (src == dst)", name);
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0, "%s: bad shape n=%d h=%d w=%d", name, n, h, w);
  IDN_CHECK_ARG(c >= 1 && c <= 4, "%s: channels must be 1..4 (got %d)", name, c);
  IDN_CHECK_ARG(row_stride >= (int64_t)w * c, "%s: row_stride %lld < w*c", name,
                (long long)row_stride);
  return IDN_OK;
}

}  // namespace idn

extern "C" int idn_gaussian_blur_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                                    int64_t row_stride, int ksize, void* stream) {
  using namespace idn;
  if (int e = check_filter_args(src, dst, n, h, w, c, row_stride, "idn_gaussian_blur_u8")) return e;
  if (n == 0) return IDN_OK;
  if (ksize == 3)
    return launch_stencil<OP_GAUSS3>(src, dst, n, h, w, c, row_stride, as_stream(stream),
                                     "idn_gaussian_blur_u8");
  if (ksize == 5)
    return launch_stencil<OP_GAUSS5>(src, dst, n, h, w, c, row_stride, as_stream(stream),
                                     "idn_gaussian_blur_u8");
  return set_error(IDN_EUNSUPPORTED, "idn_gaussian_blur_u8: ksize %d not supported (3 or 5)",
                   ksize);
}

extern "C" int idn_box_blur_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                               int64_t row_stride, int ksize, void* stream) {
  using namespace idn;
  if (int e = check_filter_args(src, dst, n, h, w, c, row_stride, "idn_box_blur_u8")) return e;
  if (n == 0) return IDN_OK;
  if (ksize == 3)
    return launch_stencil<OP_BOX3>(src, dst, n, h, w, c, row_stride, as_stream(stream),
                                   "idn_box_blur_u8");
  return set_error(IDN_EUNSUPPORTED, "idn_box_blur_u8: ksize %d not supported (3)", ksize);
}

extern "C" int idn_gaussian_blur_f64(const double* src, double* dst, int n, int h, int w, int c,
                                     int ksize, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(src && dst && src != dst, "idn_gaussian_blur_f64: bad pointers");
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0 && c >= 1 && c <= 4, "idn_gaussian_blur_f64: bad shape");
  if (n == 0) return IDN_OK;
  if (ksize == 3) return launch_f64<OP_GAUSS3>(src, dst, n, h, w, c, as_stream(stream), "idn_gaussian_blur_f64");
  if (ksize == 5) return launch_f64<OP_GAUSS5>(src, dst, n, h, w, c, as_stream(stream), "idn_gaussian_blur_f64");
  return set_error(IDN_EUNSUPPORTED, "idn_gaussian_blur_f64: ksize %d not supported", ksize);
}

extern "C" int idn_box_blur_f64(const double* src, double* dst, int n, int h, int w, int c,
                                int ksize, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(src && dst && src != dst, "idn_box_blur_f64: bad pointers");
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0 && c >= 1 && c <= 4, "idn_box_blur_f64: bad shape");
  if (n == 0) return IDN_OK;
  if (ksize == 3) return launch_f64<OP_BOX3>(src, dst, n, h, w, c, as_stream(stream), "idn_box_blur_f64");
  return set_error(IDN_EUNSUPPORTED, "idn_box_blur_f64: ksize %d not supported", ksize);
}

// ---- fused blob epilogue -----------------------------------------------------------------------
// cv2.GaussianBlur(u8, (k, k), 0) -> prep_im_for_blob at scale 1.0 (lib/utils/blob.py:33-47,
// lib/model/test.py:49-83): blob = float32(float64(filtered) - mean[ch]), dense (n, h, w, 3)
// float32, written by the filter kernel itself (the u8 filtered image never reaches HBM).
extern "C" int idn_gaussian_blob_f32(const uint8_t* src, float* blob, int n, int h, int w, int c,
                                     int64_t row_stride, int ksize, const double* mean,
                                     void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(blob && mean, "idn_gaussian_blob_f32: null pointer");
  if (int e = check_filter_args(src, (uint8_t*)blob, n, h, w, c, row_stride,
                                "idn_gaussian_blob_f32")) return e;
  if (n == 0) return IDN_OK;
  const int64_t rb = (int64_t)w * c;
  IDN_CHECK_ARG(ksize == 3 || ksize == 5, "idn_gaussian_blob_f32: ksize must be 3 or 5");
  if (!(stripe_ok(c, rb, row_stride, h, src, blob) && row_stride == rb && rb <= TILE_RBMAX &&
        h > ksize && ((uintptr_t)blob & 15) == 0))
    return set_error(IDN_EUNSUPPORTED, "idn_gaussian_blob_f32: layout not fused");
  hipStream_t st = as_stream(stream);
  if (knob("IDN_STENCIL_FORM", 1) == 1 && rb <= PT_RBMAX && rb % 16 == 8) {
    // the pitched tile (rows of 16 k + 8 bytes, the 600x1000x3 batch)
    constexpr int NB = IDN_STENCIL_PT_NB_BLOB;
    const int nsegp = (int)((rb + PT_SEG - 1) / PT_SEG);
    const int bands = (h + NB - 1) / NB;
    const int64_t blocks = (int64_t)n * bands;
    IDN_CHECK_ARG(blocks < (int64_t)0x7FFFFFFF, "idn_gaussian_blob_f32: batch too large");
    const int ntp = knob("IDN_STENCIL_NTP", IDN_STENCIL_PT_NTP_BLOB),
              nts = knob("IDN_STENCIL_NTS", IDN_STENCIL_PT_NTS_BLOB);
    const int rc = ksize == 5 ? launch_pt_blob<OP_GAUSS5, NB>(dim3((unsigned)blocks), st, src, blob,
                                                              h, (int)rb, nsegp, bands, ntp, nts, mean)
                              : launch_pt_blob<OP_GAUSS3, NB>(dim3((unsigned)blocks), st, src, blob,
                                                              h, (int)rb, nsegp, bands, ntp, nts, mean);
    if (rc) return rc;
    IDN_CHECK_LAUNCH("idn_gaussian_blob_f32");
    return IDN_OK;
  }
  const int nseg = (int)((rb + 1007) / 1008);
  const int seg_len = (int)(((rb + nseg - 1) / nseg + 7) / 8 * 8);
  constexpr int NB = 6;
  const int bands = (h + NB - 1) / NB;
  const int64_t total = (int64_t)n * bands * nseg;
  IDN_CHECK_ARG(total < (int64_t)0x7FFFFFFF, "idn_gaussian_blob_f32: batch too large");
  const dim3 grid((unsigned)((int64_t)n * bands)), block(TILE_WGT);
  if (ksize == 5 && knob("IDN_STENCIL_GLDS", 1))  // LDS-DMA tile fetch (as the u8 filters)
    hipLaunchKernelGGL((stencil_u8_lds<3, OP_GAUSS5, NB, EPI_BLOB, 0, 1>), grid, block, 0, st, src,
                       nullptr, h, (int)rb, nseg, seg_len, bands, (int)total, blob, mean[0],
                       mean[1], mean[2]);
  else if (ksize == 5)
    hipLaunchKernelGGL((stencil_u8_lds<3, OP_GAUSS5, NB, EPI_BLOB>), grid, block, 0, st, src,
                       nullptr, h, (int)rb, nseg, seg_len, bands, (int)total, blob, mean[0],
                       mean[1], mean[2]);
  else if (knob("IDN_STENCIL_GLDS", 1))
    hipLaunchKernelGGL((stencil_u8_lds<3, OP_GAUSS3, NB, EPI_BLOB, 0, 1>), grid, block, 0, st, src,
                       nullptr, h, (int)rb, nseg, seg_len, bands, (int)total, blob, mean[0],
                       mean[1], mean[2]);
  else
    hipLaunchKernelGGL((stencil_u8_lds<3, OP_GAUSS3, NB, EPI_BLOB>), grid, block, 0, st, src,
                       nullptr, h, (int)rb, nseg, seg_len, bands, (int)total, blob, mean[0],
                       mean[1], mean[2]);
  IDN_CHECK_LAUNCH("idn_gaussian_blob_f32");
  return IDN_OK;
}
