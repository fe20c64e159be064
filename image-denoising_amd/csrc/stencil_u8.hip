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
#include "noise_apply.hpp"

#include <type_traits>

namespace idn {

// OP_IDENT5: tuning probe only (IDN_STENCIL_IDENT=1 on the 5x5 Gaussian entry point) -- the 5x5
// kernels' memory structure (tile fetch, halo rows, stores) with the arithmetic reduced to a copy
// of the centre byte, to separate what the data movement costs from what the taps cost
enum StencilOp { OP_GAUSS3 = 0, OP_GAUSS5 = 1, OP_BOX3 = 2, OP_IDENT5 = 3 };

template <int OP> struct Stencil;
template <> struct Stencil<OP_GAUSS3> { static constexpr int K = 3; };
template <> struct Stencil<OP_GAUSS5> { static constexpr int K = 5; };
template <> struct Stencil<OP_BOX3> { static constexpr int K = 3; };
template <> struct Stencil<OP_IDENT5> { static constexpr int K = 5; };

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
  if constexpr (OP == OP_IDENT5) {
    return r2;
  } else if constexpr (OP == OP_GAUSS5) {
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
  if constexpr (OP == OP_IDENT5) {
    return V.at(P) << 8;  // the centre byte into the high byte of each u16 lane
  } else if constexpr (OP == OP_GAUSS5) {
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

constexpr int RING_WGT = 192;
enum RingPre { PRE_NONE = 0, PRE_GAUSSIAN = 1, PRE_SPECKLE = 2, PRE_SAP = 3 };
enum RingEpi { EPI_U8 = 0, EPI_BLOB = 1, EPI_FLAT = 2 };

struct RingArgs {
  const uint8_t* src;
  uint8_t* dst;
  float* blob;
  int h, rb, nseg, seg_len, bands, strips_per_img, bands_per_strip;
  uint64_t key, offset;
  const uint64_t* ids;
  double p1;
  uint32_t t_flip, t_salt;
  double mean[3];
};

// the blob of one lane's 16 output bytes at row byte offset q: 16 floats, 4 (full chunk) or
// 2 (half chunk) 16-byte stores; always 6 store instructions (unused ones out of range)
__device__ __forceinline__ void blob_store16(const v4u& o, const double (&means)[3],
                                             rsrc_t rb_rsrc, const StoreOffs& so,
                                             uint32_t row_off, int m0) {
  const uint32_t b[4] = {o.x, o.y, o.z, o.w};
  float f[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int ch = (m0 + i) % 3;
    const double mean = ch == 0 ? means[0] : ch == 1 ? means[1] : means[2];
    f[i] = (float)__dsub_rn((double)((b[i >> 2] >> (8 * (i & 3))) & 0xFFu), mean);
  }
  auto v = [&](int k) {
    return v4u{__float_as_uint(f[4 * k]), __float_as_uint(f[4 * k + 1]),
               __float_as_uint(f[4 * k + 2]), __float_as_uint(f[4 * k + 3])};
  };
  const uint32_t full = so.full + row_off, half = so.half + row_off;  // byte offsets
  // full chunk: bytes q..q+15 -> floats at 4*(q..q+15)
#pragma unroll
  for (int k = 0; k < 4; ++k)
    __builtin_amdgcn_raw_buffer_store_b128(v(k), rb_rsrc, full >= OOB_OFF ? OOB_OFF : 4u * full + 16u * k, 0, 0);
  // half chunk: bytes 0..7 (at q) or 8..15 (at q + 8) of the chunk
#pragma unroll
  for (int k = 0; k < 2; ++k)
    __builtin_amdgcn_raw_buffer_store_b128(so.hi ? v(2 + k) : v(k), rb_rsrc,
                                           half >= OOB_OFF ? OOB_OFF : 4u * half + 16u * k, 0, 0);
}

// ---- LDS-tiled form --------------------------------------------------------------------------
// One workgroup = one band of NB output rows of one image, nseg waves (<= 3: rows <= 3024 bytes).
// The band's NB + 2R input rows are contiguous in HBM (row_stride == row bytes), so the whole
// tile is fetched flat -- 16 B per lane, consecutive lanes on consecutive addresses, all loads in
// flight at once -- and staged in LDS; the waves then walk their row segments out of LDS with
// the vertical-first arithmetic above and store their output rows directly.  Measured on this
// chip the flat tile fetch sustains ~5.8 TB/s copy-equivalent where per-segment row loads stop
// near 5.2 (tools/membench3.hip).
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

template <int C, int OP, int NB, int NT, int EPI = EPI_U8>
__global__ __launch_bounds__(TILE_WGT) void stencil_u8_lds(const uint8_t* __restrict__ src,
                                                          uint8_t* __restrict__ dst, int h, int rb,
                                                          int nseg, int seg_len, int bands,
                                                          int total_items, int map,
                                                          float* __restrict__ blob = nullptr,
                                                          double mb = 0.0, double mg = 0.0,
                                                          double mr = 0.0) {
  constexpr int K = Stencil<OP>::K;
  constexpr int R = K / 2;
  using TS = TileShape<NB, K>;
  __shared__ __attribute__((aligned(16))) uint8_t tile[TS::LDS];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // map: bits 0-1 block order (1 XCD-contiguous, 2 plain), bit 2 the full-band fast fetch
  const int blk = (map & 3) == 1 ? xcd_contiguous_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
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

  // flat fetch of the tile into LDS (out-of-image lanes read 0 and are not written)
  {
    v4u v[TS::NL];
    // split policy (NT & 4): chunks inside the band's private rows [y0 + R, y1 - R) -- rows no
    // neighbouring band fetches -- load nontemporal, the rest default; two loads per chunk, the
    // unused one at an out-of-range offset (no memory access, returns 0)
    const uint32_t p_lo = (uint32_t)(y0 + R) * (uint32_t)rb - base_al;
    const uint32_t p_hi = y1 - R > y0 + R ? (uint32_t)(y1 - R) * (uint32_t)rb - base_al : p_lo;
    // full bands (every chunk but the last round's inside the tile): one lane offset, the round
    // in the scalar offset, no per-load compare / select and no guarded LDS stores but the last
    // round's (~30 fewer VALU per band: the filter runs at the power cap, so VALU is time)
    const bool full = (NT & 4) == 0 && (map & 4) != 0 &&
                      __builtin_amdgcn_readfirstlane(
                          (int)(nbytes >= (uint32_t)(16 * TILE_WGT * (TS::NL - 1))));
    if (full) {
      const uint32_t vo = base_al + 16u * threadIdx.x;
#pragma unroll
      for (int i = 0; i < TS::NL - 1; ++i)
        v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 16 * TILE_WGT * i, (NT & 1) ? 2 : 0);
      const uint32_t o = 16u * (uint32_t)(TILE_WGT * (TS::NL - 1) + threadIdx.x);
      v[TS::NL - 1] = __builtin_amdgcn_raw_buffer_load_b128(rs, o < nbytes ? base_al + o : OOB_OFF,
                                                            0, (NT & 1) ? 2 : 0);
#pragma unroll
      for (int i = 0; i < TS::NL - 1; ++i)
        *reinterpret_cast<v4u*>(&tile[16u * (uint32_t)(TILE_WGT * i + threadIdx.x)]) = v[i];
      if (o < nbytes) *reinterpret_cast<v4u*>(&tile[o]) = v[TS::NL - 1];
    } else {
#pragma unroll
    for (int i = 0; i < TS::NL; ++i) {
      const uint32_t o = 16u * (uint32_t)(TILE_WGT * i + threadIdx.x);
      const uint32_t off = o < nbytes ? base_al + o : OOB_OFF;
      if constexpr ((NT & 4) != 0) {
        const bool priv = o >= p_lo && o + 16u <= p_hi;
        const v4u a = __builtin_amdgcn_raw_buffer_load_b128(rs, priv ? OOB_OFF : off, 0, 0);
        const v4u b = __builtin_amdgcn_raw_buffer_load_b128(rs, priv ? off : OOB_OFF, 0, 2);
        v[i] = a | b;
      } else {
        v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, (NT & 1) ? 2 : 0);
      }
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
  if (EPI != EPI_FLAT && !active) return;

  const uint32_t ld_off = g.lead ? 0u : (uint32_t)g.q;
  const int nin = (y1 - y0) + 2 * R;
  const StoreOffs so = store_offs(g);
  uint32_t Rg[K][8];
  auto take_row = [&](int r) {
    const int y = reflect101_1(y0 - R + min(r, nin - 1), h);
    lds_take_row<C>(tile, (uint32_t)(y - ys) * (uint32_t)rb + shift + ld_off, g.lead, Rg[r % K]);
  };
  if constexpr (EPI == EPI_FLAT) {
    // Flat epilogue: the band's NB output rows are contiguous in HBM too.  Each wave keeps its
    // rows in registers until every wave has read the tile, stages them in LDS over the tile in
    // image order, and the workgroup stores the band flat -- 16 B per lane, consecutive lanes on
    // consecutive addresses, whole 128-B lines except the two a band shares with its neighbours
    // -- where the row segments' own stores leave partial lines at every segment and row edge.
    // The host takes this form when NB * rb, the image size and dst are 16-byte multiples.
    v4u ov[NB];
    if (active) {
#pragma unroll
      for (int r = 0; r < 2 * R; ++r) take_row(r);
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int r = 2 * R + u;
        take_row(r);
        ov[u] = ring_row<C, OP>(Rg, r % K, g);
        // one row at a time: without the fence the scheduler hoists every row's LDS reads and
        // the held output rows push the kernel past 128 VGPRs (3 waves per SIMD)
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __syncthreads();  // the tile is consumed: reuse it for the output band
    if (active && g.kind != 0) {
      const uint32_t lo = g.kind == 3 ? (uint32_t)g.q + 8u : (uint32_t)g.q;
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        if (y0 + u < y1) {
          const uint32_t o = (uint32_t)u * (uint32_t)rb + lo;
          const v2u a = g.kind == 3 ? v2u{ov[u].z, ov[u].w} : v2u{ov[u].x, ov[u].y};
          *reinterpret_cast<v2u*>(&tile[o]) = a;
          if (g.kind == 1) *reinterpret_cast<v2u*>(&tile[o + 8]) = v2u{ov[u].z, ov[u].w};
        }
      }
    }
    __syncthreads();
    constexpr int NLO = (NB * TILE_RBMAX + 16 * TILE_WGT - 1) / (16 * TILE_WGT);
    // bytes of the band (0 for a workgroup past the batch: it stores nothing)
    const uint32_t nout = (item < total_items && y1 > y0) ? (uint32_t)(y1 - y0) * (uint32_t)rb : 0u;
    const uint32_t gbase = (uint32_t)y0 * (uint32_t)rb;
#pragma unroll
    for (int i = 0; i < NLO; ++i) {
      const uint32_t o = 16u * (uint32_t)(TILE_WGT * i + threadIdx.x);
      const v4u v = *reinterpret_cast<const v4u*>(&tile[o < nout ? o : 0u]);
      __builtin_amdgcn_raw_buffer_store_b128(v, rd, o < nout ? gbase + o : OOB_OFF, 0,
                                             (NT & 2) ? 2 : 0);
    }
    return;
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
      const double means[3] = {mb, mg, mr};
      blob_store16(ring_row<C, OP>(Rg, r % K, g), means, rd, so, row_off, ((g.q % 3) + 3) % 3);
    } else {
      ring_out_row<C, OP, NT>(Rg, r % K, g, rd, so, row_off);
    }
  }
}


// ---- persistent band-tile form with register prefetch ------------------------------------------
// The tile form above stops fetching while its waves filter: a resident workgroup alternates a
// burst of loads with a stretch of arithmetic, so the bytes in flight per CU dip whenever several
// of its workgroups filter at once.  Here a resident workgroup walks a sequence of bands and
// issues the NEXT band's tile loads into registers right after staging the current one, so its
// loads are in flight for the whole filtering of the current band:
//   prefetch(t0) -> [ barrier; registers -> LDS; barrier; prefetch(t + P); filter band t ] ...
// Band order keeps neighbours together: XCD x (blockIdx & 7) owns the contiguous band range
// [T x / 8, T (x + 1) / 8) of the flattened (image, band) list, and its P/8 workgroups take
// consecutive bands at every step, so a band's halo rows were fetched by the band before it on
// the same XCD moments earlier and come from that XCD's L2.
template <int C, int OP, int NB, int NT>
__global__ __launch_bounds__(TILE_WGT) void stencil_u8_pf(const uint8_t* __restrict__ src,
                                                         uint8_t* __restrict__ dst, int h, int rb,
                                                         int nseg, int seg_len, int bands,
                                                         int total_bands) {
  constexpr int K = Stencil<OP>::K;
  constexpr int R = K / 2;
  using TS = TileShape<NB, K>;
  __shared__ __attribute__((aligned(16))) uint8_t tile[TS::LDS];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int xcd = blockIdx.x & 7, per = gridDim.x >> 3;  // gridDim.x % 8 == 0 (host)
  const int t_lo = (int)(((int64_t)total_bands * xcd) >> 3);
  const int t_hi = (int)(((int64_t)total_bands * (xcd + 1)) >> 3);
  const uint32_t img_bytes = (uint32_t)h * (uint32_t)rb;

  // fetch geometry of band t (workgroup-uniform)
  struct Fetch {
    int img, y0, y1, ys;
    uint32_t base_al, shift, nbytes;
  };
  auto fetch_geom = [&](int t) {
    Fetch f;
    f.img = t / bands;
    const int band = t - f.img * bands;
    f.y0 = band * NB;
    f.y1 = min(f.y0 + NB, h);
    f.ys = max(f.y0 - R, 0);
    const int ye = min(f.y1 + R, h);
    const uint32_t base = (uint32_t)f.ys * (uint32_t)rb;
    f.base_al = base & ~15u;
    f.shift = base - f.base_al;
    f.nbytes = (uint32_t)ye * (uint32_t)rb - f.base_al;
    return f;
  };
  v4u v[TS::NL];
  auto prefetch = [&](const Fetch& f) {
    const rsrc_t rs = make_rsrc(src + (size_t)f.img * img_bytes, img_bytes);
#pragma unroll
    for (int i = 0; i < TS::NL; ++i) {
      const uint32_t o = 16u * (uint32_t)(TILE_WGT * i + threadIdx.x);
      v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, o < f.nbytes ? f.base_al + o : OOB_OFF, 0,
                                                    (NT & 1) ? 2 : 0);
    }
  };

  int t = t_lo + (int)(blockIdx.x >> 3);
  Fetch f = fetch_geom(t < t_hi ? t : t_lo);
  if (t < t_hi) prefetch(f);
#pragma unroll 1
  for (; t < t_hi; t += per) {
    __syncthreads();  // every wave has finished reading the previous band's tile
#pragma unroll
    for (int i = 0; i < TS::NL; ++i) {
      const uint32_t o = 16u * (uint32_t)(TILE_WGT * i + threadIdx.x);
      if (o < f.nbytes) *reinterpret_cast<v4u*>(&tile[o]) = v[i];
    }
    __syncthreads();
    const Fetch cur = f;
    if (t + per < t_hi) {  // the next band's loads stay in flight while this band is filtered
      f = fetch_geom(t + per);
      prefetch(f);
    }
    if (wave >= nseg) continue;  // rows narrower than 3 segments: the spare wave only fetches
    const int band = t - cur.img * bands;
    const StripeGeom g = stripe_geom((cur.img * bands + band) * nseg + wave, lane, rb, nseg,
                                     seg_len, bands);
    const rsrc_t rd = make_rsrc(dst + (size_t)cur.img * img_bytes, img_bytes);
    const uint32_t ld_off = g.lead ? 0u : (uint32_t)g.q;
    const int nin = (cur.y1 - cur.y0) + 2 * R;
    const StoreOffs so = store_offs(g);
    uint32_t Rg[K][8];
    auto take_row = [&](int r) {
      const int y = reflect101_1(cur.y0 - R + min(r, nin - 1), h);
      lds_take_row<C>(tile, (uint32_t)(y - cur.ys) * (uint32_t)rb + cur.shift + ld_off, g.lead,
                      Rg[r % K]);
    };
#pragma unroll
    for (int r = 0; r < 2 * R; ++r) take_row(r);
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int r = 2 * R + u;
      take_row(r);
      const int y = cur.y0 + u;
      ring_out_row<C, OP, NT>(Rg, r % K, g, rd, so,
                              y < cur.y1 ? (uint32_t)y * (uint32_t)rb : OOB_OFF);
    }
  }
}

// ---- streaming ring form (+ fused noise prologue / blob epilogue) ------------------------------
// One workgroup (3 waves) walks a STRIP of consecutive bands of one image top to bottom.  The
// image's bytes stream through an LDS ring of NSLOT 1 KB chunks by LDS-DMA
// (buffer_load_dwordx4 ... lds), PD bands ahead of the band being filtered: every input byte is
// fetched from HBM once per strip (no halo re-reads by neighbouring bands) and, with a noise
// prologue, noised once per strip -- which is what makes it the form for the fused
// noise -> filter step (BASELINE config 2: random_noise + cv2.blur, lib/model/test.py:220-241):
// the noise is VALU-bound, and the band-tiled form would recompute it for every halo row.
//   chunk m (image bytes [1024 m, 1024 m + 1024)) lives in ring slot m mod NSLOT; image byte B
//   sits at ring offset (B >> 10) mod NSLOT * 1024 + (B & 1023); a row is read with the tile
//   form's lane layout (two 8-byte LDS reads per lane, each in one chunk).
// Per band i (all counts wave-uniform, so one immediate vmcnt serves every wave):
//   issue band i+PD's new chunks (exactly MAXC DMAs per wave; unused ones land in a dump slot)
//   -> s_waitcnt vmcnt(PD*MAXC + PD*NB*SPR) retires band i's chunks (younger: PD bands of DMAs
//   and PD bands of NB*SPR stores; the prologue issues PD*NB*SPR dummy stores so the count holds
//   from the first band) -> s_barrier -> [noise prologue: the waves noise band i's new chunks in
//   place in LDS, s_barrier] -> filter + store NB rows (u8, or the float32 blob) -> s_barrier.
// Epilogue EPI_BLOB: blob = float32(float64(v) - PIXEL_MEANS[ch]) (lib/utils/blob.py:35-36,
// numpy's float64 subtract then float32 store), written straight from the filter registers:
// the blob of a filtered image without the u8 round trip through HBM.
template <int NB, int PD, int NSLOT, int EPI>
struct RingShape {
  static constexpr int RING = NSLOT * 1024;
  // chunks a band's new rows can touch (<= 3024-byte rows), split over 3 waves
  static constexpr int MAXC = ((NB * TILE_RBMAX + 1023) / 1024 + 1 + 2) / 3;
  static constexpr int MAXC0 = (((NB + 4) * TILE_RBMAX + 1023) / 1024 + 1 + 2) / 3;
  static constexpr int SPR = EPI == EPI_BLOB ? 6 : 2;  // stores per output row per lane
  static constexpr int VMCNT = PD * MAXC + PD * NB * SPR;
  static_assert((NB * (PD + 1) + 4) * TILE_RBMAX + 2048 <= RING, "ring too small for NB / PD");
  static_assert(VMCNT <= 63, "vmcnt field is 6 bits");
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  // s_waitcnt vmcnt(N) only; asm (with a memory clobber) so no memory op moves across it
  static_assert(N >= 0 && N <= 63, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int C, int OP, int NB, int PD, int NSLOT, int LAUX, int SAUX, int PRE, int EPI>
__global__ __launch_bounds__(RING_WGT) void stencil_u8_ring(RingArgs a) {
  constexpr int K = Stencil<OP>::K;
  constexpr int R = K / 2;
  using RS = RingShape<NB, PD, NSLOT, EPI>;
  __shared__ __attribute__((aligned(16))) uint8_t lds[RS::RING + 1024];
  uint8_t* const ring = lds;
  uint8_t* const dump = lds + RS::RING;

  const int h = a.h, rb = a.rb;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int strip = blockIdx.x;
  const int img = strip / a.strips_per_img;
  const int b0 = (strip % a.strips_per_img) * a.bands_per_strip;
  const int nbands = min(b0 + a.bands_per_strip, a.bands) - b0;
  if (nbands <= 0) return;  // whole workgroup: no barrier is pending
  const uint32_t img_bytes = (uint32_t)h * (uint32_t)rb;
  const rsrc_t rs = make_rsrc(a.src + (size_t)img * img_bytes, img_bytes);
  const rsrc_t rd = EPI == EPI_U8 ? make_rsrc(a.dst + (size_t)img * img_bytes, img_bytes)
                                  : make_rsrc(a.blob + (size_t)img * img_bytes, 4u * img_bytes);
  const uint64_t gimg = a.ids ? a.ids[img] : a.offset + (uint64_t)img;

  auto slot_off = [](uint32_t m) -> uint32_t { return (m % (uint32_t)NSLOT) << 10; };
  // band g of the strip needs image rows up to min(y0(g) + NB + R, h) resident
  auto chunk_end = [&](int g) -> uint32_t {
    const int yend = min((b0 + g) * NB + NB + R, h);
    return ((uint32_t)yend * (uint32_t)rb + 1023u) >> 10;
  };
  const uint32_t first = ((uint32_t)max(b0 * NB - R, 0) * (uint32_t)rb) >> 10;
  uint32_t F = first;
  auto issue = [&](uint32_t to, int maxc) {
    for (int i = 0; i < maxc; ++i) {
      const uint32_t m = F + (uint32_t)wave + 3u * (uint32_t)i;
      const bool valid = m < to;
      uint8_t* d = valid ? ring + slot_off(m) : dump;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)d, 16,
          valid ? (m << 10) + 16u * (uint32_t)lane : OOB_OFF, 0, 0, LAUX);
    }
    F = max(F, to);
  };

  // prologue: band 0's whole tile, then the new rows of bands 1..PD-1; dummy stores
  issue(chunk_end(0), RS::MAXC0);
  for (int g = 1; g < PD; ++g) issue(g < nbands ? chunk_end(g) : F, RS::MAXC);
  // (distinct out-of-range offsets: identical stores to one address would be merged away, and
  // the vmcnt arithmetic counts every one of them)
  for (int i = 0; i < PD * NB * RS::SPR; ++i)
    __builtin_amdgcn_raw_buffer_store_b128(v4u{0u, 0u, 0u, 0u}, rd, OOB_OFF + 16u * (uint32_t)i,
                                           0, SAUX);

  const StripeGeom g = stripe_geom(min(wave, a.nseg - 1), lane, rb, a.nseg, a.seg_len, 1);
  const bool active = wave < a.nseg;
  const uint32_t ld_off = g.lead ? 0u : (uint32_t)g.q;
  const StoreOffs so = store_offs(g);
  // channel of chunk byte 0 (q may be -8 for the row's lead lane)
  const int m0 = ((g.q % 3) + 3) % 3;
  const double means[3] = {a.mean[0], a.mean[1], a.mean[2]};

  for (int i = 0; i < nbands; ++i) {
    issue(i + PD < nbands ? chunk_end(i + PD) : F, RS::MAXC);
    wait_vmcnt<RS::VMCNT>();
    asm volatile("s_barrier" ::: "memory");
    if constexpr (PRE != PRE_NONE) {
      // noise the chunks that became resident for this band, in place
      const uint32_t lo = i == 0 ? first : max(first, chunk_end(i - 1));
      const uint32_t hi = max(lo, chunk_end(i));
      for (uint32_t m = lo + (uint32_t)wave; m < hi; m += 3u) {
        const uint32_t e0 = (m << 10) + 16u * (uint32_t)lane;
        if (e0 < img_bytes) {
          v4u* p = reinterpret_cast<v4u*>(ring + slot_off(m) + 16u * (uint32_t)lane);
          constexpr int KIND = PRE == PRE_GAUSSIAN ? IDN_NOISE_GAUSSIAN
                               : PRE == PRE_SPECKLE ? IDN_NOISE_SPECKLE : IDN_NOISE_SAP;
          *p = noise16_u8<KIND, true>(*p, e0 >> 4, gimg, a.key, 0.0, a.p1, a.t_flip, a.t_salt,
                                      nullptr);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    const int y0 = (b0 + i) * NB;
    const int y1 = min(y0 + NB, h);
    const int nin = (y1 - y0) + 2 * R;
    // all of the band's LDS reads first (one wait), then the arithmetic
    v4u raw[NB + 2 * R];
#pragma unroll
    for (int r = 0; r < NB + 2 * R; ++r) {
      const int y = reflect101_1(y0 - R + min(r, nin - 1), h);
      const uint32_t B = (uint32_t)y * (uint32_t)rb + ld_off;
      const v2u lo = *reinterpret_cast<const v2u*>(&ring[slot_off(B >> 10) + (B & 1023u)]);
      const uint32_t B8 = B + 8u;
      const v2u hi = *reinterpret_cast<const v2u*>(&ring[slot_off(B8 >> 10) + (B8 & 1023u)]);
      raw[r] = v4u{lo.x, lo.y, hi.x, hi.y};
    }
    uint32_t Rg[K][8];
    auto take_row = [&](int r) {
      v4u Lv = raw[r];
      const uint32_t L[4] = {Lv.x, Lv.y, Lv.z, Lv.w};
      const v4u F4 = v4u{lead_fix<C, BORDER_REFLECT101>(L, -8),
                         lead_fix<C, BORDER_REFLECT101>(L, -4), L[0], L[1]};
      Lv = g.lead ? F4 : Lv;
      unpack_row(Lv, Rg[r % K]);
    };
#pragma unroll
    for (int r = 0; r < 2 * R; ++r) take_row(r);
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int r = 2 * R + u;
      take_row(r);
      const int y = y0 + u;
      const uint32_t row_off = (active && y < y1) ? (uint32_t)y * (uint32_t)rb : OOB_OFF;
      if constexpr (EPI == EPI_BLOB) {
        blob_store16(ring_row<C, OP>(Rg, r % K, g), means, rd, so, row_off, m0);
      } else {
        ring_out_row<C, OP, (SAUX & 2)>(Rg, r % K, g, rd, so, row_off);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
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

// ---- ring launch helpers -------------------------------------------------------------------------
inline bool ring_ok(int c, int64_t rb, int64_t row_stride, int h, const void* src, const void* dst,
                    int n, int K) {
  return stripe_ok(c, rb, row_stride, h, src, dst) && row_stride == rb && rb <= TILE_RBMAX &&
         h > K && n <= 65535;
}

// strips per image: about wg_per_cu resident workgroups per CU over the batch, strips of at
// least 4 bands
template <int OP, int NB, int PD, int NSLOT, int LAUX, int SAUX, int PRE, int EPI>
static void launch_ring(RingArgs a, int n, int h, int rb, int wg_per_cu, hipStream_t st) {
  a.h = h;
  a.rb = rb;
  a.nseg = (rb + 1007) / 1008;
  a.seg_len = ((rb + a.nseg - 1) / a.nseg + 7) / 8 * 8;
  a.bands = (h + NB - 1) / NB;
  const int64_t target = (int64_t)256 * wg_per_cu;
  int spi = (int)std::max<int64_t>(1, (target + n - 1) / n);
  spi = std::min(spi, std::max(1, a.bands / 4));
  a.bands_per_strip = (a.bands + spi - 1) / spi;
  a.strips_per_img = (a.bands + a.bands_per_strip - 1) / a.bands_per_strip;
  hipLaunchKernelGGL((stencil_u8_ring<3, OP, NB, PD, NSLOT, LAUX, SAUX, PRE, EPI>),
                     dim3((unsigned)(n * a.strips_per_img)), dim3(RING_WGT), 0, st, a);
}

// ---- host launchers --------------------------------------------------------------------------
// Band heights measured best on MI355X (256 x 600 x 1000 x 3 batch, tools/sweep_stencil.py):
// the tiled kernel with 6-row bands (10 / 8 input rows in LDS, 30 / 24 KB per workgroup, up to
// 5-6 workgroups per CU).  IDN_STENCIL_TILE=0 forces the stripe form, 2 / 3 pick other heights.
template <int OP>
static int launch_stencil(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                          int64_t row_stride, hipStream_t st, const char* name) {
  constexpr int K = Stencil<OP>::K;
  constexpr int R = K / 2;
  const int64_t rb = (int64_t)w * c;
  const int tile_mode = env_int("IDN_STENCIL_TILE", 1);
  // cache-policy variants (tuning): bit 0 nontemporal loads, bit 1 nontemporal stores, bit 2
  // split loads (nontemporal only for the band's private rows, default for the halo rows its
  // neighbours read too)
  const int ntmode = env_int("IDN_STENCIL_NT", 0) & 7;
  const bool ntst = (ntmode & 2) != 0;  // nontemporal stores
  const int map = (env_int("IDN_STENCIL_MAP", 1) == 2 ? 2 : 1) |
                  (env_int("IDN_STENCIL_FASTFETCH", 1) ? 4 : 0);  // stencil_u8_lds only
  const int ring_cfg = env_int("IDN_STENCIL_RING", 0);  // the band-tiled form is faster plain
  if (ring_cfg > 0 && ring_ok(c, rb, row_stride, h, src, dst, n, K)) {
    RingArgs a{};
    a.src = src;
    a.dst = dst;
    switch (ring_cfg) {
      case 2: launch_ring<OP, 4, 1, 38, 0, 0, PRE_NONE, EPI_U8>(a, n, h, (int)rb, 4, st); break;
      case 3: launch_ring<OP, 4, 1, 38, 2, 2, PRE_NONE, EPI_U8>(a, n, h, (int)rb, 4, st); break;
      case 4: launch_ring<OP, 6, 1, 50, 0, 0, PRE_NONE, EPI_U8>(a, n, h, (int)rb, 3, st); break;
      case 5: launch_ring<OP, 2, 3, 38, 0, 0, PRE_NONE, EPI_U8>(a, n, h, (int)rb, 4, st); break;
      default: launch_ring<OP, 6, 1, 64, 0, 0, PRE_NONE, EPI_U8>(a, n, h, (int)rb, 2, st); break;
    }
  } else if (env_int("IDN_STENCIL_PF", 0) && tile_mode && stripe_ok(c, rb, row_stride, h, src, dst) &&
             row_stride == rb && rb <= TILE_RBMAX && h > 2 * R) {
    // persistent register-prefetch form: as many 3-wave workgroups as are resident (LDS-bound),
    // a multiple of 8 (one band range per XCD)
    const int nseg = (int)((rb + 1007) / 1008);
    const int seg_len = (int)(((rb + nseg - 1) / nseg + 7) / 8 * 8);
    constexpr int NBP = 6;
    const int bands = (h + NBP - 1) / NBP;
    const int64_t total = (int64_t)n * bands;
    IDN_CHECK_ARG(total * nseg < (int64_t)0x7FFFFFFF, "%s: batch too large", name);
    const int per_cu = 160 * 1024 / TileShape<NBP, K>::LDS;
    int64_t grid = (int64_t)cu_count() * per_cu;
    const int64_t want = (total + 7) / 8 * 8;
    if (grid > want) grid = want;
    grid = (grid + 7) / 8 * 8;
    if (ntst)
      hipLaunchKernelGGL((stencil_u8_pf<3, OP, NBP, 2>), dim3((unsigned)grid), dim3(TILE_WGT), 0,
                         st, src, dst, h, (int)rb, nseg, seg_len, bands, (int)total);
    else
      hipLaunchKernelGGL((stencil_u8_pf<3, OP, NBP, 0>), dim3((unsigned)grid), dim3(TILE_WGT), 0,
                         st, src, dst, h, (int)rb, nseg, seg_len, bands, (int)total);
  } else if (tile_mode && stripe_ok(c, rb, row_stride, h, src, dst) && row_stride == rb &&
      rb <= TILE_RBMAX && h > 2 * R) {
    const int nseg = (int)((rb + 1007) / 1008);
    const int seg_len = (int)(((rb + nseg - 1) / nseg + 7) / 8 * 8);
    constexpr int NB1 = 6, NB2 = K == 5 ? 11 : 10, NB3 = K == 5 ? 8 : 4;
    const int nb = tile_mode == 2 ? NB2 : tile_mode == 3 ? NB3 : tile_mode == 4 ? 5
                 : tile_mode == 5 ? 4 : tile_mode == 6 ? 7 : NB1;
    const int bands = (h + nb - 1) / nb;
    const int64_t total = (int64_t)n * bands * nseg;
    IDN_CHECK_ARG(total < (int64_t)0x7FFFFFFF, "%s: batch too large", name);
    const dim3 grid((unsigned)((int64_t)n * bands)), block(TILE_WGT);
    // flat output epilogue (EPI_FLAT): band starts and image bases on 16-byte boundaries
    const int flat_cfg = env_int("IDN_STENCIL_FLAT", 0);
    const bool flat = flat_cfg != 0 && ((int64_t)nb * rb) % 16 == 0 &&
                      ((int64_t)h * rb) % 16 == 0 && ((uintptr_t)dst & 15) == 0;
#define IDN_LAUNCH_TILE_NT(NBX, NTV)                                                              \
  if (flat)                                                                                       \
    hipLaunchKernelGGL((stencil_u8_lds<3, OP, NBX, NTV, EPI_FLAT>), grid, block, 0, st, src, dst, \
                       h, (int)rb, nseg, seg_len, bands, (int)total, map);                        \
  else                                                                                            \
    hipLaunchKernelGGL((stencil_u8_lds<3, OP, NBX, NTV>), grid, block, 0, st, src, dst, h,         \
                       (int)rb, nseg, seg_len, bands, (int)total, map)
#define IDN_LAUNCH_TILE(NBX)                                                                      \
  if (ntmode == 1)                                                                                \
    IDN_LAUNCH_TILE_NT(NBX, 1);                                                                   \
  else if (ntmode == 6)                                                                           \
    IDN_LAUNCH_TILE_NT(NBX, 6);                                                                   \
  else if (ntmode == 3)                                                                           \
    IDN_LAUNCH_TILE_NT(NBX, 3);                                                                   \
  else if (ntst)                                                                                  \
    IDN_LAUNCH_TILE_NT(NBX, 2);                                                                   \
  else                                                                                            \
    IDN_LAUNCH_TILE_NT(NBX, 0)
    if (tile_mode == 2) {
      IDN_LAUNCH_TILE(NB2);
    } else if (tile_mode == 3) {
      IDN_LAUNCH_TILE(NB3);
    } else if (tile_mode == 4) {
      IDN_LAUNCH_TILE(5);
    } else if (tile_mode == 5) {
      IDN_LAUNCH_TILE(4);
    } else if (tile_mode == 6) {
      IDN_LAUNCH_TILE(7);
    } else {
      IDN_LAUNCH_TILE(NB1);
    }
#undef IDN_LAUNCH_TILE
#undef IDN_LAUNCH_TILE_NT
  } else if (stripe_ok(c, rb, row_stride, h, src, dst)) {
    // strided or wide rows: stripe form.  Rows of <= 4 segments: short bands, one workgroup per
    // band, all band rows loaded up front; wider rows: long bands of independent waves.
    constexpr int PF = (K == 5) ? 5 : 6;
    constexpr int NBS = 6;
    const bool burst = (rb + 1007) / 1008 <= 4;
    const StripePlan p = plan_stripe(n, h, rb, K, burst ? 1 : PF, 5120, burst ? map : 0, NBS,
                                     burst ? NBS : 0);
    IDN_CHECK_ARG(p.total < (int64_t)0x7FFFFFFF, "%s: batch too large", name);
    const dim3 grid(p.grid), block(p.block);
#define IDN_LAUNCH_VF(NTV)                                                                        \
  if (burst)                                                                                      \
    hipLaunchKernelGGL((stencil_u8_vf<3, OP, NBS + K - 1, NTV, NBS>), grid, block, 0, st, src,    \
                       dst, h, (int)rb, (uint32_t)row_stride, p.nseg, p.seg_len, p.bands,         \
                       p.band_rows, (int)p.total, p.map);                                         \
  else                                                                                            \
    hipLaunchKernelGGL((stencil_u8_vf<3, OP, PF, NTV, 0>), grid, block, 0, st, src, dst, h,       \
                       (int)rb, (uint32_t)row_stride, p.nseg, p.seg_len, p.bands, p.band_rows,    \
                       (int)p.total, p.map)
    if (ntst) {
      IDN_LAUNCH_VF(2);
    } else {
      IDN_LAUNCH_VF(0);
    }
#undef IDN_LAUNCH_VF
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
  if (ksize == 5 && env_int("IDN_STENCIL_IDENT", 0))  // tuning probe: copy through the 5x5 form
    return launch_stencil<OP_IDENT5>(src, dst, n, h, w, c, row_stride, as_stream(stream),
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

// ---- fused entry points -----------------------------------------------------------------------
// noise -> filter in one pass (BASELINE config 2: random_noise(img, 'gaussian', var) + U8 +
// cv2.blur / cv2.GaussianBlur, lib/model/test.py:220-241, minibatch.py:115-146): the same
// Philox stream and float64 apply as idn_noise_u8 (flat form), so the result equals
// idn_noise_u8 followed by the filter bit for bit.  Supported: compact 3-channel rows of
// <= 3024 bytes, kind gaussian / speckle with mean 0, or s&p; otherwise IDN_EUNSUPPORTED and the
// caller runs the two steps.
extern "C" int idn_noise_filter_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                                   int64_t row_stride, int kind, double p0, double p1,
                                   uint64_t seed, uint64_t offset, const uint64_t* image_ids,
                                   int filter, int ksize, void* stream) {
  using namespace idn;
  if (int e = check_filter_args(src, dst, n, h, w, c, row_stride, "idn_noise_filter_u8")) return e;
  IDN_CHECK_ARG(n <= 65535, "idn_noise_filter_u8: at most 65535 images per call");
  if (n == 0) return IDN_OK;
  const int64_t rb = (int64_t)w * c;
  const int op = filter == 0 ? (ksize == 5 ? OP_GAUSS5 : ksize == 3 ? OP_GAUSS3 : -1)
                             : (filter == 1 && ksize == 3 ? OP_BOX3 : -1);
  const int K = ksize;
  // the flat noise stream (noise16_u8) is what idn_noise_u8 draws only for 16-element images
  // on 16-byte aligned buffers; other layouts use its element stream, so they are not fused
  const bool flat = ((int64_t)h * rb) % 16 == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0;
  if (op < 0 || !flat || !ring_ok(c, rb, row_stride, h, src, dst, n, K) ||
      (kind != IDN_NOISE_SAP && p0 != 0.0) || kind < 0 || kind > IDN_NOISE_SAP)
    return set_error(IDN_EUNSUPPORTED, "idn_noise_filter_u8: combination not fused");
  RingArgs a{};
  a.src = src;
  a.dst = dst;
  a.key = seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(kind + 1));  // noise.hip KIND_TAG
  a.offset = offset;
  a.ids = image_ids;
  if (kind == IDN_NOISE_SAP) {
    IDN_CHECK_ARG(p0 >= 0.0 && p0 <= 1.0 && p1 >= 0.0 && p1 <= 1.0,
                  "idn_noise_filter_u8: amount / salt_vs_pepper must be in [0, 1]");
    a.t_flip = sap_threshold(p0 / (p0 + (1.0 - p0)));
    a.t_salt = sap_threshold(p1 / (p1 + (1.0 - p1)));
  } else {
    IDN_CHECK_ARG(p1 >= 0.0, "idn_noise_filter_u8: var must be >= 0");
    a.p1 = pow(p1, 0.5);
  }
  hipStream_t st = as_stream(stream);
#define IDN_NF(OPV, PREV) launch_ring<OPV, 4, 1, 38, 0, 0, PREV, EPI_U8>(a, n, h, (int)rb, 4, st)
#define IDN_NF_OP(PREV)                     \
  if (op == OP_GAUSS5) IDN_NF(OP_GAUSS5, PREV); \
  else if (op == OP_GAUSS3) IDN_NF(OP_GAUSS3, PREV); \
  else IDN_NF(OP_BOX3, PREV)
  if (kind == IDN_NOISE_GAUSSIAN) {
    IDN_NF_OP(PRE_GAUSSIAN);
  } else if (kind == IDN_NOISE_SPECKLE) {
    IDN_NF_OP(PRE_SPECKLE);
  } else if (kind == IDN_NOISE_SAP) {
    IDN_NF_OP(PRE_SAP);
  } else {
    return set_error(IDN_EUNSUPPORTED, "idn_noise_filter_u8: poisson is not fused");
  }
#undef IDN_NF_OP
#undef IDN_NF
  IDN_CHECK_LAUNCH("idn_noise_filter_u8");
  return IDN_OK;
}

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
  const int nseg = (int)((rb + 1007) / 1008);
  const int seg_len = (int)(((rb + nseg - 1) / nseg + 7) / 8 * 8);
  constexpr int NB = 6;
  const int bands = (h + NB - 1) / NB;
  const int64_t total = (int64_t)n * bands * nseg;
  IDN_CHECK_ARG(total < (int64_t)0x7FFFFFFF, "idn_gaussian_blob_f32: batch too large");
  const dim3 grid((unsigned)((int64_t)n * bands)), block(TILE_WGT);
  hipStream_t st = as_stream(stream);
  if (ksize == 5)
    hipLaunchKernelGGL((stencil_u8_lds<3, OP_GAUSS5, NB, 0, EPI_BLOB>), grid, block, 0, st, src,
                       nullptr, h, (int)rb, nseg, seg_len, bands, (int)total, 1, blob, mean[0],
                       mean[1], mean[2]);
  else
    hipLaunchKernelGGL((stencil_u8_lds<3, OP_GAUSS3, NB, 0, EPI_BLOB>), grid, block, 0, st, src,
                       nullptr, h, (int)rb, nseg, seg_len, bands, (int)total, 1, blob, mean[0],
                       mean[1], mean[2]);
  IDN_CHECK_LAUNCH("idn_gaussian_blob_f32");
  return IDN_OK;
}
