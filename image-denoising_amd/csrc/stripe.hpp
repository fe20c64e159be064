// Shared building blocks of the "wave stripe" kernels (stencil, median): one wave owns one
// <=1008-byte segment of a band of rows; lane l holds the 16-byte chunk
// [seg_start - 8 + 16 l, +16) of the current row; the 8-byte halos come from the neighbouring
// lanes through DPP wave shifts; row and segment edges rebuild border bytes in registers.
#pragma once

#include "idn_common.hpp"

namespace idn {

enum Border { BORDER_REFLECT101 = 0, BORDER_REPLICATE = 1 };

// lane i <- lane i-1 (wave_shr:1); lane 0 reads 0 (bound_ctrl).  Lane 0 and lane 63 never consume
// the halo they would receive (lane 0 outputs only chunk bytes 8..15, lane 63 only 0..7, and
// R*C <= 8), so no zero-fill (and no extra v_mov) is needed.
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xF, 0xF, true);
}
// lane i <- lane i+1 (wave_shl:1); lane 63 reads 0
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xF, 0xF, true);
}

// byte P (0..31) of the 8-dword window W (window byte 0 = chunk byte -8)
__device__ __forceinline__ uint32_t wbyte(const uint32_t (&W)[8], int P) {
  return (W[P >> 2] >> (8 * (P & 3))) & 0xFFu;
}
// 4 bytes of the window starting at window byte P (P compile-time after unrolling)
__device__ __forceinline__ uint32_t wdword(const uint32_t (&W)[8], int P) {
  const int lo = P >> 2, s = P & 3;
  if (s == 0) return W[lo];
  return __builtin_amdgcn_alignbyte(W[lo + 1], W[lo], s);
}
__device__ __forceinline__ uint32_t even_u16(uint32_t x) { return x & 0x00FF00FFu; }
__device__ __forceinline__ uint32_t odd_u16(uint32_t x) { return (x >> 8) & 0x00FF00FFu; }

// u16-lane view of the window: for window byte b, the register holding bytes (b, b+2) in its
// two u16 lanes.  SE[j] = bytes (4j, 4j+2), SO[j] = (4j+1, 4j+3); b = 4m+2 / 4m+3 straddle two
// dwords and are formed with one v_alignbyte_b32 (a 2-byte funnel shift).
struct Lanes16 {
  uint32_t SE[8], SO[8];
  __device__ __forceinline__ uint32_t at(int b) const {
    const int m = b >> 2;
    switch (b & 3) {
      case 0: return SE[m];
      case 1: return SO[m];
      case 2: return __builtin_amdgcn_alignbyte(SE[m + 1], SE[m], 2);
      default: return __builtin_amdgcn_alignbyte(SO[m + 1], SO[m], 2);
    }
  }
};

// Build the 4 bytes at row positions [p0, p0+4) (p0 < 0) that lie left of the row start from
// the 16 bytes L (row bytes 0..15).
template <int C, int BORDER>
__device__ __forceinline__ uint32_t lead_fix(const uint32_t (&L)[4], int p0) {
  uint32_t r = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int p = p0 + b;                // negative row byte
    const int pix = (p - (C - 1)) / C;   // floor(p / C) for p < 0
    const int ch = p - pix * C;
    const int src = (BORDER == BORDER_REFLECT101) ? (-pix * C + ch) : ch;  // < 16 for C <= 4
    r |= ((L[src >> 2] >> (8 * (src & 3))) & 0xFFu) << (8 * b);
  }
  return r;
}

// Bytes at row positions rb + k (k = k0..k0+3) rebuilt from window bytes; `base` = window byte of
// row position rb.
template <int C, int BORDER>
__device__ __forceinline__ uint32_t tail_fix(const uint32_t (&W)[8], int base, int k0) {
  uint32_t r = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int k = k0 + b;
    const int src = (BORDER == BORDER_REFLECT101) ? base - 2 * C - (k / C) * C + (k % C)
                                                  : base - C + (k % C);
    r |= wbyte(W, src) << (8 * b);
  }
  return r;
}

// Assemble the 8-dword window of one row for this lane (DPP halos + border fixups).
template <int C, int BORDER>
__device__ __forceinline__ void build_window(const v4u& Lv, bool lead, bool fix_t0, bool fix_t8,
                                             uint32_t (&W)[8]) {
  W[2] = Lv.x;
  W[3] = Lv.y;
  W[4] = Lv.z;
  W[5] = Lv.w;
  if (lead) {  // chunk starts 8 bytes left of the row: rebuild from row bytes 0..15
    const uint32_t L[4] = {Lv.x, Lv.y, Lv.z, Lv.w};
    W[2] = lead_fix<C, BORDER>(L, -8);
    W[3] = lead_fix<C, BORDER>(L, -4);
    W[4] = L[0];
    W[5] = L[1];
  }
  W[0] = from_prev_lane(W[4]);
  W[1] = from_prev_lane(W[5]);
  W[6] = from_next_lane(W[2]);
  W[7] = from_next_lane(W[3]);
  if (fix_t0) {  // row end at chunk end: window bytes 24.. are past the row
    const uint32_t a = tail_fix<C, BORDER>(W, 24, 0);
    const uint32_t b = tail_fix<C, BORDER>(W, 24, 4);
    W[6] = a;
    W[7] = b;
  }
  if (fix_t8) {  // row end mid-chunk: window byte 16 == rb
    const uint32_t a = tail_fix<C, BORDER>(W, 16, 0);
    const uint32_t b = tail_fix<C, BORDER>(W, 16, 4);
    W[4] = a;
    W[5] = b;
  }
}

// u16-lane view of a raw window: the register holding window bytes (b, b+2) in its two lanes.
__device__ __forceinline__ uint32_t lanes16_at(const uint32_t (&W)[8], int b) {
  const int m = b >> 2;
  switch (b & 3) {
    case 0: return W[m] & 0x00FF00FFu;
    case 1: return __builtin_amdgcn_perm(0u, W[m], 0x0C030C01u);
    case 2: return __builtin_amdgcn_alignbyte(W[m + 1], W[m], 2) & 0x00FF00FFu;
    default: return __builtin_amdgcn_perm(0u, __builtin_amdgcn_alignbyte(W[m + 1], W[m], 2), 0x0C030C01u);
  }
}

// u16 window of vertical sums: SE[m] = window bytes (4m, 4m+2), SO[m] = (4m+1, 4m+3);
// window byte 0 = chunk byte -8.
struct VWin {
  uint32_t SE[8], SO[8];
  __device__ __forceinline__ uint32_t at(int b) const {  // (b, b+2) as a u16 pair
    const int m = b >> 2;
    switch (b & 3) {
      case 0: return SE[m];
      case 1: return SO[m];
      case 2: return __builtin_amdgcn_alignbyte(SE[m + 1], SE[m], 2);
      default: return __builtin_amdgcn_alignbyte(SO[m + 1], SO[m], 2);
    }
  }
  // register and half holding window byte b
  __device__ __forceinline__ uint32_t reg(int b) const { return (b & 1) ? SO[b >> 2] : SE[b >> 2]; }
};
// (a.half[ha], b.half[hb]) -> one u16 pair, one v_perm_b32
__device__ __forceinline__ uint32_t pick16(uint32_t a, int ha, uint32_t b, int hb) {
  const uint32_t sel = (uint32_t)(2 * ha) | (uint32_t)(2 * ha + 1) << 8 |
                       (uint32_t)(4 + 2 * hb) << 16 | (uint32_t)(5 + 2 * hb) << 24;
  return __builtin_amdgcn_perm(b, a, sel);
}
// rebuild window bytes [base, base+8) past the row end (row end = window byte `base`) by
// BORDER_REFLECT_101 / BORDER_REPLICATE from the bytes before it
template <int C, int BORDER = BORDER_REFLECT101>
__device__ __forceinline__ void vwin_tail_fix(VWin& V, int base) {
  uint32_t nE[2], nO[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      int src[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int k = 4 * m + par + 2 * t;  // window byte base + k
        src[t] = BORDER == BORDER_REFLECT101 ? base - 2 * C - (k / C) * C + (k % C)
                                             : base - C + (k % C);
      }
      const uint32_t r = pick16(V.reg(src[0]), (src[0] >> 1) & 1, V.reg(src[1]), (src[1] >> 1) & 1);
      (par ? nO : nE)[m] = r;
    }
  }
  const int mb = base >> 2;
  V.SE[mb] = nE[0];
  V.SO[mb] = nO[0];
  V.SE[mb + 1] = nE[1];
  V.SO[mb + 1] = nO[1];
}

// as unpack_row with 0x64 in the high byte of every u16 lane: each lane is the float16 value
// 1024 + v (a normal number, exact), whose bit pattern orders as v does, so the u16 and the
// float16 min/max instructions (v_pk_minimum3_f16 / v_pk_maximum3_f16) agree on it; the low byte
// is still v
__device__ __forceinline__ void unpack_row_f16(const v4u& x, uint32_t (&U)[8]) {
  const uint32_t d[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    U[j] = (d[j] & 0x00FF00FFu) | 0x64006400u;
    U[4 + j] = __builtin_amdgcn_perm(0x64646464u, d[j], 0x04030401u);
  }
}

// one input row -> 8 u16x2 dwords: [0..3] even bytes of chunk dwords 0..3, [4..7] odd bytes
__device__ __forceinline__ void unpack_row(const v4u& x, uint32_t (&U)[8]) {
  const uint32_t d[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    U[j] = d[j] & 0x00FF00FFu;
    U[4 + j] = __builtin_amdgcn_perm(0u, d[j], 0x0C030C01u);
  }
}

// Work-item geometry of a stripe launch (all wave-uniform).
struct StripeGeom {
  int seg, band, img;
  int seg_start, seg_end, q;
  bool lead, fix_t0, fix_t8;
  bool tail;  // wave-uniform: the wave owns the row's last segment (the only one with fix lanes)
  int kind;  // 0 none, 1 full 16 B, 2 low 8 B, 3 high 8 B
};

__device__ __forceinline__ StripeGeom stripe_geom(int item, int lane, int rb, int nseg,
                                                  int seg_len, int bands) {
  StripeGeom g;
  g.seg = item % nseg;
  const int tq = item / nseg;
  g.band = tq % bands;
  g.img = tq / bands;
  g.seg_start = g.seg * seg_len;
  g.seg_end = min(g.seg_start + seg_len, rb);
  g.q = g.seg_start - 8 + 16 * lane;
  g.lead = (g.seg_start == 0) && (lane == 0);
  const bool last_seg = (g.seg_end == rb);
  g.tail = last_seg;
  const int tail = (rb - g.seg_start + 8) & 15;
  g.fix_t0 = last_seg && tail == 0 && (g.q + 16 == rb);
  g.fix_t8 = last_seg && tail == 8 && (g.q + 8 == rb);
  const int o_lo = max(g.q, g.seg_start), o_hi = min(g.q + 16, g.seg_end);
  g.kind = (o_hi <= o_lo) ? 0 : (o_lo == g.q && o_hi == g.q + 16) ? 1 : (o_lo == g.q) ? 2 : 3;
  return g;
}

// Workgroup -> work-item mapping of a stripe launch.
//   map 0: 4 independent waves per workgroup, item = 4*block + wave (long bands, one round)
//   map 1: one workgroup = the nseg segments of one short band (whole rows, contiguous in HBM),
//          blocks renumbered so each XCD walks a contiguous run of bands: vertical neighbours
//          run on the same XCD at about the same time and their halo rows hit its L2
//   map 2: as 1 without the XCD renumbering
__device__ __forceinline__ int stripe_item(int map, int nseg) {
  const int wave = threadIdx.x >> 6;
  if (map == 0) return __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wave);
  const int b = map == 1 ? xcd_contiguous_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  return __builtin_amdgcn_readfirstlane(b * nseg + wave);
}

template <int NT>
__device__ __forceinline__ void stripe_store(const v4u& o, rsrc_t rd, uint32_t off, int kind) {
  constexpr int aux = (NT & 2) ? 2 : 0;
  if (kind == 1) {
    __builtin_amdgcn_raw_buffer_store_b128(o, rd, off, 0, aux);
  } else if (kind == 2) {
    v2u lo2 = {o.x, o.y};
    __builtin_amdgcn_raw_buffer_store_b64(lo2, rd, off, 0, aux);
  } else if (kind == 3) {
    v2u hi2 = {o.z, o.w};
    __builtin_amdgcn_raw_buffer_store_b64(hi2, rd, off + 8u, 0, aux);
  }
}

// Branch-free form of stripe_store: out-of-range buffer offsets drop a store in hardware, so the
// lane's kind and the row's validity select offsets instead of exec-masked branches.  Lanes of
// kind 1 issue one 16-byte store; the (at most two) edge lanes of kind 2/3 issue an 8-byte store.
// >= any image (stripe_ok bounds images below 2^30); the sum of two offsets never wraps
constexpr uint32_t OOB_OFF = 0x40000000u;
struct StoreOffs {
  uint32_t full, half;  // per-lane byte offsets relative to the row start (OOB when unused)
  bool hi;              // the half store carries bytes 8..15 of the chunk
};
__device__ __forceinline__ StoreOffs store_offs(const StripeGeom& g) {
  StoreOffs s;
  s.full = g.kind == 1 ? (uint32_t)g.q : OOB_OFF;
  s.hi = g.kind == 3;
  s.half = g.kind == 2 ? (uint32_t)g.q : (g.kind == 3 ? (uint32_t)g.q + 8u : OOB_OFF);
  return s;
}
template <int NT>
__device__ __forceinline__ void stripe_store_nb(const v4u& o, rsrc_t rd, const StoreOffs& so,
                                                uint32_t row_off) {
  constexpr int aux = (NT & 2) ? 2 : 0;
  // row_off == OOB_OFF for a row that must not be written: every offset lands out of range
  __builtin_amdgcn_raw_buffer_store_b128(o, rd, so.full + row_off, 0, aux);
  v2u h2 = so.hi ? v2u{o.z, o.w} : v2u{o.x, o.y};
  __builtin_amdgcn_raw_buffer_store_b64(h2, rd, so.half + row_off, 0, aux);
}

// BORDER_REFLECT_101 row index for -len < i < 2*len - 1 (one reflection; callers guarantee
// len > kernel radius), without the loop of reflect101()
__device__ __forceinline__ int reflect101_1(int i, int len) {
  i = i < 0 ? -i : i;
  return i >= len ? 2 * len - 2 - i : i;
}

// Host-side stripe geometry: segments of <= 1008 bytes, bands sized to one resident round.
struct StripePlan {
  int nseg, seg_len, bands, band_rows;
  int64_t total;
  int map;       // see stripe_item()
  unsigned grid, block;
};


// map_default: the workgroup mapping used when IDN_STRIPE_MAP is unset; short_rows: band height
// target of the row-workgroup maps (rounded up so band + halo fills whole unroll groups).
inline StripePlan plan_stripe(int n, int h, int64_t rb, int K, int U, int64_t cap,
                              int map_default = 0, int short_rows = 32, int fixed_rows = 0) {
  StripePlan p;
  p.nseg = (int)((rb + 1007) / 1008);
  p.seg_len = (int)(((rb + p.nseg - 1) / p.nseg + 7) / 8 * 8);
  p.map = knob("IDN_STRIPE_MAP", map_default);
  if (p.nseg > 4) p.map = 0;  // rows wider than 4 segments: independent waves
  int band_rows = fixed_rows > 0 ? fixed_rows : knob("IDN_BAND_ROWS", 0);
  if (band_rows <= 0 && p.map != 0) {
    band_rows = short_rows < h ? short_rows : h;
    while ((band_rows + (K - 1)) % U != 0 && band_rows < h) ++band_rows;
  }
  if (band_rows <= 0) {
    int64_t bands = cap / ((int64_t)n * p.nseg);
    if (bands < 1) bands = 1;
    band_rows = (int)((h + bands - 1) / bands);
    if (band_rows < 24) band_rows = 24;
    while ((band_rows + (K - 1)) % U != 0 && band_rows < h) ++band_rows;
  }
  p.band_rows = band_rows;
  p.bands = (h + band_rows - 1) / band_rows;
  p.total = (int64_t)n * p.bands * p.nseg;
  if (p.map == 0) {
    p.block = 256;
    p.grid = (unsigned)((p.total + 3) / 4);
  } else {
    p.block = 64u * (unsigned)p.nseg;
    p.grid = (unsigned)((int64_t)n * p.bands);
  }
  return p;
}

inline bool stripe_ok(int c, int64_t rb, int64_t row_stride, int h, const void* src,
                      const void* dst) {
  return c == 3 && rb % 8 == 0 && row_stride % 8 == 0 && rb >= 32 && h >= 5 &&
         (int64_t)h * row_stride < (int64_t)0x40000000 && ((uintptr_t)src & 7) == 0 &&
         ((uintptr_t)dst & 7) == 0 && knob("IDN_FORCE_GENERIC", 0) == 0;
}

}  // namespace idn
