// cv2.medianBlur(u8, 3|5) on interleaved HxWxC images, BORDER_REPLICATE, bit-exact.
// Reference call sites: lib/model/test.py:259, lib/roi_data_layer/minibatch.py:153,1644-1648.
//
// Same wave-stripe streaming as the stencils (stripe.hpp): one wave = one segment of a band of
// rows, 16 bytes per lane, DPP halos, replicated borders rebuilt in registers, a K-row ring of
// unpacked rows.  Selection runs on packed u16 pairs (v_pk_min_u16 / v_pk_max_u16): every
// comparator handles two output bytes.
//   3x3: each input row is unpacked once into u16 lanes; per output row every window column is
//        sorted once and shared by the 3 outputs that read it (halos by DPP on the sorted
//        columns), then med3(max3(col mins), med3(col medians), min3(col maxes)).
//   5x5: each input row is unpacked once into u16 lanes; per output row every window column is
//        sorted once (SORT5) and shared by the 5 outputs that read it; the sorted columns'
//        6-byte halos come from the neighbouring lanes by DPP; two chains of 5 same-channel
//        outputs (window bytes 8,11,..,20 and 9,12,..,21) each take their medians from 9 sorted
//        columns with a shared selection network (median_cols.hpp: 276 min/max per chain,
//        generated and proven by tools/gen_median_cols.py with the 0-1 principle).  ~55 min/max
//        per output byte pair instead of 202 for the unsorted 25-input network.
#include "stripe.hpp"
#include "median_cols.hpp"

namespace idn {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// Lanes hold float16 1024 + v (unpack_row_f16): 2-input min/max as packed u16, 3-input as the
// packed float16 v_pk_minimum3_f16 / v_pk_maximum3_f16 (exact: they return one of the inputs)
struct PkOps {
  __device__ __forceinline__ uint32_t mn(uint32_t a, uint32_t b) const {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
  }
  __device__ __forceinline__ uint32_t mx(uint32_t a, uint32_t b) const {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
  }
  __device__ __forceinline__ uint32_t mn3(uint32_t a, uint32_t b, uint32_t c) const {
    return __builtin_bit_cast(
        uint32_t, __builtin_elementwise_minimum(
                      __builtin_bit_cast(f16x2, a),
                      __builtin_elementwise_minimum(__builtin_bit_cast(f16x2, b),
                                                    __builtin_bit_cast(f16x2, c))));
  }
  __device__ __forceinline__ uint32_t mx3(uint32_t a, uint32_t b, uint32_t c) const {
    return __builtin_bit_cast(
        uint32_t, __builtin_elementwise_maximum(
                      __builtin_bit_cast(f16x2, a),
                      __builtin_elementwise_maximum(__builtin_bit_cast(f16x2, b),
                                                    __builtin_bit_cast(f16x2, c))));
  }
  __device__ __forceinline__ uint32_t med3(uint32_t a, uint32_t b, uint32_t c) const {
    return mx(mn(a, b), mn(mx(a, b), c));
  }
};

// one output row of the 3x3 median from the 3 unpacked rows of its window (oldest first): every
// window column is sorted once (shared by the 3 outputs that read it), the sorted columns' 3-byte
// halos come by DPP, then med3(max of the 3 column minima, med3 of the medians, min of the maxima)
template <int C>
__device__ __forceinline__ v4u median3_cols_out(const uint32_t (&U0)[8], const uint32_t (&U1)[8],
                                                const uint32_t (&U2)[8], bool fix_t0, bool fix_t8) {
  const PkOps op;
  VWin V[3];  // per rank (min, median, max): u16 window of the sorted columns
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t a = U0[j], b = U1[j], c = U2[j];
    const uint32_t l1 = op.mn(a, b), h1 = op.mx(a, b);
    const uint32_t lo = op.mn(l1, c), h2 = op.mx(l1, c);
    const uint32_t r[3] = {lo, op.mn(h1, h2), op.mx(h1, h2)};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (j < 4) V[k].SE[2 + j] = r[k];
      else V[k].SO[2 + (j - 4)] = r[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {  // 3-byte halos each side (R*C = 3): one dword per parity
    V[k].SE[0] = V[k].SO[0] = V[k].SE[7] = V[k].SO[7] = 0u;
    V[k].SE[1] = from_prev_lane(V[k].SE[5]);
    V[k].SO[1] = from_prev_lane(V[k].SO[5]);
    V[k].SE[6] = from_next_lane(V[k].SE[2]);
    V[k].SO[6] = from_next_lane(V[k].SO[2]);
    if (fix_t0) vwin_tail_fix<C, BORDER_REPLICATE>(V[k], 24);
    if (fix_t8) vwin_tail_fix<C, BORDER_REPLICATE>(V[k], 16);
  }
  uint32_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t v[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int P = 4 * q + 8 + e;
      const uint32_t lmax = op.mx3(V[0].at(P - C), V[0].at(P), V[0].at(P + C));
      const uint32_t mmed = op.med3(V[1].at(P - C), V[1].at(P), V[1].at(P + C));
      const uint32_t hmin = op.mn3(V[2].at(P - C), V[2].at(P), V[2].at(P + C));
      v[e] = op.med3(lmax, mmed, hmin);
    }
    o[q] = __builtin_amdgcn_perm(v[1], v[0], 0x06020400u);  // low byte of each u16 lane
  }
  return v4u{o[0], o[1], o[2], o[3]};
}

// one output row of the 5x5 median from the 5 unpacked rows of its window (oldest first)
template <int C>
__device__ __forceinline__ v4u median5_cols_out(const uint32_t (&U0)[8], const uint32_t (&U1)[8],
                                                const uint32_t (&U2)[8], const uint32_t (&U3)[8],
                                                const uint32_t (&U4)[8], bool fix_t0, bool fix_t8) {
  const PkOps op;
  VWin V[5];  // per rank: u16 window of the sorted columns
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t v[5] = {U0[j], U1[j], U2[j], U3[j], U4[j]};
    sort5(v, op);
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      if (j < 4) V[r].SE[2 + j] = v[r];
      else V[r].SO[2 + (j - 4)] = v[r];
    }
  }
#pragma unroll
  for (int r = 0; r < 5; ++r) {  // 6-byte halos each side (R*C = 6): two dwords per parity
    V[r].SE[0] = from_prev_lane(V[r].SE[4]);
    V[r].SO[0] = from_prev_lane(V[r].SO[4]);
    V[r].SE[1] = from_prev_lane(V[r].SE[5]);
    V[r].SO[1] = from_prev_lane(V[r].SO[5]);
    V[r].SE[6] = from_next_lane(V[r].SE[2]);
    V[r].SO[6] = from_next_lane(V[r].SO[2]);
    V[r].SE[7] = from_next_lane(V[r].SE[3]);
    V[r].SO[7] = from_next_lane(V[r].SO[3]);
    if (fix_t0) vwin_tail_fix<C, BORDER_REPLICATE>(V[r], 24);
    if (fix_t8) vwin_tail_fix<C, BORDER_REPLICATE>(V[r], 16);
  }
  // chain A: output pairs at window bytes 8+3k (bytes 8+3k, 10+3k); chain B: 9+3k (9+3k, 11+3k)
  uint32_t xa[9][5], xb[9][5];
#pragma unroll
  for (int c = 0; c < 9; ++c) {
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      xa[c][r] = V[r].at(2 + 3 * c);
      xb[c][r] = V[r].at(3 + 3 * c);
    }
  }
  uint32_t A[5], B[5];
  median25_chain5(xa, A, op);
  median25_chain5(xb, B, op);
  // each u16 lane holds one output byte in its low byte (b0 = lo lane, b2 = hi lane)
  //   bytes  8..11 = A0.lo B0.lo A0.hi B0.hi      12..15 = B1.lo A1.hi B1.hi B2.lo
  //   bytes 16..19 = A2.hi A3.lo B3.lo A3.hi      20..23 = A4.lo B4.lo A4.hi B4.hi
  const uint32_t o0 = __builtin_amdgcn_perm(B[0], A[0], 0x06020400u);
  const uint32_t t1 = __builtin_amdgcn_perm(A[1], B[1], 0x0C020600u);  // B1.lo A1.hi B1.hi -
  const uint32_t o1 = __builtin_amdgcn_perm(B[2], t1, 0x04020100u);
  const uint32_t t2 = __builtin_amdgcn_perm(A[3], A[2], 0x0C060402u);  // A2.hi A3.lo A3.hi -
  const uint32_t o2 = __builtin_amdgcn_perm(B[3], t2, 0x02040100u);
  const uint32_t o3 = __builtin_amdgcn_perm(B[4], A[4], 0x06020400u);
  return v4u{o0, o1, o2, o3};
}

template <int C, int K, int NT>
__global__ __launch_bounds__(256) void median_u8_fast(const uint8_t* __restrict__ src,
                                                      uint8_t* __restrict__ dst, int h, int rb,
                                                      uint32_t row_stride, int nseg, int seg_len,
                                                      int bands, int band_rows, int total_items,
                                                      int map) {
  constexpr int R = K / 2;
  constexpr int PF = K;  // prefetch depth == ring depth: one static slot pattern per group
  constexpr int U = K;

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
  const int ngroups = (nin + U - 1) / U;
  auto load_row = [&](int r) -> v4u {
    const int y = clampi(y0 - R + min(r, nin - 1), 0, h - 1);  // BORDER_REPLICATE
    return __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)y * row_stride + ld_off, 0,
                                                  (NT & 1) ? 2 : 0);
  };

  v4u Lq[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) Lq[i] = load_row(i);
  uint32_t Wr[K][8];  // unpacked u16 rows (even / odd bytes)

  for (int gi = 0; gi < ngroups; ++gi) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = gi * U + u;
      const v4u Lv = Lq[u % PF];
      Lq[u % PF] = load_row(r + PF);
      {
        v4u Lx = Lv;
        if (g.lead) {  // chunk = row bytes -8..7: rebuild the replicated 8 bytes
          const uint32_t L[4] = {Lv.x, Lv.y, Lv.z, Lv.w};
          Lx = v4u{lead_fix<C, BORDER_REPLICATE>(L, -8), lead_fix<C, BORDER_REPLICATE>(L, -4),
                   L[0], L[1]};
        }
        unpack_row_f16(Lx, Wr[u % K]);
      }
      const int y = y0 + r - 2 * R;
      if (r >= 2 * R && y < y1) {
        v4u o;
        if constexpr (K == 3) {
          o = median3_cols_out<C>(Wr[(u + 1) % K], Wr[(u + 2) % K], Wr[u % K], g.fix_t0, g.fix_t8);
        } else {
          o = median5_cols_out<C>(Wr[(u + 1) % K], Wr[(u + 2) % K], Wr[(u + 3) % K],
                                  Wr[(u + 4) % K], Wr[u % K], g.fix_t0, g.fix_t8);
        }
        stripe_store<NT>(o, rd, (uint32_t)y * row_stride + (uint32_t)g.q, g.kind);
      }
    }
  }
}

// ---- 5x5, 24-byte lanes (C = 3) -----------------------------------------------------------------
// Lane l of a wave holds row bytes [S - 12 + 24 l, +24) of its segment (S = the segment's first
// output byte): 8 whole pixels, since 24 is a multiple of both 3 and 4 -- every lane sees the
// same channel layout, which the 16-byte lanes above cannot (16 = 1 mod 3: their same-channel
// chains cover 20 byte positions for 16 outputs).  Per channel the lane pairs pixel p with pixel
// p + 4 in one u16x2 dword, so ONE chain of 4 medians (median_cols.hpp, 174 instructions, 43.5 per
// output against 51 for the chain of 5) yields all 8 of its pixels, and the three chains cover
// the lane's 24 bytes with nothing computed twice.  The chains' halo columns (pixels -2, -1, 8, 9)
// are the neighbouring lanes' sorted columns, one DPP move + one v_alignbyte each.  Lanes 0 and 63
// store one half (their other half is the halo): 1512 output bytes per wave.  Row starts rebuild
// the lead lane's left half from pixel 0 and the row end always falls on a lane's half boundary
// (rows are multiples of 24 bytes: stripe_ok), whose right half then repeats the last pixel
// (BORDER_REPLICATE); lanes past the row end feed only outputs that are never stored.
constexpr int M24_SEG = 63 * 24;

__device__ __forceinline__ void m24_unpack(const v3u& A, const v3u& B, uint32_t (&P)[12]) {
  const uint32_t a[3] = {A.x, A.y, A.z}, b[3] = {B.x, B.y, B.z};
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      // pair (pixel p, pixel p + 4) of channel c: byte 3p + c of the left and of the right half,
      // as float16 1024 + v lanes (see unpack_row_f16)
      const int by = 3 * p + c, k = by >> 2, j = by & 3;
      const uint32_t sel = (uint32_t)j | 0x0Cu << 8 | (uint32_t)(4 + j) << 16 | 0x0Cu << 24;
      P[4 * c + p] = __builtin_amdgcn_perm(b[k], a[k], sel) | 0x64006400u;
    }
}

// the lane's 24 output bytes from its sorted window columns S[rank][column]
__device__ __forceinline__ void m24_select(const uint32_t (&S)[5][12], v3u& outA, v3u& outB) {
  const PkOps op;
  uint32_t o[3][4];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    uint32_t x[8][5];  // columns p' = -2 .. 5 of channel c: (pixel p', pixel p' + 4)
#pragma unroll
    for (int r = 0; r < 5; ++r) {
#pragma unroll
      for (int p = 0; p < 4; ++p) x[p + 2][r] = S[r][4 * c + p];
      // (prev lane's pixel 6 / 7, own pixel 2 / 3) and (own pixel 4 / 5, next lane's pixel 8 / 9)
      x[0][r] = __builtin_amdgcn_alignbyte(S[r][4 * c + 2], from_prev_lane(S[r][4 * c + 2]), 2);
      x[1][r] = __builtin_amdgcn_alignbyte(S[r][4 * c + 3], from_prev_lane(S[r][4 * c + 3]), 2);
      x[6][r] = __builtin_amdgcn_alignbyte(from_next_lane(S[r][4 * c + 0]), S[r][4 * c + 0], 2);
      x[7][r] = __builtin_amdgcn_alignbyte(from_next_lane(S[r][4 * c + 1]), S[r][4 * c + 1], 2);
    }
    median25_chain4(x, o[c], op);
  }
  // byte 3p + c of the left half = low byte of o[c][p], of the right half = its third byte
  uint32_t A[3], B[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    uint32_t src[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int by = 4 * k + j;
      src[j] = o[by % 3][by / 3];
    }
    const uint32_t u1 = __builtin_amdgcn_perm(src[1], src[0], 0x06020400u);
    const uint32_t u2 = __builtin_amdgcn_perm(src[3], src[2], 0x06020400u);
    A[k] = __builtin_amdgcn_perm(u2, u1, 0x05040100u);
    B[k] = __builtin_amdgcn_perm(u2, u1, 0x07060302u);
  }
  outA = v3u{A[0], A[1], A[2]};
  outB = v3u{B[0], B[1], B[2]};
}

// one output row of 24 bytes per lane from the 5 unpacked rows of its window (oldest first)
__device__ __forceinline__ void m24_row(const uint32_t (&R0)[12], const uint32_t (&R1)[12],
                                        const uint32_t (&R2)[12], const uint32_t (&R3)[12],
                                        const uint32_t (&R4)[12], v3u& outA, v3u& outB) {
  const PkOps op;
  uint32_t S[5][12];  // [rank][column]
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint32_t v[5] = {R0[i], R1[i], R2[i], R3[i], R4[i]};
    sort5(v, op);
#pragma unroll
    for (int r = 0; r < 5; ++r) S[r][i] = v[r];
  }
  m24_select(S, outA, outB);
}

// two vertically adjacent output rows: their windows share 4 rows (C1..C4), sorted once per
// column (5 comparators); each output then inserts its own fifth row (Xa: the row above, Xb: the
// row below) into the sorted 4: rank i = max(c[i-1], min(x, c[i])), 8 min/max.  26 min/max per
// column for the two rows instead of 2 x 18.
__device__ __forceinline__ void m24_pair(const uint32_t (&Xa)[12], const uint32_t (&C1)[12],
                                         const uint32_t (&C2)[12], const uint32_t (&C3)[12],
                                         const uint32_t (&C4)[12], const uint32_t (&Xb)[12],
                                         v3u& oA0, v3u& oB0, v3u& oA1, v3u& oB1) {
  const PkOps op;
  uint32_t c[4][12];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint32_t a = C1[i], b = C2[i], d = C3[i], e = C4[i], t;
    t = op.mn(a, b); b = op.mx(a, b); a = t;   // (0, 1)
    t = op.mn(d, e); e = op.mx(d, e); d = t;   // (2, 3)
    t = op.mn(a, d); d = op.mx(a, d); a = t;   // (0, 2)
    t = op.mn(b, e); e = op.mx(b, e); b = t;   // (1, 3)
    t = op.mn(b, d); d = op.mx(b, d); b = t;   // (1, 2)
    c[0][i] = a;
    c[1][i] = b;
    c[2][i] = d;
    c[3][i] = e;
  }
  uint32_t S[5][12];
  auto insert = [&](const uint32_t (&X)[12]) {
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const uint32_t x = X[i];
      S[0][i] = op.mn(x, c[0][i]);
      S[1][i] = op.mx(c[0][i], op.mn(x, c[1][i]));
      S[2][i] = op.mx(c[1][i], op.mn(x, c[2][i]));
      S[3][i] = op.mx(c[2][i], op.mn(x, c[3][i]));
      S[4][i] = op.mx(x, c[3][i]);
    }
  };
  insert(Xa);
  m24_select(S, oA0, oB0);
  insert(Xb);
  m24_select(S, oA1, oB1);
}

__global__ __launch_bounds__(256) void median5_u8_w24(const uint8_t* __restrict__ src,
                                                      uint8_t* __restrict__ dst, int h, int rb,
                                                      uint32_t row_stride, int nseg, int bands,
                                                      int band_rows, int total_items) {
  constexpr int K = 5, R = 2, PF = K, U = K;
  const int lane = threadIdx.x & 63;
  const int item = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (item >= total_items) return;
  const int seg = item % nseg, tq = item / nseg;
  const int band = tq % bands, img = tq / bands;
  const int seg_start = seg * M24_SEG, seg_end = min(seg_start + M24_SEG, rb);
  const int q = seg_start - 12 + 24 * lane;
  const bool lead = q < 0;              // segment 0, lane 0: left half before the row
  const bool tail = q + 12 == rb;       // the row ends between this lane's halves
  const uint32_t img_bytes = (uint32_t)h * row_stride;
  const rsrc_t rs = make_rsrc(src + (size_t)img * img_bytes, img_bytes);
  const rsrc_t rd = make_rsrc(dst + (size_t)img * img_bytes, img_bytes);
  const uint32_t offA = lead ? OOB_OFF : (uint32_t)q, offB = (uint32_t)(q + 12);
  // stores: a half whose 12 bytes lie in [seg_start, seg_end) (segment and row bounds are
  // multiples of 12)
  const uint32_t stA = (q >= seg_start && q + 12 <= seg_end) ? (uint32_t)q : OOB_OFF;
  const uint32_t stB = (q + 12 >= seg_start && q + 24 <= seg_end) ? (uint32_t)(q + 12) : OOB_OFF;

  const int y0 = band * band_rows;
  const int y1 = min(y0 + band_rows, h);
  if (y0 >= y1) return;
  const int nin = (y1 - y0) + 2 * R;
  const int ngroups = (nin + U - 1) / U;
  auto load_row = [&](int r, v3u& A, v3u& B) {
    const uint32_t ro = (uint32_t)clampi(y0 - R + min(r, nin - 1), 0, h - 1) * row_stride;
    A = __builtin_amdgcn_raw_buffer_load_b96(rs, offA, ro, 0);
    B = __builtin_amdgcn_raw_buffer_load_b96(rs, offB, ro, 0);
  };
  v3u LA[PF], LB[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) load_row(i, LA[i], LB[i]);
  uint32_t Wr[K][12];
  for (int gi = 0; gi < ngroups; ++gi) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = gi * U + u;
      v3u A = LA[u % PF], B = LB[u % PF];
      load_row(r + PF, LA[u % PF], LB[u % PF]);
      if (lead) {  // pixels -4 .. -1 := pixel 0 (bytes 0..2 of the right half)
        A = v3u{__builtin_amdgcn_perm(0u, B.x, 0x00020100u), __builtin_amdgcn_perm(0u, B.x, 0x01000201u),
                __builtin_amdgcn_perm(0u, B.x, 0x02010002u)};
      }
      if (tail) {  // pixels 4..7 := pixel 3 (bytes 9..11 of the left half)
        B = v3u{__builtin_amdgcn_perm(0u, A.z, 0x01030201u), __builtin_amdgcn_perm(0u, A.z, 0x02010302u),
                __builtin_amdgcn_perm(0u, A.z, 0x03020103u)};
      }
      m24_unpack(A, B, Wr[u % K]);
      const int y = y0 + r - 2 * R;
      if (r >= 2 * R && y < y1) {
        v3u oA, oB;
        m24_row(Wr[(u + 1) % K], Wr[(u + 2) % K], Wr[(u + 3) % K], Wr[(u + 4) % K], Wr[u % K], oA, oB);
        const uint32_t ro = (uint32_t)y * row_stride;
        __builtin_amdgcn_raw_buffer_store_b96(oA, rd, stA, ro, 0);
        __builtin_amdgcn_raw_buffer_store_b96(oB, rd, stB, ro, 0);
      }
    }
  }
}

// the 24-byte-lane 5x5 median two output rows at a time (m24_pair): a six-row ring, rows taken in
// pairs; three pairs per unrolled group keep every ring slot a compile-time index
__global__ __launch_bounds__(256) void median5_u8_w24p(const uint8_t* __restrict__ src,
                                                       uint8_t* __restrict__ dst, int h, int rb,
                                                       uint32_t row_stride, int nseg, int bands,
                                                       int band_rows, int total_items) {
  // prefetch one pair ahead: a pair's ~1800 VALU hide the loads, and 2 waves per SIMD (<= 256
  // VGPRs) need the registers
  constexpr int R = 2, PF = 2;
  const int lane = threadIdx.x & 63;
  const int item = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (item >= total_items) return;
  const int seg = item % nseg, tq = item / nseg;
  const int band = tq % bands, img = tq / bands;
  const int seg_start = seg * M24_SEG, seg_end = min(seg_start + M24_SEG, rb);
  const int q = seg_start - 12 + 24 * lane;
  const bool lead = q < 0, tail = q + 12 == rb;
  const uint32_t img_bytes = (uint32_t)h * row_stride;
  const rsrc_t rs = make_rsrc(src + (size_t)img * img_bytes, img_bytes);
  const rsrc_t rd = make_rsrc(dst + (size_t)img * img_bytes, img_bytes);
  const uint32_t offA = lead ? OOB_OFF : (uint32_t)q, offB = (uint32_t)(q + 12);
  const uint32_t stA = (q >= seg_start && q + 12 <= seg_end) ? (uint32_t)q : OOB_OFF;
  const uint32_t stB = (q + 12 >= seg_start && q + 24 <= seg_end) ? (uint32_t)(q + 12) : OOB_OFF;

  const int y0 = band * band_rows;
  const int y1 = min(y0 + band_rows, h);
  if (y0 >= y1) return;
  const int nin = (y1 - y0) + 2 * R;
  auto load_row = [&](int r, v3u& A, v3u& B) {
    const uint32_t ro = (uint32_t)clampi(y0 - R + min(r, nin - 1), 0, h - 1) * row_stride;
    A = __builtin_amdgcn_raw_buffer_load_b96(rs, offA, ro, 0);
    B = __builtin_amdgcn_raw_buffer_load_b96(rs, offB, ro, 0);
  };
  v3u LA[PF], LB[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) load_row(i, LA[i], LB[i]);
  uint32_t Wr[6][12];
  auto take = [&](int r, int slot) {  // slot == r % 6; the load queue slot is r % 2
    v3u A = LA[slot & 1], B = LB[slot & 1];
    load_row(r + PF, LA[slot & 1], LB[slot & 1]);
    if (lead)
      A = v3u{__builtin_amdgcn_perm(0u, B.x, 0x00020100u), __builtin_amdgcn_perm(0u, B.x, 0x01000201u),
              __builtin_amdgcn_perm(0u, B.x, 0x02010002u)};
    if (tail)
      B = v3u{__builtin_amdgcn_perm(0u, A.z, 0x01030201u), __builtin_amdgcn_perm(0u, A.z, 0x02010302u),
              __builtin_amdgcn_perm(0u, A.z, 0x03020103u)};
    m24_unpack(A, B, Wr[slot]);
  };
#pragma unroll
  for (int r = 0; r < 4; ++r) take(r, r);
  const int npairs = (y1 - y0 + 1) / 2;
  for (int j0 = 0; j0 < npairs; j0 += 3) {
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      const int j = j0 + jj;
      if (j >= npairs) break;  // wave-uniform
      // pair j: outputs y0 + 2j (input rows 2j .. 2j+4) and y0 + 2j + 1 (2j+1 .. 2j+5)
      const int ra = 4 + 2 * j;
      take(ra, (4 + 2 * jj) % 6);
      take(ra + 1, (5 + 2 * jj) % 6);
      v3u oA0, oB0, oA1, oB1;
      m24_pair(Wr[(2 * jj) % 6], Wr[(2 * jj + 1) % 6], Wr[(2 * jj + 2) % 6], Wr[(2 * jj + 3) % 6],
               Wr[(4 + 2 * jj) % 6], Wr[(5 + 2 * jj) % 6], oA0, oB0, oA1, oB1);
      const int ya = y0 + 2 * j;
      const uint32_t ro0 = (uint32_t)ya * row_stride;
      __builtin_amdgcn_raw_buffer_store_b96(oA0, rd, stA, ro0, 0);
      __builtin_amdgcn_raw_buffer_store_b96(oB0, rd, stB, ro0, 0);
      const uint32_t ro1 = ya + 1 < y1 ? ro0 + row_stride : OOB_OFF;
      __builtin_amdgcn_raw_buffer_store_b96(oA1, rd, stA, ro1, 0);
      __builtin_amdgcn_raw_buffer_store_b96(oB1, rd, stB, ro1, 0);
    }
  }
}

// generic path: one thread per pixel, exact median by counting (any C, any alignment)
template <int K>
__global__ __launch_bounds__(256) void median_u8_generic(const uint8_t* __restrict__ src,
                                                         uint8_t* __restrict__ dst, int n, int h,
                                                         int w, int c, int64_t row_stride) {
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
      uint8_t v[K * K];
#pragma unroll
      for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j)
          v[i * K + j] = s[(int64_t)clampi(y + i - R, 0, h - 1) * row_stride +
                           (int64_t)clampi(x + j - R, 0, w - 1) * c + ch];
      // rank selection: the median is the value with < K*K/2+1 smaller and >= ... elements
      uint8_t med = 0;
#pragma unroll
      for (int a = 0; a < K * K; ++a) {
        int lt = 0, le = 0;
#pragma unroll
        for (int b = 0; b < K * K; ++b) {
          lt += v[b] < v[a];
          le += v[b] <= v[a];
        }
        if (lt <= (K * K) / 2 && le > (K * K) / 2) med = v[a];
      }
      d[ch] = med;
    }
  }
}

template <int K>
static int launch_median(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                         int64_t row_stride, hipStream_t st) {
  const int64_t rb = (int64_t)w * c;
  // (an LDS band-tile form like the stencils' was bit-exact but measured no faster for 3x3 and
  // 4-6 % slower for 5x5 in steady state, profiles/r02/median_tile/; removed in round 3)
  if (K == 5 && knob("IDN_MEDIAN_W24", 1) && c == 3 && rb % 24 == 0 &&
      stripe_ok(c, rb, row_stride, h, src, dst)) {
    // 24-byte lanes: independent waves over bands of IDN_MEDIAN_ROWS rows
    const int nseg = (int)((rb + M24_SEG - 1) / M24_SEG);
    const int band_rows = std::max(1, std::min(h, knob("IDN_MEDIAN_ROWS", 32)));
    const int bands = (h + band_rows - 1) / band_rows;
    const int64_t total = (int64_t)n * bands * nseg;
    IDN_CHECK_ARG(total < (int64_t)0x7FFFFFFF, "idn_median_blur_u8: batch too large");
    if (knob("IDN_MEDIAN_PAIR", 1))
      hipLaunchKernelGGL(median5_u8_w24p, dim3((unsigned)((total + 3) / 4)), dim3(256), 0, st, src,
                         dst, h, (int)rb, (uint32_t)row_stride, nseg, bands, band_rows, (int)total);
    else
      hipLaunchKernelGGL(median5_u8_w24, dim3((unsigned)((total + 3) / 4)), dim3(256), 0, st, src,
                         dst, h, (int)rb, (uint32_t)row_stride, nseg, bands, band_rows, (int)total);
  } else if (stripe_ok(c, rb, row_stride, h, src, dst)) {
    // measured (tools/sweep_stencil.py): 3x3 is near the memory side -> whole-row workgroups over
    // 16-row bands with XCD-contiguous band order; 5x5 is VALU-bound -> independent waves
    const StripePlan p = plan_stripe(n, h, rb, K, K, 4096, knob("IDN_MEDIAN_MAP", K == 3 ? 1 : 0),
                                     knob("IDN_MEDIAN_ROWS", K == 3 ? 16 : 32));
    IDN_CHECK_ARG(p.total < (int64_t)0x7FFFFFFF, "idn_median_blur_u8: batch too large");
    hipLaunchKernelGGL((median_u8_fast<3, K, 0>), dim3(p.grid), dim3(p.block), 0, st, src, dst, h,
                       (int)rb, (uint32_t)row_stride, p.nseg, p.seg_len, p.bands, p.band_rows,
                       (int)p.total, p.map);
  } else {
    const int64_t npix = (int64_t)n * h * w;
    int64_t blocks = (npix + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL((median_u8_generic<K>), dim3((unsigned)blocks), dim3(256), 0, st, src, dst,
                       n, h, w, c, row_stride);
  }
  IDN_CHECK_LAUNCH("idn_median_blur_u8");
  return IDN_OK;
}

}  // namespace idn

extern "C" int idn_median_blur_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                                  int64_t row_stride, int ksize, void* stream) {
  using namespace idn;
  if (int e = check_filter_args(src, dst, n, h, w, c, row_stride, "idn_median_blur_u8")) return e;
  if (n == 0) return IDN_OK;
  if (ksize == 3) return launch_median<3>(src, dst, n, h, w, c, row_stride, as_stream(stream));
  if (ksize == 5) return launch_median<5>(src, dst, n, h, w, c, row_stride, as_stream(stream));
  return set_error(IDN_EUNSUPPORTED, "idn_median_blur_u8: ksize %d not supported (3 or 5)", ksize);
}
