// Baseline JPEG decode front-end: cv2.imread(path) (IMREAD_COLOR, BGR u8) for the reference's
// images (lib/model/test.py:191, lib/roi_data_layer/minibatch.py:85), decoded on the GPU.
//
// Output = what libjpeg(-turbo) with its defaults produces (the decoder behind both cv2.imread and
// PIL): the ISLOW integer IDCT (jidctint.c), "fancy" triangular chroma upsampling for 4:2:0 / 4:2:2
// (jdsample.c h2v2 / h2v1), the integer YCbCr -> RGB tables (jdcolor.c), all restated here from
// the published algorithms; tests check bit-exactness against PIL's decode.
//
// Host: the marker parser (SOI .. SOS, DQT / DHT / SOF0 / DRI / APPn), Huffman lookup tables per
// image, one packed host->device copy of the images' entropy-coded segments and tables.
// Device, three launches per batch:
//   1 jpeg_huff_kernel   one wave per image; lane r decodes restart interval r, r + 64, ... (lane 0
//                        decodes the whole scan when the image has no restart markers): Huffman +
//                        byte unstuffing + DC prediction into int16 coefficient blocks (natural order)
//   2 jpeg_idct_kernel   one thread per 8x8 block: dequantise + ISLOW IDCT into u8 component planes
//   3 jpeg_color_kernel  one thread per output pixel: chroma upsampling + YCbCr -> BGR (or gray ->
//                        BGR), written into the caller's NHWC batch
// Supported: 8-bit baseline sequential (SOF0/SOF1) Huffman, one interleaved scan, 1 or 3
// components, sampling 4:4:4 / 4:2:2 (h2v1) / 4:2:0 (h2v2), optional restart intervals.  Anything
// else (progressive, arithmetic, 12-bit, CMYK, multi-scan) is IDN_EUNSUPPORTED.
#include "idn_common.hpp"

#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

namespace idn {

constexpr int JPG_LUTB = 9;  // fast Huffman lookup bits

struct JpegDev {
  uint64_t scan_off;   // entropy-coded bytes in the batch buffer
  uint32_t scan_len;
  int width, height, ncomp, mcux, mcuy, restart;  // restart: MCUs per interval (0: none)
  int hmax, vmax, nintervals;
  int ch[3], cv[3], tq[3], td[3], ta[3];
  int bw[3], bh[3];         // blocks per row / column of each component plane (MCU-padded)
  int dw[3], dh[3];         // downsampled component size (libjpeg downsampled_width / _height)
  uint64_t blk_off[3];      // first block of each component in the batch coefficient buffer
  uint64_t pl_off[3];       // component plane byte offset in the batch plane buffer
  uint16_t q[4][64];        // quantisation tables, natural order
  uint16_t lut[4][1 << JPG_LUTB];  // [DC0, DC1, AC0, AC1]: len << 8 | symbol, 0 = longer code
  int32_t maxcode[4][18];   // libjpeg jdhuff: largest code of each length (-1: none), [17] sentinel
  int32_t valoff[4][18];    // huffval index of the first code of each length, minus that code
  uint8_t huffval[4][256];
};

// jpeg_natural_order: zigzag index -> natural (row-major) index
__constant__ uint8_t jpg_natural[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};  // overrun guard (libjpeg)
static const uint8_t jpg_natural_host[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// ---- host: marker parser ---------------------------------------------------------------------
struct HuffSpec {
  bool present = false;
  uint8_t bits[17] = {};
  uint8_t val[256] = {};
};
struct JpegHost {
  int width = 0, height = 0, ncomp = 0, restart = 0;
  int cid[3] = {}, ch[3] = {}, cv[3] = {}, tq[3] = {}, td[3] = {}, ta[3] = {};
  bool qpresent[4] = {};
  uint16_t q[4][64] = {};  // natural order
  HuffSpec dc[4], ac[4];
  size_t scan_begin = 0, scan_end = 0;
  bool adobe_rgb = false;
};

static int jpg_fail(std::string* err, const char* msg) {
  if (err) *err = msg;
  return IDN_EUNSUPPORTED;
}

static int jpeg_parse(const uint8_t* p, size_t n, JpegHost& J, std::string* err) {
  if (n < 4 || p[0] != 0xFF || p[1] != 0xD8) return jpg_fail(err, "not a JPEG (no SOI)");
  size_t i = 2;
  bool sof = false;
  while (i + 4 <= n) {
    if (p[i] != 0xFF) return jpg_fail(err, "corrupt marker stream");
    uint8_t m = p[i + 1];
    if (m == 0xFF) {  // fill byte
      ++i;
      continue;
    }
    i += 2;
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;  // no length
    if (m == 0xD9) return jpg_fail(err, "EOI before SOS");
    const size_t len = ((size_t)p[i] << 8) | p[i + 1];
    if (len < 2 || i + len > n) return jpg_fail(err, "truncated segment");
    const uint8_t* s = p + i + 2;
    const size_t sl = len - 2;
    switch (m) {
      case 0xC0:
      case 0xC1: {  // SOF0 / SOF1: baseline / extended sequential Huffman
        if (sl < 6 || s[0] != 8) return jpg_fail(err, "only 8-bit sequential JPEG");
        J.height = (s[1] << 8) | s[2];
        J.width = (s[3] << 8) | s[4];
        J.ncomp = s[5];
        if (J.ncomp != 1 && J.ncomp != 3) return jpg_fail(err, "only 1 or 3 components");
        if (sl < 6 + 3 * (size_t)J.ncomp || J.width <= 0 || J.height <= 0)
          return jpg_fail(err, "bad SOF");
        for (int c = 0; c < J.ncomp; ++c) {
          J.cid[c] = s[6 + 3 * c];
          J.ch[c] = s[7 + 3 * c] >> 4;
          J.cv[c] = s[7 + 3 * c] & 15;
          J.tq[c] = s[8 + 3 * c];
          if (J.ch[c] < 1 || J.cv[c] < 1 || J.tq[c] > 3) return jpg_fail(err, "bad component");
        }
        sof = true;
        break;
      }
      case 0xC2: case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB:
      case 0xCD: case 0xCE: case 0xCF:
        return jpg_fail(err, "progressive / lossless / arithmetic JPEG not supported");
      case 0xC4: {  // DHT
        size_t k = 0;
        while (k < sl) {
          if (k + 17 > sl) return jpg_fail(err, "bad DHT");
          const int tc = s[k] >> 4, th = s[k] & 15;
          if (tc > 1 || th > 3) return jpg_fail(err, "bad DHT class");
          HuffSpec& H = tc ? J.ac[th] : J.dc[th];
          int tot = 0;
          for (int l = 1; l <= 16; ++l) {
            H.bits[l] = s[k + l];
            tot += H.bits[l];
          }
          if (tot > 256 || k + 17 + tot > sl) return jpg_fail(err, "bad DHT counts");
          memcpy(H.val, s + k + 17, tot);
          H.present = true;
          k += 17 + tot;
        }
        break;
      }
      case 0xDB: {  // DQT
        size_t k = 0;
        while (k < sl) {
          const int pq = s[k] >> 4, tq = s[k] & 15;
          if (tq > 3) return jpg_fail(err, "bad DQT");
          const size_t need = 1 + 64 * (pq ? 2 : 1);
          if (k + need > sl) return jpg_fail(err, "truncated DQT");
          for (int z = 0; z < 64; ++z)
            J.q[tq][jpg_natural_host[z]] =
                pq ? (uint16_t)((s[k + 1 + 2 * z] << 8) | s[k + 2 + 2 * z]) : s[k + 1 + z];
          J.qpresent[tq] = true;
          k += need;
        }
        break;
      }
      case 0xDD:  // DRI
        if (sl < 2) return jpg_fail(err, "bad DRI");
        J.restart = (s[0] << 8) | s[1];
        break;
      case 0xEE:  // APP14 Adobe: transform 0 = RGB / CMYK stored as-is
        if (sl >= 12 && memcmp(s, "Adobe", 5) == 0 && s[11] == 0) J.adobe_rgb = true;
        break;
      case 0xDA: {  // SOS
        if (!sof) return jpg_fail(err, "SOS before SOF");
        const int ns = s[0];
        if (ns != J.ncomp) return jpg_fail(err, "multi-scan (non-interleaved) JPEG not supported");
        if (sl < 1 + 2 * (size_t)ns + 3) return jpg_fail(err, "bad SOS");
        for (int k = 0; k < ns; ++k) {
          int c = 0;
          while (c < J.ncomp && J.cid[c] != s[1 + 2 * k]) ++c;
          if (c != k) return jpg_fail(err, "scan component order differs from the frame");
          J.td[c] = s[2 + 2 * k] >> 4;
          J.ta[c] = s[2 + 2 * k] & 15;
          if (J.td[c] > 3 || J.ta[c] > 3) return jpg_fail(err, "bad SOS table");
        }
        const uint8_t* ss = s + 1 + 2 * ns;
        if (ss[0] != 0 || ss[1] != 63 || ss[2] != 0) return jpg_fail(err, "not a sequential scan");
        J.scan_begin = i + len;
        // entropy-coded segment: up to the EOI (scanning back from the end) or the end of data
        size_t e = n;
        while (e >= J.scan_begin + 2 && !(p[e - 2] == 0xFF && p[e - 1] == 0xD9)) --e;
        J.scan_end = (e >= J.scan_begin + 2) ? e - 2 : n;
        for (int c = 0; c < J.ncomp; ++c)
          if (!J.qpresent[J.tq[c]] || !J.dc[J.td[c]].present || !J.ac[J.ta[c]].present)
            return jpg_fail(err, "missing quantisation / Huffman table");
        if (J.adobe_rgb) return jpg_fail(err, "Adobe RGB / CMYK JPEG not supported");
        if (J.ncomp == 3) {
          const bool s444 = J.ch[0] == 1 && J.cv[0] == 1;
          const bool s422 = J.ch[0] == 2 && J.cv[0] == 1;
          const bool s420 = J.ch[0] == 2 && J.cv[0] == 2;
          if (!(s444 || s422 || s420) || J.ch[1] != 1 || J.cv[1] != 1 || J.ch[2] != 1 || J.cv[2] != 1)
            return jpg_fail(err, "chroma sampling other than 4:4:4 / 4:2:2 / 4:2:0");
        }
        return IDN_OK;
      }
      default:
        if (m < 0xC0) return jpg_fail(err, "corrupt marker");
        break;  // APPn, COM, ...: skip
    }
    i += len;
  }
  return jpg_fail(err, "no SOS");
}

// jdhuff.c jpeg_make_d_derived_tbl: canonical codes -> fast lookup + maxcode / valoffset
static int jpeg_build_huff(const HuffSpec& H, bool dc, uint16_t* lut, int32_t* maxcode,
                           int32_t* valoff, uint8_t* huffval, std::string* err) {
  int code = 0, k = 0;
  memset(lut, 0, sizeof(uint16_t) << JPG_LUTB);
  for (int l = 1; l <= 16; ++l) {
    if (H.bits[l]) {
      valoff[l] = k - code;
      for (int t = 0; t < H.bits[l]; ++t, ++k, ++code) {
        if (l <= JPG_LUTB) {
          const int lo = code << (JPG_LUTB - l), hi = (code + 1) << (JPG_LUTB - l);
          for (int x = lo; x < hi; ++x) lut[x] = (uint16_t)(l << 8 | H.val[k]);
        }
      }
      maxcode[l] = code - 1;
    } else {
      valoff[l] = 0;
      maxcode[l] = -1;
    }
    if (code > (1 << l)) return jpg_fail(err, "bad Huffman table");
    code <<= 1;
  }
  maxcode[0] = -1;
  maxcode[17] = 0x7FFFFFFF;  // sentinel: a corrupt stream stops at length 17
  valoff[0] = valoff[17] = 0;
  memcpy(huffval, H.val, 256);
  if (dc)
    for (int t = 0; t < k; ++t)
      if (H.val[t] > 15) return jpg_fail(err, "bad DC Huffman value");
  return IDN_OK;
}

// ---- device: entropy decoding -----------------------------------------------------------------
struct BitReader {
  const uint8_t* p;
  uint32_t pos, end;
  uint64_t acc;  // left-aligned
  int nb;
  bool marker;   // hit a marker: feed zero bits (libjpeg does the same)
  __device__ __forceinline__ void fill() {
    while (nb <= 56) {
      uint32_t b = 0;
      if (!marker && pos < end) {
        b = p[pos];
        if (b == 0xFF) {
          const uint32_t b2 = pos + 1 < end ? p[pos + 1] : 0xD9u;
          if (b2 == 0x00) {
            pos += 2;
          } else {
            marker = true;  // pos stays on the 0xFF
            b = 0;
          }
        } else {
          ++pos;
        }
      }
      acc |= (uint64_t)b << (56 - nb);
      nb += 8;
    }
  }
  __device__ __forceinline__ uint32_t bits(int s) {  // s <= 16, nb >= s
    const uint32_t r = (uint32_t)(acc >> (64 - s));
    acc <<= s;
    nb -= s;
    return r;
  }
};

__device__ __forceinline__ int jpg_extend(uint32_t v, int s) {  // HUFF_EXTEND
  return (int)v < (1 << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v;
}

// one Huffman symbol (nb >= 16 on entry)
__device__ __forceinline__ int jpg_decode(BitReader& br, const uint16_t* __restrict__ lut,
                                          const int32_t* __restrict__ maxcode,
                                          const int32_t* __restrict__ valoff,
                                          const uint8_t* __restrict__ huffval) {
  const uint32_t e = lut[br.acc >> (64 - JPG_LUTB)];
  if (e) {
    br.acc <<= e >> 8;
    br.nb -= e >> 8;
    return e & 0xFF;
  }
  int l = JPG_LUTB + 1;
  int32_t code = (int32_t)(br.acc >> (64 - l));
  while (code > maxcode[l]) {
    ++l;
    code = (int32_t)(br.acc >> (64 - l));
  }
  if (l > 16) {  // corrupt data: libjpeg warns and returns 0
    br.acc <<= 16;
    br.nb -= 16;
    return 0;
  }
  br.acc <<= l;
  br.nb -= l;
  return huffval[(valoff[l] + code) & 0xFF];
}

struct JpegLds {
  uint16_t lut[4][1 << JPG_LUTB];
  int32_t maxcode[4][18], valoff[4][18];
  uint8_t huffval[4][256];
};

__global__ __launch_bounds__(64) void jpeg_huff_kernel(const JpegDev* __restrict__ imgs,
                                                       const uint8_t* __restrict__ scans,
                                                       int16_t* __restrict__ coef) {
  __shared__ JpegLds T;
  const JpegDev& D = imgs[blockIdx.x];
  {  // tables into LDS
    const uint32_t* s = reinterpret_cast<const uint32_t*>(&D.lut[0][0]);
    uint32_t* d = reinterpret_cast<uint32_t*>(&T.lut[0][0]);
    for (int k = threadIdx.x; k < (int)(sizeof(T.lut) / 4); k += 64) d[k] = s[k];
    for (int k = threadIdx.x; k < 4 * 18; k += 64) {
      (&T.maxcode[0][0])[k] = (&D.maxcode[0][0])[k];
      (&T.valoff[0][0])[k] = (&D.valoff[0][0])[k];
    }
    for (int k = threadIdx.x; k < 4 * 256; k += 64) (&T.huffval[0][0])[k] = (&D.huffval[0][0])[k];
  }
  __syncthreads();
  const int nint = D.nintervals;
  const int mcus = D.mcux * D.mcuy;
  const int per = D.restart ? D.restart : mcus;
  for (int iv = threadIdx.x; iv < nint; iv += 64) {
    // the interval's first byte: lane 0 starts at the scan start; other intervals start right
    // after their RST marker (found by a forward scan: a marker is 0xFF followed by 0xD0-0xD7)
    BitReader br;
    br.p = scans + D.scan_off;
    br.end = D.scan_len;
    br.pos = 0;
    if (iv > 0) {
      int seen = 0;
      uint32_t q = 0;
      while (q + 1 < br.end) {
        if (br.p[q] == 0xFF && br.p[q + 1] >= 0xD0 && br.p[q + 1] <= 0xD7) {
          if (++seen == iv) {
            q += 2;
            break;
          }
          q += 2;
        } else {
          ++q;
        }
      }
      br.pos = q;
    }
    br.acc = 0;
    br.nb = 0;
    br.marker = false;
    int pred[3] = {0, 0, 0};
    const int m0 = iv * per, m1 = min(m0 + per, mcus);
    for (int m = m0; m < m1; ++m) {
      const int my = m / D.mcux, mx = m - my * D.mcux;
      for (int c = 0; c < D.ncomp; ++c) {
        const int hs = D.ncomp == 1 ? 1 : D.ch[c], vs = D.ncomp == 1 ? 1 : D.cv[c];
        const int dct = D.td[c], act = 2 + D.ta[c];
        for (int v = 0; v < vs; ++v)
          for (int hh = 0; hh < hs; ++hh) {
            const int by = my * vs + v, bx = mx * hs + hh;
            int16_t* blk = coef + (D.blk_off[c] + (uint64_t)by * D.bw[c] + bx) * 64;
            br.fill();
            int s = jpg_decode(br, T.lut[dct], T.maxcode[dct], T.valoff[dct], T.huffval[dct]);
            int diff = 0;
            if (s) diff = jpg_extend(br.bits(s), s);
            pred[c] += diff;
            blk[0] = (int16_t)pred[c];
            for (int k = 1; k < 64; ++k) {
              br.fill();
              const int rs = jpg_decode(br, T.lut[act], T.maxcode[act], T.valoff[act], T.huffval[act]);
              const int r = rs >> 4;
              s = rs & 15;
              if (s) {
                k += r;
                const int val = jpg_extend(br.bits(s), s);
                if (k < 64) blk[jpg_natural[k]] = (int16_t)val;
              } else {
                if (r != 15) break;  // EOB
                k += 15;
              }
            }
          }
      }
    }
  }
}

// ---- device: ISLOW IDCT (jidctint.c) ------------------------------------------------------------
constexpr int JCB = 13, JP1 = 2;  // CONST_BITS, PASS1_BITS
__device__ __forceinline__ int jpg_descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }
// libjpeg's IDCT range limit: the descaled value's low 10 bits as a signed number, + 128, clamped
__device__ __forceinline__ uint32_t jpg_range(int x) {
  const int v = ((x & 1023) ^ 512) - 512;
  return (uint32_t)min(max(v + 128, 0), 255);
}

template <bool ROW>
__device__ __forceinline__ void jpg_idct1(int i0, int i1, int i2, int i3, int i4, int i5, int i6,
                                          int i7, int (&o)[8]) {
  // even part
  int z2 = i2, z3 = i6;
  int z1 = (z2 + z3) * 4433;  // FIX_0_541196100
  int tmp2 = z1 + z3 * -15137;  // FIX_1_847759065
  int tmp3 = z1 + z2 * 6270;    // FIX_0_765366865
  int tmp0 = (i0 + i4) * (1 << JCB);
  int tmp1 = (i0 - i4) * (1 << JCB);
  const int tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
  // odd part
  tmp0 = i7;
  tmp1 = i5;
  tmp2 = i3;
  tmp3 = i1;
  z1 = tmp0 + tmp3;
  z2 = tmp1 + tmp2;
  z3 = tmp0 + tmp2;
  int z4 = tmp1 + tmp3;
  const int z5 = (z3 + z4) * 9633;  // FIX_1_175875602
  tmp0 *= 2446;                     // FIX_0_298631336
  tmp1 *= 16819;                    // FIX_2_053119869
  tmp2 *= 25172;                    // FIX_3_072711026
  tmp3 *= 12299;                    // FIX_1_501321110
  z1 *= -7373;                      // FIX_0_899976223
  z2 *= -20995;                     // FIX_2_562915447
  z3 *= -16069;                     // FIX_1_961570560
  z4 *= -3196;                      // FIX_0_390180644
  z3 += z5;
  z4 += z5;
  tmp0 += z1 + z3;
  tmp1 += z2 + z4;
  tmp2 += z2 + z3;
  tmp3 += z1 + z4;
  constexpr int SH = ROW ? JCB + JP1 + 3 : JCB - JP1;
  o[0] = jpg_descale(tmp10 + tmp3, SH);
  o[7] = jpg_descale(tmp10 - tmp3, SH);
  o[1] = jpg_descale(tmp11 + tmp2, SH);
  o[6] = jpg_descale(tmp11 - tmp2, SH);
  o[2] = jpg_descale(tmp12 + tmp1, SH);
  o[5] = jpg_descale(tmp12 - tmp1, SH);
  o[3] = jpg_descale(tmp13 + tmp0, SH);
  o[4] = jpg_descale(tmp13 - tmp0, SH);
}

// one thread per block; blocks of all components of all images in one flat index space
__global__ __launch_bounds__(256) void jpeg_idct_kernel(const JpegDev* __restrict__ imgs,
                                                        const uint64_t* __restrict__ blk_end,
                                                        int n, uint64_t nblk,
                                                        const int16_t* __restrict__ coef,
                                                        uint8_t* __restrict__ planes) {
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nblk) return;
  int img = 0;  // the image holding block b (blk_end: exclusive prefix ends per image)
  {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (blk_end[mid] > b) hi = mid;
      else lo = mid + 1;
    }
    img = lo;
  }
  const JpegDev& D = imgs[img];
  int c = D.ncomp - 1;
  while (c > 0 && b < D.blk_off[c]) --c;
  const uint64_t lb = b - D.blk_off[c];
  const int by = (int)(lb / D.bw[c]), bx = (int)(lb - (uint64_t)by * D.bw[c]);
  const uint16_t* q = D.q[D.tq[c]];
  const int16_t* in = coef + b * 64;
  int x[64];
#pragma unroll
  for (int k = 0; k < 8; ++k) {  // 8 x 16-byte loads
    const int4 v = reinterpret_cast<const int4*>(in)[k];
    const int w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[8 * k + 2 * j] = (int)(int16_t)(w4[j] & 0xFFFF) * (int)q[8 * k + 2 * j];
      x[8 * k + 2 * j + 1] = (int)(int16_t)((uint32_t)w4[j] >> 16) * (int)q[8 * k + 2 * j + 1];
    }
  }
  int ws[64];
#pragma unroll
  for (int col = 0; col < 8; ++col) {  // pass 1: columns (the all-zero-AC shortcut is exact)
    int o[8];
    jpg_idct1<false>(x[col], x[8 + col], x[16 + col], x[24 + col], x[32 + col], x[40 + col],
                     x[48 + col], x[56 + col], o);
#pragma unroll
    for (int r = 0; r < 8; ++r) ws[8 * r + col] = o[r];
  }
  uint8_t* out = planes + D.pl_off[c] + (uint64_t)(by * 8) * (D.bw[c] * 8) + bx * 8;
#pragma unroll
  for (int r = 0; r < 8; ++r) {  // pass 2: rows
    int o[8];
    jpg_idct1<true>(ws[8 * r], ws[8 * r + 1], ws[8 * r + 2], ws[8 * r + 3], ws[8 * r + 4],
                    ws[8 * r + 5], ws[8 * r + 6], ws[8 * r + 7], o);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lo |= jpg_range(o[j]) << (8 * j);
      hi |= jpg_range(o[4 + j]) << (8 * j);
    }
    reinterpret_cast<uint2*>(out + (uint64_t)r * (D.bw[c] * 8))[0] = make_uint2(lo, hi);
  }
}

// ---- device: upsampling + colour ---------------------------------------------------------------
// h2v1 / h2v2 "fancy" upsampling (jdsample.c) of chroma plane P (dw x dh real samples, row pitch
// pw) at output (x, y)
template <int V>
__device__ __forceinline__ int jpg_up(const uint8_t* __restrict__ P, int pw, int dw, int dh,
                                      int x, int y) {
  const int col = x >> 1, s = x & 1;
  if (V == 1) {  // h2v1: 3/4 nearer + 1/4 further sample of the row
    const uint8_t* r = P + (int64_t)y * pw;
    const int in = r[col];
    if (s == 0) return col == 0 ? in : (in * 3 + r[col - 1] + 1) >> 2;
    return col == dw - 1 ? in : (in * 3 + r[col + 1] + 2) >> 2;
  }
  // h2v2: column sums 3 * nearer row + further row (rows replicated at the top and bottom)
  const int inrow = y >> 1;
  const int other = min(max((y & 1) ? inrow + 1 : inrow - 1, 0), dh - 1);
  const uint8_t* r0 = P + (int64_t)inrow * pw;
  const uint8_t* r1 = P + (int64_t)other * pw;
  auto cs = [&](int k) { return r0[k] * 3 + r1[k]; };
  const int t = cs(col);
  if (s == 0) return col == 0 ? (t * 4 + 8) >> 4 : (t * 3 + cs(col - 1) + 8) >> 4;
  return col == dw - 1 ? (t * 4 + 7) >> 4 : (t * 3 + cs(col + 1) + 7) >> 4;
}

__device__ __forceinline__ uint32_t jpg_clamp(int v) { return (uint32_t)min(max(v, 0), 255); }

// grid (row tiles, n): one thread per pixel of 256 consecutive pixels of one image
__global__ __launch_bounds__(256) void jpeg_color_kernel(const JpegDev* __restrict__ imgs,
                                                         const uint8_t* __restrict__ planes,
                                                         uint8_t* __restrict__ dst, int h, int w,
                                                         int64_t row_stride) {
  const JpegDev& D = imgs[blockIdx.y];
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= (int64_t)h * w) return;
  const int y = (int)(p / w), x = (int)(p - (int64_t)y * w);
  uint8_t* o = dst + (int64_t)blockIdx.y * h * row_stride + (int64_t)y * row_stride + (int64_t)x * 3;
  const int pw0 = D.bw[0] * 8;
  const int Y = planes[D.pl_off[0] + (int64_t)y * pw0 + x];
  if (D.ncomp == 1) {
    o[0] = o[1] = o[2] = (uint8_t)Y;
    return;
  }
  int cb, cr;
  const int pw1 = D.bw[1] * 8, pw2 = D.bw[2] * 8;
  const uint8_t* P1 = planes + D.pl_off[1];
  const uint8_t* P2 = planes + D.pl_off[2];
  if (D.hmax == 1) {
    cb = P1[(int64_t)y * pw1 + x];
    cr = P2[(int64_t)y * pw2 + x];
  } else if (D.vmax == 1) {
    cb = jpg_up<1>(P1, pw1, D.dw[1], D.dh[1], x, y);
    cr = jpg_up<1>(P2, pw2, D.dw[2], D.dh[2], x, y);
  } else {
    cb = jpg_up<2>(P1, pw1, D.dw[1], D.dh[1], x, y);
    cr = jpg_up<2>(P2, pw2, D.dw[2], D.dh[2], x, y);
  }
  // jdcolor.c build_ycc_rgb_table / ycc_rgb_convert (SCALEBITS 16)
  const int xb = cb - 128, xr = cr - 128;
  const int r = Y + ((91881 * xr + 32768) >> 16);                    // FIX(1.40200)
  const int g = Y + ((-46802 * xr + (-22554 * xb + 32768)) >> 16);   // FIX(0.71414), FIX(0.34414)
  const int b = Y + ((116130 * xb + 32768) >> 16);                   // FIX(1.77200)
  o[0] = (uint8_t)jpg_clamp(b);  // BGR, as cv2.imread
  o[1] = (uint8_t)jpg_clamp(g);
  o[2] = (uint8_t)jpg_clamp(r);
}

// ---- host: batch plan ---------------------------------------------------------------------------
struct JpegPlan {
  std::vector<JpegDev> dev;
  std::vector<uint64_t> blk_end;
  uint64_t scan_bytes = 0, nblk = 0, plane_bytes = 0;
  size_t off_imgs = 0, off_blkend = 0, off_scan = 0, off_coef = 0, off_planes = 0, total = 0;
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static int jpeg_plan(const uint8_t* const* files, const size_t* lens, int n, int h, int w,
                     JpegPlan& P, std::string* err) {
  P.dev.assign(n, JpegDev{});
  P.blk_end.assign(n, 0);
  for (int i = 0; i < n; ++i) {
    JpegHost J;
    if (!files[i]) return jpg_fail(err, "null file pointer");
    int rc = jpeg_parse(files[i], lens[i], J, err);
    if (rc != IDN_OK) return rc;
    if ((h > 0 && J.height != h) || (w > 0 && J.width != w)) {
      if (err) *err = "image size differs from the batch size";
      return IDN_EINVAL;
    }
    JpegDev& D = P.dev[i];
    memset(&D, 0, sizeof(D));
    D.width = J.width;
    D.height = J.height;
    D.ncomp = J.ncomp;
    D.restart = J.restart;
    D.hmax = D.vmax = 1;
    for (int c = 0; c < J.ncomp; ++c) {
      D.hmax = std::max(D.hmax, J.ch[c]);
      D.vmax = std::max(D.vmax, J.cv[c]);
    }
    if (J.ncomp == 1) {  // non-interleaved single component: MCU = one block of the component
      D.hmax = D.vmax = 1;
      D.ch[0] = D.cv[0] = 1;
      D.mcux = (J.width + 7) / 8;
      D.mcuy = (J.height + 7) / 8;
    } else {
      for (int c = 0; c < 3; ++c) {
        D.ch[c] = J.ch[c];
        D.cv[c] = J.cv[c];
      }
      D.mcux = (J.width + 8 * D.hmax - 1) / (8 * D.hmax);
      D.mcuy = (J.height + 8 * D.vmax - 1) / (8 * D.vmax);
    }
    const int mcus = D.mcux * D.mcuy;
    D.nintervals = D.restart ? (mcus + D.restart - 1) / D.restart : 1;
    for (int c = 0; c < J.ncomp; ++c) {
      D.tq[c] = J.tq[c];
      D.td[c] = J.td[c];
      D.ta[c] = J.ta[c];
      D.bw[c] = D.mcux * D.ch[c];
      D.bh[c] = D.mcuy * D.cv[c];
      // libjpeg: downsampled size = ceil(image size * samp / max samp)
      D.dw[c] = (J.width * D.ch[c] + D.hmax - 1) / D.hmax;
      D.dh[c] = (J.height * D.cv[c] + D.vmax - 1) / D.vmax;
      D.blk_off[c] = P.nblk;
      P.nblk += (uint64_t)D.bw[c] * D.bh[c];
      D.pl_off[c] = P.plane_bytes;
      P.plane_bytes += (uint64_t)D.bw[c] * 8 * D.bh[c] * 8;
    }
    P.blk_end[i] = P.nblk;
    for (int t = 0; t < 4; ++t) memcpy(D.q[t], J.q[t], sizeof(D.q[t]));
    for (int t = 0; t < 4; ++t) {
      for (int k = 0; k < 18; ++k) D.maxcode[t][k] = -1;
      const HuffSpec& H = t < 2 ? J.dc[t] : J.ac[t - 2];
      if (!H.present) continue;
      rc = jpeg_build_huff(H, t < 2, D.lut[t], D.maxcode[t], D.valoff[t], D.huffval[t], err);
      if (rc != IDN_OK) return rc;
    }
    D.scan_off = P.scan_bytes;
    D.scan_len = (uint32_t)(J.scan_end - J.scan_begin);
    P.scan_bytes += (D.scan_len + 15) & ~15u;
  }
  P.off_imgs = 0;
  P.off_blkend = align256(P.off_imgs + sizeof(JpegDev) * (size_t)n);
  P.off_scan = align256(P.off_blkend + sizeof(uint64_t) * (size_t)n);
  P.off_coef = align256(P.off_scan + P.scan_bytes + 16);
  P.off_planes = align256(P.off_coef + P.nblk * 128);
  P.total = align256(P.off_planes + P.plane_bytes);
  return IDN_OK;
}

}  // namespace idn

using namespace idn;

extern "C" int idn_jpeg_info(const uint8_t* file, size_t len, int* height, int* width,
                             int* components) {
  IDN_CHECK_ARG(file && height && width && components, "idn_jpeg_info: null pointer");
  JpegHost J;
  std::string err;
  const int rc = jpeg_parse(file, len, J, &err);
  if (rc != IDN_OK) return set_error(rc, "idn_jpeg_info: %s", err.c_str());
  *height = J.height;
  *width = J.width;
  *components = J.ncomp;
  return IDN_OK;
}

extern "C" size_t idn_jpeg_workspace_size(const uint8_t* const* files, const size_t* lens, int n) {
  if (!files || !lens || n <= 0) return 0;
  JpegPlan P;
  if (jpeg_plan(files, lens, n, 0, 0, P, nullptr) != IDN_OK) return 0;
  return P.total;
}

extern "C" int idn_jpeg_decode_u8(const uint8_t* const* files, const size_t* lens, int n,
                                  uint8_t* dst, int h, int w, int64_t row_stride, void* workspace,
                                  size_t ws_bytes, void* stream) {
  IDN_CHECK_ARG(n >= 0 && (n == 0 || (files && lens && dst)), "idn_jpeg_decode_u8: null pointer");
  IDN_CHECK_ARG(h > 0 && w > 0 && row_stride >= (int64_t)w * 3,
                "idn_jpeg_decode_u8: bad output shape");
  IDN_CHECK_ARG(n <= 65535, "idn_jpeg_decode_u8: batch too large");
  if (n == 0) return IDN_OK;
  JpegPlan P;
  std::string err;
  const int rc = jpeg_plan(files, lens, n, h, w, P, &err);
  if (rc != IDN_OK) return set_error(rc, "idn_jpeg_decode_u8: %s", err.c_str());
  if (!workspace || ws_bytes < P.total)
    return set_error(IDN_EWORKSPACE, "idn_jpeg_decode_u8: needs %zu workspace bytes (got %zu)",
                     P.total, ws_bytes);
  hipStream_t st = as_stream(stream);
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  // one host staging buffer -> one copy: per-image descriptors, block ends, entropy segments
  std::vector<uint8_t> host(P.off_coef);
  memcpy(host.data() + P.off_imgs, P.dev.data(), sizeof(JpegDev) * (size_t)n);
  memcpy(host.data() + P.off_blkend, P.blk_end.data(), sizeof(uint64_t) * (size_t)n);
  for (int i = 0; i < n; ++i) {
    JpegHost J;
    jpeg_parse(files[i], lens[i], J, nullptr);
    memcpy(host.data() + P.off_scan + P.dev[i].scan_off, files[i] + J.scan_begin,
           P.dev[i].scan_len);
  }
  if (hipMemcpyAsync(ws, host.data(), host.size(), hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemsetAsync(ws + P.off_coef, 0, P.nblk * 128, st) != hipSuccess)
    return set_error(IDN_EHIP, "idn_jpeg_decode_u8: staging copy failed");
  const JpegDev* dimg = reinterpret_cast<const JpegDev*>(ws + P.off_imgs);
  int16_t* coef = reinterpret_cast<int16_t*>(ws + P.off_coef);
  hipLaunchKernelGGL(jpeg_huff_kernel, dim3(n), dim3(64), 0, st, dimg, ws + P.off_scan, coef);
  const uint64_t gb = (P.nblk + 255) / 256;
  IDN_CHECK_ARG(gb < 0x7FFFFFFF, "idn_jpeg_decode_u8: batch too large");
  hipLaunchKernelGGL(jpeg_idct_kernel, dim3((unsigned)gb), dim3(256), 0, st, dimg,
                     reinterpret_cast<const uint64_t*>(ws + P.off_blkend), n, P.nblk, coef,
                     ws + P.off_planes);
  const int64_t gx = ((int64_t)h * w + 255) / 256;
  hipLaunchKernelGGL(jpeg_color_kernel, dim3((unsigned)gx, (unsigned)n), dim3(256), 0, st, dimg,
                     ws + P.off_planes, dst, h, w, row_stride);
  // the staging buffer must outlive the async copy
  if (hipStreamSynchronize(st) != hipSuccess)
    return set_error(IDN_EHIP, "idn_jpeg_decode_u8: decode failed");
  IDN_CHECK_LAUNCH("idn_jpeg_decode_u8");
  return IDN_OK;
}
