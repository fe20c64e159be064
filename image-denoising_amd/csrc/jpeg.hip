// JPEG decode front-end: cv2.imread(path) (IMREAD_COLOR, BGR u8) for the reference's images
// (lib/model/test.py:191, lib/roi_data_layer/minibatch.py:85), decoded on the GPU.
//
// Output = what the reference's pinned decoder produces with its defaults: IJG libjpeg 9d
// (requirements.txt:74, under OpenCV 3.4.2) -- the ISLOW integer IDCT (jidctint.c) for full-size
// components and, since libjpeg 7, a scaled IDCT for subsampled chroma (jdmaster.c: with fancy
// upsampling a component sampled at half the maximum rate gets jpeg_idct_16x16 (4:2:0) or
// jpeg_idct_16x8 (4:2:2), decoding straight to full resolution, no upsampling pass), then the
// integer YCbCr -> RGB tables of libjpeg 9's jdcolor.c (FIX(0.344136286) for Cb -> G).
// IDN_JPEG_TURBO selects libjpeg-turbo's decode instead (8x8 IDCT everywhere, "fancy" triangular
// h2v1 / h2v2 upsampling from jdsample.c, FIX(0.34414)): what PIL 9+ / turbo-linked OpenCV make.
// All restated from the published algorithms; tests check bit-exactness against the real libjpeg
// 9d decode (committed fixtures) and the GPU box's turbo-linked PIL.
//
// Host: the marker parser (SOI .. SOS: DQT / DHT / DAC / SOFn / DRI / APPn), Huffman lookup tables
// per image and scan, one packed host->device copy of the images' entropy-coded segments.
// Device:
//   unstuff        per 16 KiB tile: the segments without stuffing and markers, every marker's code
//                  and offset; per segment each restart interval's data as libjpeg reads it
//                  (jdmarker.c resync on damaged files)
//   the parallel path: single-scan Huffman files of 1 or 3 components (SOF0 / SOF1)
//     sync A / B   self-synchronising chunk decoders (each restart interval its own chunks) with
//                  checkpoints; B passes until no chunk's end state changes
//     prefix       per image: each chunk's first block and DC predictors
//     write        one thread per 256-bit sub-chunk from the checkpoints: coefficient blocks
//   the scan path: progressive (SOF2), multi-scan, arithmetic-coded (SOF9 / SOF10) and
//     4-component files; one wave per image walks the scans in file order, lanes over restart
//     intervals: jpeg_prog_kernel (Huffman: jdhuff.c's decoders) or jpeg_arith_kernel
//     (jdarith.c's QM-coder)
//   idct           one thread per block: libjpeg 9d block smoothing of progressive files whose last
//                  scan leaves AC 1..5 imprecise (jpg_smooth), dequantise, ISLOW IDCT (8x8, or
//                  16x16 / 16x8 for libjpeg 9's scaled chroma) into u8 component planes
//   color          8 output pixels per thread: chroma upsampling (turbo), then YCbCr -> BGR, RGB
//                  copied, gray replicated, or CMYK / YCCK (libjpeg's CMYK output) through OpenCV's
//                  CMYK -> BGR (jpg_color_space: component IDs, JFIF / Adobe markers, per library)
// Supported: 8-bit DCT JPEG (Huffman or arithmetic), 1, 3 or 4 components, sampling 4:4:4 /
// 4:2:2 (h2v1) / 4:2:0 (h2v2) (a fourth component sampled as the first), optional restart
// intervals.  Anything else (lossless, hierarchical, 12-bit, big-gamut colour, extension
// markers) is IDN_EUNSUPPORTED -- as libjpeg 9d (8-bit, DCT) refuses the first three too.
// Damaged entropy-coded data decodes as libjpeg decodes it: past an interval's data the bits are
// 0 and an MCU is decoded only if the data lasted up to its start (jdhuff.c insufficient_data),
// a bit pattern that is no code takes 17 bits and decodes as 0.
#include "idn_common.hpp"

#include <string.h>

#include <algorithm>
#include <string>
#include <atomic>
#include <thread>
#include <vector>

namespace idn {

#ifndef IDN_JPG_LUTB  // A/B builds set it
#define IDN_JPG_LUTB 9
#endif
constexpr int JPG_LUTB = IDN_JPG_LUTB;  // fast Huffman lookup bits

struct JpegDev {
  uint64_t scan_off;   // entropy-coded bytes in the batch buffer
  uint32_t scan_len;
  int width, height, ncomp, mcux, mcuy, restart;  // restart: MCUs per interval (0: none)
  int hmax, vmax, nintervals;
  int ch[4], cv[4], tq[4], td[4], ta[4];
  int bw[4], bh[4];         // blocks per row / column of each component plane (MCU-padded)
  int sh[4], sv[4];         // IDCT output scale per component: 1 (8 samples) or 2 (16 samples)
  int pw[4];                // component plane row pitch in bytes (bw * 8 * sh)
  int dw[4], dh[4];         // component plane size after the IDCT (libjpeg downsampled_width)
  int up;                   // chroma upsampling: 0 none (full-size planes), 1 h2v1, 2 h2v2 fancy
  int cb_g;                 // jdcolor.c Cb -> G multiplier: libjpeg 9 22553, turbo 22554
  int rgb;                  // jpg_color_space: 0 YCbCr, 1 RGB, 2 CMYK, 3 YCCK
  uint64_t blk_off[4];      // first block of each component in the batch coefficient buffer
  uint64_t pl_off[4];       // component plane byte offset in the batch plane buffer
  uint64_t ub_off;          // unstuffed entropy bytes (workspace), capacity scan_len + 64
  uint32_t iv_off;          // first entry of the image's interval tables (jpeg_unstuff_final)
  uint32_t mk_off, mk_cap;  // the markers found in the segment (jpeg_unstuff_write): first, room
  uint32_t ch_off, nchunks; // the image's chunks in the batch chunk arrays
  uint32_t chunk_bits;
  int bpm;                  // blocks per MCU (1 for a single-component scan)
  uint32_t total_blocks;    // MCUs x bpm
  int wib[4], hib[4];       // blocks with data per component row / column (jdinput.c
                            // width_in_blocks): what a non-interleaved scan codes
  uint32_t scan0, nscan;    // scan path: the image's scans in the batch scan table (0: none)
  int arith;                // arithmetic-coded (the scan path's jpeg_arith_kernel)
  int smooth;               // libjpeg 9d block smoothing (jdcoefct.c decompress_smooth_data)
  int orient;               // the EXIF orientation cv2.imread applies (1: none; jpg_exif_orientation)
  int8_t cbits[4][6];       // its coef_bits latch per component (zigzag 0..5; -1: never coded)
  uint8_t ph_comp[10], ph_dv[10], ph_dh[10];  // block of the MCU -> component, block row, column
  uint16_t q[4][64];        // quantisation tables, natural order
  uint16_t lut[4][1 << JPG_LUTB];  // [DC0, DC1, AC0, AC1]: len << 8 | symbol, 0 = longer code
  int32_t maxcode[4][18];   // libjpeg jdhuff: largest code of each length (-1: none), [17] sentinel
  int32_t valoff[4][18];    // huffval index of the first code of each length, minus that code
  uint8_t huffval[4][256];
};

// one scan of the scan path (progressive / multi-scan files).  Table slots: k = the DC table of
// scan component k, 4 + k = its AC table (only the slots the scan's kind reads are filled).
enum { JPG_SEQ = 0, JPG_DC_FIRST = 1, JPG_DC_REFINE = 2, JPG_AC_FIRST = 3, JPG_AC_REFINE = 4 };
struct JpegScanDev {
  uint64_t scan_off;        // entropy-coded bytes in the batch buffer (unstuffed like JpegDev's)
  uint32_t scan_len;
  uint64_t ub_off;
  uint32_t iv_off;
  uint32_t mk_off, mk_cap;
  int nintervals;
  int img, ns, comp[4], Ss, Se, Ah, Al, restart, kind;
  uint32_t nunits;          // MCUs (interleaved) or the component's blocks (non-interleaved)
  int arith;                // arithmetic-coded: the statistics of tables td / ta per scan component,
  int td[4], ta[4];         // conditioned by aL / aU (DC) and aK (AC); no Huffman tables
  uint8_t aL[4], aU[4], aK[4];
  uint16_t lut[8][1 << JPG_LUTB];
  int32_t maxcode[8][18], valoff[8][18];
  uint8_t huffval[8][256];
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
// one scan of a progressive / multi-scan file: its components (frame indices), their tables as
// defined when the scan starts, spectral band and successive-approximation bits, restart interval
struct ScanHost {
  int ns = 0, comp[4] = {}, Ss = 0, Se = 63, Ah = 0, Al = 0, restart = 0;
  HuffSpec dc[4], ac[4];  // per scan component
  int td[4] = {}, ta[4] = {};                   // its table numbers
  uint8_t aL[4] = {}, aU[4] = {}, aK[4] = {};  // arithmetic conditioning of those tables (DAC)
  size_t begin = 0, end = 0;
};
struct JpegHost {
  int width = 0, height = 0, ncomp = 0, restart = 0;
  int cid[4] = {}, ch[4] = {}, cv[4] = {}, tq[4] = {}, td[4] = {}, ta[4] = {};
  bool qpresent[4] = {};
  uint16_t q[4][64] = {};  // natural order
  HuffSpec dc[4], ac[4];
  size_t scan_begin = 0, scan_end = 0;
  bool arith = false;       // arithmetic-coded frame (SOF9 / SOF10)
  // arithmetic conditioning per table (DAC; jdmarker.c get_soi's defaults L 0, U 1, K 5)
  uint8_t dacL[16] = {}, dacU[16] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1},
          dacK[16] = {5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5};
  bool jfif = false, adobe = false;  // APP0 "JFIF" / APP14 "Adobe" seen (jdmarker.c examine_app0/14)
  int adobe_transform = 0;
  bool progressive = false;
  bool smooth = false;      // libjpeg 9d block-smooths the file (jpg_scans_done)
  int8_t cbits[4][6] = {};  // its coef_bits latch: per component, zigzag 0..5 (-1: never coded)
  std::vector<ScanHost> scans;  // the scan path (progressive or multi-scan); empty: one scan
};

// end of the entropy-coded segment starting at p[i]: the first marker that is neither RSTn nor
// below SOF0 (stuffed 0xFF00 and fill bytes skipped).  A stray marker below SOF0 stays inside: it
// ends the data of its restart interval (jpeg_unstuff_final), as jdmarker.c's resync reads it.
static size_t jpg_segment_end(const uint8_t* p, size_t n, size_t i) {
  while (i + 1 < n) {
    if (p[i] != 0xFF) {
      ++i;
      continue;
    }
    const uint8_t nb = p[i + 1];
    if (nb < 0xC0 || (nb >= 0xD0 && nb <= 0xD7)) i += 2;  // (0x00: stuffing)
    else if (nb == 0xFF) i += 1;
    else return i;
  }
  return n;
}

static int jpg_fail(std::string* err, const char* msg) {
  if (err) *err = msg;
  return IDN_EUNSUPPORTED;
}

// ---- host: the EXIF orientation cv2.imread applies ----------------------------------------------
// OpenCV 3.4.2's imread (loadsave.cpp) calls ApplyExifOrientation on the decoded image unless
// IMREAD_IGNORE_ORIENTATION is set; the tag comes from exif.cpp's ExifReader, which walks the
// file's markers two bytes at a time (the 0xFF is not checked) and takes the FIRST APP1 segment
// as EXIF data whatever its identifier.  Restated from the published OpenCV source [recalled: cv2
// is not importable here], including when it gives up (orientation 1, the image as decoded):
//   - the walk skips (by their length field) SOF0, SOF2, DHT, DQT, DRI, SOS, RST0-7, APP0,
//     APP2-15, COM; SOI / EOI have no length; any other code ends the search (no EXIF);
//   - a length below 2, or an APP1 length <= 6, is a parse error (no EXIF); the APP1 data is
//     the length - 6 bytes after the 6-byte identifier slot (zero-filled past the end of file);
//   - the TIFF header: "II" little-endian, "MM" or any other equal pair big-endian, unequal
//     bytes big-endian too; u16 at 2 must be 42, else no entries; IFD0 at the u32 at 4;
//   - every IFD0 entry is parsed, and the tags exif.cpp knows read their values: an offset past
//     the data (getU16 / getU32 bounds, getString's size check) aborts the whole parse, so a
//     broken MAKE string after a good Orientation still leaves the image unrotated; the first
//     entry of a tag wins (std::map insert); Orientation = the u16 at entry + 8.
// 32-bit offset arithmetic wraps as exif.cpp's uint32_t does.
struct CvExifReader {
  const uint8_t* d;
  size_t n;
  bool intel = false, bad = false;
  uint32_t u16(size_t o) {
    if (o + 1 >= n) {
      bad = true;
      return 0;
    }
    return intel ? (uint32_t)d[o] | (uint32_t)d[o + 1] << 8 : (uint32_t)d[o] << 8 | d[o + 1];
  }
  uint32_t u32(size_t o) {
    if (o + 3 >= n) {
      bad = true;
      return 0;
    }
    return intel ? (uint32_t)d[o] | (uint32_t)d[o + 1] << 8 | (uint32_t)d[o + 2] << 16 |
                       (uint32_t)d[o + 3] << 24
                 : (uint32_t)d[o] << 24 | (uint32_t)d[o + 1] << 16 | (uint32_t)d[o + 2] << 8 |
                       d[o + 3];
  }
  void rationals(size_t entry, int count) {  // getResolution / WhitePoint / ... / RefBW
    uint32_t r = u32(entry + 8);
    for (int k = 0; k < count && !bad; ++k, r += 8) {
      (void)u32(r);
      (void)u32((uint32_t)(r + 4));
    }
  }
  void string(size_t entry) {  // getString: the size check only
    const uint32_t size = u32(entry + 4);
    uint32_t off = 8;
    if (!bad && size > 4) off = u32(entry + 8);
    if (!bad && (off > n || (uint32_t)(off + size) > n)) bad = true;
  }
};

// the orientation (1..8 acts, anything else is left as decoded) OpenCV 3.4.2 applies to file p
static int jpg_exif_orientation(const uint8_t* p, size_t n) {
  size_t i = 0;
  std::vector<uint8_t> data;
  bool found = false;
  while (!found) {
    if (i + 2 > n) break;  // (a short read ends the search)
    const uint8_t m = p[i + 1];
    i += 2;
    auto field = [&]() -> size_t {  // getFieldSize: 0 on a short read
      if (i + 2 > n) {
        i = n;
        return 0;
      }
      const size_t v = (size_t)p[i] << 8 | p[i + 1];
      i += 2;
      return v;
    };
    if (m == 0xC0 || m == 0xC2 || m == 0xC4 || m == 0xDB || m == 0xDD || m == 0xDA ||
        (m >= 0xD0 && m <= 0xD7) || m == 0xE0 || (m >= 0xE2 && m <= 0xEF) || m == 0xFE) {
      const size_t skip = field();
      if (skip < 2) return 1;
      i += skip - 2;
    } else if (m == 0xD8 || m == 0xD9) {
    } else if (m == 0xE1) {
      const size_t len = field();
      if (len <= 6) return 1;
      data.assign(len - 6, 0);
      i += 6;
      if (i < n) memcpy(data.data(), p + i, std::min(len - 6, n - i));
      found = true;
    } else {
      break;
    }
  }
  if (!found) return 1;
  CvExifReader R{data.data(), data.size()};
  // getFormat: unequal first bytes -> NONE (read big-endian), 'I' Intel, 'M' or other -> big-endian
  R.intel = !(data.size() > 1 && data[0] != data[1]) && data[0] == 'I';
  if (R.u16(2) != 0x2A || R.bad) return 1;  // checkTagMark (a short block throws)
  uint32_t off = R.u32(4);
  const uint32_t nent = R.u16(off);
  if (R.bad) return 1;
  off += 2;
  int orient = -1;
  for (uint32_t e = 0; e < nent; ++e, off += 12) {
    const uint32_t tag = R.u16(off);
    switch (tag) {
      case 0x010E: case 0x010F: case 0x0110: case 0x0131: case 0x0132: case 0x8298:
        R.string(off);
        break;  // description, make, model, software, date-time, copyright
      case 0x0112: {
        const uint32_t v = R.u16((size_t)off + 8);
        if (orient < 0) orient = (int)v;
        break;
      }
      case 0x011A: case 0x011B: R.rationals(off, 1); break;  // x / y resolution
      case 0x0128: case 0x0213: (void)R.u16((size_t)off + 8); break;
      case 0x013E: R.rationals(off, 2); break;   // white point
      case 0x013F: R.rationals(off, 6); break;   // primary chromaticities
      case 0x0211: R.rationals(off, 3); break;   // YCbCr coefficients
      case 0x0214: R.rationals(off, 6); break;   // reference black / white
      default: break;                            // EXIF_OFFSET and unknown tags: no value read
    }
    if (R.bad) return 1;
  }
  return orient >= 1 && orient <= 8 ? orient : 1;
}

// the end of a scan-path file (EOI or end of data): at least one scan.  libjpeg block-smooths a
// progressive file (jdcoefct.c smoothing_ok, libjpeg 9d) only when EVERY component has DC data
// (coef_bits[0] >= 0: jdphuff.c sets coef_bits[k] = Al for k in Ss..Se at each scan's start) and
// nonzero quantisers Q00 Q01 Q10 Q20 Q11 Q02, and some component's AC coefficients 1..5 stay
// imprecise after the last scan (coef_bits != 0): J.smooth and the latched coef_bits, applied by
// the IDCT pass (jpg_smooth)
static int jpg_scans_done(JpegHost& J, std::string* err) {
  if (J.scans.empty()) return jpg_fail(err, "no SOS");
  if (J.progressive) {
    int bits[4][6];
    for (auto& b : bits)
      for (int& v : b) v = -1;
    for (const ScanHost& S : J.scans)
      for (int k = 0; k < S.ns; ++k)
        for (int z = S.Ss; z <= std::min(S.Se, 5); ++z) bits[S.comp[k]][z] = S.Al;
    bool useful = false;
    for (int c = 0; c < J.ncomp; ++c) {
      const uint16_t* q = J.q[J.tq[c]];
      if (bits[c][0] < 0 || q[0] == 0 || q[1] == 0 || q[8] == 0 || q[16] == 0 || q[9] == 0 ||
          q[2] == 0)
        return IDN_OK;  // smoothing_ok() is FALSE for the whole image
      for (int z = 1; z <= 5; ++z) useful |= bits[c][z] != 0;
    }
    J.smooth = useful;
    for (int c = 0; c < J.ncomp; ++c)
      for (int z = 0; z < 6; ++z) J.cbits[c][z] = (int8_t)bits[c][z];
  }
  return IDN_OK;
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
    if (m == 0xD9) return jpg_scans_done(J, err);
    const size_t len = ((size_t)p[i] << 8) | p[i + 1];
    if (len < 2 || i + len > n) return jpg_fail(err, "truncated segment");
    const uint8_t* s = p + i + 2;
    const size_t sl = len - 2;
    switch (m) {
      case 0xC0:
      case 0xC1:
      case 0xC2:
      case 0xC9:
      case 0xCA: {  // SOF0 / 1 / 2: baseline / extended sequential / progressive Huffman; SOF9 /
                    // SOF10: sequential / progressive arithmetic
        if (sof) return jpg_fail(err, "second frame header");
        if (sl < 6 || s[0] != 8) return jpg_fail(err, "only 8-bit JPEG");
        J.progressive = m == 0xC2 || m == 0xCA;
        J.arith = m == 0xC9 || m == 0xCA;
        J.height = (s[1] << 8) | s[2];
        J.width = (s[3] << 8) | s[4];
        J.ncomp = s[5];
        if (J.ncomp != 1 && J.ncomp != 3 && J.ncomp != 4)
          return jpg_fail(err, "only 1, 3 or 4 components");
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
      case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xCB: case 0xCD: case 0xCE: case 0xCF:
        return jpg_fail(err, "lossless / hierarchical JPEG not supported");
      case 0xCC: {  // DAC (jdmarker.c get_dac): arithmetic conditioning, 2 bytes per table
        if (sl % 2) return jpg_fail(err, "bad DAC length");
        for (size_t k = 0; k + 2 <= sl; k += 2) {
          const int idx = s[k], val = s[k + 1];
          if (idx >= 32) return jpg_fail(err, "bad DAC table index");
          if (idx >= 16) {
            J.dacK[idx - 16] = (uint8_t)val;
          } else {
            J.dacL[idx] = (uint8_t)(val & 15);
            J.dacU[idx] = (uint8_t)(val >> 4);
            if (J.dacL[idx] > J.dacU[idx]) return jpg_fail(err, "bad DAC value");
          }
        }
        break;
      }
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
      case 0xE0:  // APP0: JFIF (jdmarker.c examine_app0: identifier + at least 14 bytes)
        if (sl >= 14 && memcmp(s, "JFIF", 5) == 0) J.jfif = true;
        break;
      case 0xEE:  // APP14 Adobe (examine_app14: at least 12 bytes): the colour transform flag
        if (sl >= 12 && memcmp(s, "Adobe", 5) == 0) {
          J.adobe = true;
          J.adobe_transform = s[11];
        }
        break;
      case 0xDE: case 0xDF: case 0xF0: case 0xF1: case 0xF2: case 0xF3: case 0xF4: case 0xF5:
      case 0xF6: case 0xF7: case 0xF8: case 0xF9: case 0xFA: case 0xFB: case 0xFC: case 0xFD:
        // DHP / EXP / JPGn: fatal in libjpeg-turbo (read_markers' reserved-marker error); in libjpeg
        // 9 JPG8 is the LSE colour-transform marker (not restated)
        return jpg_fail(err, "reserved / extension marker (DHP, EXP, JPGn, LSE) not supported");
      case 0xDA: {  // SOS
        if (!sof) return jpg_fail(err, "SOS before SOF");
        if (sl < 1) return jpg_fail(err, "bad SOS");
        const int ns = s[0];
        if (ns < 1 || ns > J.ncomp || sl < 1 + 2 * (size_t)ns + 3) return jpg_fail(err, "bad SOS");
        if (J.ncomp >= 3) {  // (a fourth component, K, sampled as the first)
          const bool s444 = J.ch[0] == 1 && J.cv[0] == 1;
          const bool s422 = J.ch[0] == 2 && J.cv[0] == 1;
          const bool s420 = J.ch[0] == 2 && J.cv[0] == 2;
          if (!(s444 || s422 || s420) || J.ch[1] != 1 || J.cv[1] != 1 || J.ch[2] != 1 ||
              J.cv[2] != 1 || (J.ncomp == 4 && (J.ch[3] != J.ch[0] || J.cv[3] != J.cv[0])))
            return jpg_fail(err, "chroma sampling other than 4:4:4 / 4:2:2 / 4:2:0");
        }
        ScanHost S;
        S.ns = ns;
        S.restart = J.restart;
        for (int k = 0; k < ns; ++k) {
          int c = 0;
          while (c < J.ncomp && J.cid[c] != s[1 + 2 * k]) ++c;
          if (c == J.ncomp) return jpg_fail(err, "scan names an unknown component");
          if (k > 0 && c <= S.comp[k - 1]) return jpg_fail(err, "scan component order differs from the frame");
          S.comp[k] = c;
          const int td = s[2 + 2 * k] >> 4, ta = s[2 + 2 * k] & 15;
          if (td > 3 || ta > 3) return jpg_fail(err, "bad SOS table");
          J.td[c] = td;
          J.ta[c] = ta;
          S.dc[k] = J.dc[td];
          S.ac[k] = J.ac[ta];
          S.td[k] = td;
          S.ta[k] = ta;
          S.aL[k] = J.dacL[td];
          S.aU[k] = J.dacU[td];
          S.aK[k] = J.dacK[ta];
        }
        const uint8_t* ss = s + 1 + 2 * ns;
        S.Ss = ss[0];
        S.Se = ss[1];
        S.Ah = ss[2] >> 4;
        S.Al = ss[2] & 15;
        if (J.progressive) {  // jdinput.c / jdhuff.c start_pass_huff_decoder checks
          const bool dc = S.Ss == 0;
          if ((dc && S.Se != 0) || (!dc && (S.Se < S.Ss || S.Se > 63 || ns != 1)) || S.Ah > 13 ||
              S.Al > 13 || (S.Ah != 0 && S.Al != S.Ah - 1))
            return jpg_fail(err, "bad progressive scan parameters");
        } else if (S.Ss != 0 || S.Se != 63 || ss[2] != 0) {
          return jpg_fail(err, "not a sequential scan");
        }
        for (int k = 0; k < ns; ++k) {
          const int c = S.comp[k];
          if (!J.qpresent[J.tq[c]]) return jpg_fail(err, "missing quantisation table");
          const bool need_dc = S.Ss == 0 && S.Ah == 0, need_ac = S.Se > 0 && !(J.progressive && S.Ah);
          const bool need_ac_ref = J.progressive && S.Ss > 0 && S.Ah;
          if (!J.arith &&
              ((need_dc && !S.dc[k].present) || ((need_ac || need_ac_ref) && !S.ac[k].present)))
            return jpg_fail(err, "missing Huffman table");
        }
        S.begin = i + len;
        if (!J.progressive && !J.arith && J.ncomp <= 3 && J.scans.empty() && ns == J.ncomp) {
          // one interleaved sequential scan: the parallel path.  Its segment runs up to the EOI
          // (scanning back from the end) or the end of data
          for (int c = 0; c < J.ncomp; ++c)
            if (J.td[c] > 1 || J.ta[c] > 1) return jpg_fail(err, "Huffman table id > 1");
          J.scan_begin = S.begin;
          size_t e = n;
          while (e >= J.scan_begin + 2 && !(p[e - 2] == 0xFF && p[e - 1] == 0xD9)) --e;
          J.scan_end = (e >= J.scan_begin + 2) ? e - 2 : n;
          return IDN_OK;
        }
        S.end = jpg_segment_end(p, n, S.begin);
        J.scans.push_back(S);
        if (J.scans.size() > 64) return jpg_fail(err, "too many scans");
        i = S.end;
        continue;  // the next marker
      }
      default:
        if (m < 0xC0) return jpg_fail(err, "corrupt marker");
        break;  // APPn, COM, ...: skip
    }
    i += len;
  }
  return jpg_scans_done(J, err);
}

// jdhuff.c jpeg_make_d_derived_tbl: canonical codes -> fast lookup + maxcode / valoffset
static int jpeg_build_huff(const HuffSpec& H, bool dc, uint16_t* lut, int32_t* maxcode,
                           int32_t* valoff, uint8_t* huffval, std::string* err) {
  int code = 0, k = 0;
  memset(lut, 0, sizeof(uint16_t) << JPG_LUTB);
  for (int l = 1; l <= 16; ++l) {
    // jdhuff.c jpeg_make_d_derived_tbl: the codes of length l must fit in l bits and none may be
    // all ones (code after the last >= 2^l is JERR_BAD_HUFF_TABLE); checked before any LUT write
    if (code + (int)H.bits[l] >= (1 << l)) return jpg_fail(err, "bad Huffman table");
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
// Stage 1, jpeg_unstuff_count / _write / _final (16 KiB tiles): the entropy-coded segment without its
// stuffed 0x00 bytes, fill bytes and RST markers, and the bit offset where each restart interval
// starts.  The decoders then read a plain big-endian bit string.
//
// Stage 2, images without restart markers: the scan is cut into chunk_bits-bit chunks, one thread
// each, decoded in parallel by self-synchronisation (Huffman codes and the block structure
// resynchronise: from an arbitrary start state a trajectory joins the true one after ~0.8 kbit
// median, 9 kbit max on the test images).  A decoder state is (bit position, block of the MCU,
// coefficient index z; z = 0: a DC symbol is next).
//   pass A   every chunk from (its first bit, block 0, z 0)              -> end state
//   pass B   every chunk from its predecessor's end state, repeated until no end state changes
//            (chunk 0 starts from the true state, so the chain is then exact by induction); the
//            final pass also counts the chunk's DC symbols and per-component DC differences
//   prefix   per image: each chunk's first block index and DC predictors
//   write    every chunk again from its exact start state, writing coefficient blocks
// Images with restart markers: each interval is cut into its own chunks (jpeg_chunk_map_kernel);
// an interval's first chunk starts from its known state, the prefix restarts at each interval.
// Chunk size: the ABI's flags may set one; the default depends on the batch (jpeg_plan)
// Checkpoints (round 5): every pass records, per chunk and JPG_SUB-bit sub-chunk, the decoder state
// at the first symbol that starts at or after the sub-chunk's first bit and the counts (blocks, DC
// sums) from the chunk start to it.  A later pass that decodes the chunk from a new start state
// stops at the first checkpoint where its state equals the recorded one -- from there the
// trajectory is the recorded one, so the end state is and the counts shift by the difference at
// that checkpoint (a chunk's trajectories typically join within ~1 kbit, so the B passes no
// longer decode whole chunks) -- and the write pass runs one thread per sub-chunk from the final
// checkpoints: many times the threads of one per chunk, each as much shorter (a single image's
// write pass was 0.76 ms of serial decoding per thread).  256 bits measured best against 128, 512
// and 1024 (profiles/r05/jpeg/sub_ab_sweep.txt: a joining trajectory stops sooner).
#ifndef IDN_JPG_SUB  // A/B builds set it
#define IDN_JPG_SUB 256
#endif
constexpr uint32_t JPG_SUB = IDN_JPG_SUB;
__host__ __device__ __forceinline__ uint32_t jpg_nsub(uint32_t chunk_bits) {
  return (chunk_bits + JPG_SUB - 1) / JPG_SUB;
}

__device__ __forceinline__ uint32_t jpg_be32(const uint8_t* __restrict__ p) {
  const uint32_t w = *reinterpret_cast<const uint32_t*>(p);
  return __builtin_bswap32(w);
}

// reads one restart interval of a plain big-endian bit string through a range-checked buffer
// resource, through a per-lane ring of JRG_S byte-swapped 16-byte groups in LDS refilled one group
// ahead from a load held in a register (as the chunk decoders' jpg_run): a register queue of
// groups in flight made every group change wait for the youngest load (moving a register whose
// load is pending waits for it).  Bits from `end` on read as 0 (jdhuff.c jpeg_fill_bit_buffer past
// a marker); `pos` counts the bits taken, so pos > end says the data ran out (insufficient_data).
constexpr int JRG_S = 4;
constexpr int JRING_S = JRG_S * 4 + 4;  // ring words per lane (a pad group)
struct BitStream {
  rsrc_t rs;
  uint32_t* ring;
  uint64_t acc;    // left-aligned
  int nb;
  uint32_t wi, pos, end;  // wi: the next word to append
  v4u pend;               // group (wi >> 2) + JRG_S, raw
  __device__ __forceinline__ void put(uint32_t g, const v4u v) {
    *reinterpret_cast<v4u*>(ring + (g & (JRG_S - 1)) * 4) =
        v4u{__builtin_bswap32(v.x), __builtin_bswap32(v.y), __builtin_bswap32(v.z),
            __builtin_bswap32(v.w)};
  }
  __device__ __forceinline__ uint32_t word() {
    uint32_t w = ring[wi & (4 * JRG_S - 1)];
    const uint32_t wbit = wi * 32u;  // (bit positions are below 2^31: 32-bit arithmetic)
    w = wbit + 32u <= end ? w : wbit >= end ? 0u : w & ~(0xFFFFFFFFu >> (end - wbit));
    if ((++wi & 3) == 0) {  // group (wi >> 2) - 1 retired: its slot takes the pending group
      put((wi >> 2) + JRG_S - 1, pend);
      pend = __builtin_amdgcn_raw_buffer_load_b128(rs, ((wi >> 2) + JRG_S) * 16u, 0, 0);
    }
    return w;
  }
  __device__ __forceinline__ void start(rsrc_t r, uint32_t* rg, uint32_t p, uint32_t e) {
    rs = r;
    ring = rg;
    end = e;
    pos = p;
    wi = p >> 5;
    const uint32_t g0 = wi >> 2;
#pragma unroll
    for (int k = 0; k < JRG_S; ++k)
      put(g0 + k, __builtin_amdgcn_raw_buffer_load_b128(rs, (g0 + k) * 16u, 0, 0));
    pend = __builtin_amdgcn_raw_buffer_load_b128(rs, (g0 + JRG_S) * 16u, 0, 0);
    const uint32_t w0 = word(), w1 = word();
    acc = ((uint64_t)w0 << 32 | w1) << (p & 31);
    nb = 64 - (int)(p & 31);
  }
  __device__ __forceinline__ void refill() {
    if (nb < 32) {
      acc |= (uint64_t)word() << (32 - nb);
      nb += 32;
    }
  }
  __device__ __forceinline__ uint32_t bits(int s) {
    const uint32_t r = s ? (uint32_t)(acc >> (64 - s)) : 0u;
    acc <<= s;
    nb -= s;
    pos += (uint32_t)s;
    return r;
  }
};

__device__ __forceinline__ int jpg_extend(uint32_t v, int s) {  // HUFF_EXTEND
  return (int)v < (1 << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v;
}

// mca[t][l - 10] (l = 10..16): the largest code of length <= l, left-aligned to 16 bits with
// ones below (-1 while there is none; a length without codes repeats the one before), so that
// "code16 <= mca" is monotone in l and a longer-than-LUT code's length is 10 + the number of
// lengths it exceeds -- seven compares on two 16-byte LDS reads instead of a walk of dependent
// maxcode reads (one per length) that every wave took whenever one of its 64 lanes missed the LUT
struct JpegLds {
  alignas(16) int32_t mca[4][8];
  uint8_t natural[80];  // jpg_natural (the write pass's coefficient positions)
  uint16_t lut[4][1 << JPG_LUTB];
  int32_t maxcode[4][18], valoff[4][18];
  uint8_t huffval[4][256];
};

// the scan path's tables (JpegScanDev slots)
struct JpegLdsScan {
  alignas(16) int32_t mca[8][8];
  uint8_t natural[80];  // jpg_natural: a __constant__ read at a computed index is a vector load
  uint16_t lut[8][1 << JPG_LUTB];
  int32_t maxcode[8][18], valoff[8][18];
  uint8_t huffval[8][256];
};

// entry i of mca (see JpegLds) from a table's maxcode[18]: the codes longer than the fast table,
// lengths 10 .. 16, so the table must be exactly 9 bits
static_assert(JPG_LUTB == 9, "jpg_mca and jpg_decode's compare-count assume 9-bit fast tables");
__device__ __forceinline__ int32_t jpg_mca(const int32_t* __restrict__ maxcode, int i) {
  int32_t m = -1;
  for (int l = 10; l <= 10 + i && l <= 16; ++l)
    if (maxcode[l] >= 0) m = maxcode[l] << (16 - l) | ((1 << (16 - l)) - 1);
  return i == 7 ? 0x7FFFFFFF : m;
}

// one Huffman symbol (nb >= 32 on entry); returns the symbol and its code length in *len.  A bit
// pattern that is no code: symbol 0, badlen bits, *bad set (see jpeg_write_kernel on badlen)
template <typename TT>
__device__ __forceinline__ int jpg_decode(uint64_t acc, const TT& T, int t, int* len,
                                          int badlen = 17, bool* bad = nullptr) {
  const uint32_t e = T.lut[t][acc >> (64 - JPG_LUTB)];
  if (e) {
    *len = (int)(e >> 8);
    return e & 0xFF;
  }
  const int32_t c16 = (int32_t)(acc >> 48);
  const int4 m0 = *reinterpret_cast<const int4*>(&T.mca[t][0]);
  const int4 m1 = *reinterpret_cast<const int4*>(&T.mca[t][4]);
  const int l = 10 + (c16 > m0.x) + (c16 > m0.y) + (c16 > m0.z) + (c16 > m0.w) + (c16 > m1.x) +
                (c16 > m1.y) + (c16 > m1.z);
  if (l > 16) {  // not a code (a speculative trajectory or a corrupt file): jdhuff.c
    *len = badlen;  // jpeg_huff_decode reads up to length 17, then JWRN_HUFF_BAD_CODE, symbol 0
    if (bad) *bad = true;
    return 0;
  }
  *len = l;
  return T.huffval[t][(T.valoff[t][l] + (c16 >> (16 - l))) & 0xFF];
}

__device__ __forceinline__ void jpg_load_tables(JpegLds& T, const JpegDev& D) {
  const uint32_t* s = reinterpret_cast<const uint32_t*>(&D.lut[0][0]);
  uint32_t* d = reinterpret_cast<uint32_t*>(&T.lut[0][0]);
  for (int k = threadIdx.x; k < (int)(sizeof(T.lut) / 4); k += blockDim.x) d[k] = s[k];
  for (int k = threadIdx.x; k < 4 * 18; k += blockDim.x) {
    (&T.maxcode[0][0])[k] = (&D.maxcode[0][0])[k];
    (&T.valoff[0][0])[k] = (&D.valoff[0][0])[k];
  }
  for (int k = threadIdx.x; k < 4 * 256; k += blockDim.x) (&T.huffval[0][0])[k] = (&D.huffval[0][0])[k];
  for (int k = threadIdx.x; k < 4 * 8; k += blockDim.x) T.mca[k >> 3][k & 7] = jpg_mca(D.maxcode[k >> 3], k & 7);
  for (int k = threadIdx.x; k < 80; k += blockDim.x) T.natural[k] = jpg_natural[k];
}

// decoder state packed in 64 bits: bit position | block of the MCU << 32 | z << 40
__device__ __forceinline__ uint64_t jpg_state(uint32_t pos, uint32_t ph, uint32_t z) {
  return (uint64_t)pos | (uint64_t)ph << 32 | (uint64_t)z << 40;
}

struct ChunkOut {
  uint32_t nblk;
  int32_t dcsum[3];
};

// the per-image constants jpg_run needs, loaded once into (scalar) registers: inside the symbol
// loop a lane-indexed read of JpegDev (phase -> component -> tables) was a global load on the
// critical path of every symbol
struct JpgConst {
  uint64_t phase_info;  // per block of the MCU, 6 bits: component | DC table << 2 | AC table << 4
  uint64_t phase_pos;   // per block of the MCU, 6 bits: block row | block column << 3
  // per-component values packed into integers and picked by shifts: selecting among fields of a
  // local struct was turned into a lane-indexed load from a stack copy (scratch)
  uint32_t bo0;          // first block of component 0
  uint64_t bo12;         // first blocks of components 1, 2 relative to component 0 (32 bits each)
  uint64_t bw;           // blocks per row, 16 bits per component
  uint32_t vshs;         // per component 4 bits: vertical | horizontal blocks per MCU << 2
  int mcux, bpm;
  uint32_t total_blocks;
};

__device__ __forceinline__ JpgConst jpg_const(const JpegDev& D) {
  JpgConst K;
  K.phase_info = 0;
  K.phase_pos = 0;
  for (int p = 0; p < D.bpm; ++p) {
    const int c = D.ph_comp[p];
    K.phase_info |= (uint64_t)(c | D.td[c] << 2 | (2 + D.ta[c]) << 4) << (6 * p);
    K.phase_pos |= (uint64_t)(D.ph_dv[p] | D.ph_dh[p] << 3) << (6 * p);
  }
  const bool one = D.ncomp == 1;
  K.bo0 = (uint32_t)D.blk_off[0];
  K.bo12 = (uint64_t)(uint32_t)(D.blk_off[1] - D.blk_off[0]) |
           (uint64_t)(uint32_t)(D.blk_off[2] - D.blk_off[0]) << 32;
  K.bw = (uint64_t)(D.bw[0] & 0xFFFF) | (uint64_t)(D.bw[1] & 0xFFFF) << 16 |
         (uint64_t)(D.bw[2] & 0xFFFF) << 32;
  K.vshs = 0;
  for (int c = 0; c < 3; ++c)
    K.vshs |= (uint32_t)((one ? 1 : D.cv[c]) | (one ? 1 : D.ch[c]) << 2) << (4 * c);
  K.mcux = D.mcux;
  K.bpm = D.bpm;
  K.total_blocks = D.total_blocks;
  return K;
}

__device__ __forceinline__ int16_t* jpg_block(const JpgConst& K, int16_t* coef, int32_t blk,
                                              uint32_t ph, int c) {
  if (blk < 0 || (uint32_t)blk >= K.total_blocks) return nullptr;
  const int mcu = blk / K.bpm;
  const int my = mcu / K.mcux, mx = mcu - my * K.mcux;
  const uint32_t pp = (uint32_t)(K.phase_pos >> (6 * ph));
  const uint32_t vh = K.vshs >> (4 * c);
  const int vs = (int)(vh & 3), hs = (int)((vh >> 2) & 3);
  const int bw = (int)((K.bw >> (16 * c)) & 0xFFFF);
  const uint64_t bo = (uint64_t)K.bo0 + (c ? (uint32_t)(K.bo12 >> (32 * (c - 1))) : 0u);
  const int by = my * vs + (int)(pp & 7), bx = mx * hs + (int)((pp >> 3) & 7);
  return coef + (bo + (uint64_t)by * bw + bx) * 64;
}

// The chunk decoders' bit source: a per-lane ring of JRG 16-byte groups of the (byte-swapped)
// stream in LDS, refilled one group ahead from a range-checked buffer load held in registers.
// The 64 lanes of a wave sit at unrelated bit positions, so any per-lane branch in the symbol loop
// is taken by some lane on most iterations and the wave executes it every time; here the refill
// is branch-free (the next word is read from the ring every iteration, one iteration before it
// is needed) and only a group change (every 4 words of a lane) branches.
constexpr int JRG = 4;                 // ring groups per lane
constexpr int JRING_W = JRG * 4 + 4;   // ring words per lane (one pad group: lane stride 80 bytes)

// Decode symbols from state st while the next symbol starts before end_bit (and at most dc_limit
// DC symbols).  WRITE: coefficient blocks (blk = the block in progress; a DC symbol starts blk + 1)
// with DC predictors pred[]; else count DC symbols and DC differences.  Returns the end state.
// One symbol per iteration, DC or AC through the same decode (a DC symbol is a size 0..15, i.e. a
// run/size byte with run 0) and the block bookkeeping by selects.
// Where the data ends, libjpeg (jdhuff.c: jpeg_fill_bit_buffer's zero bits, insufficient_data)
// decodes an MCU only if the data lasted up to its start, reading 0 past the end:
//   tail  (chunked decoder, WRITE) end_bit is the end of the data: complete the MCU in progress,
//         and one that starts exactly at the end, never past the image's last block
//   MASK  (a restart interval, whose data the next one's follows) bits from end_bit on read as 0;
//         stop at dc_limit DC symbols or at an MCU that starts past end_bit
//   CLAMP (any other piece of a restart interval: the sync passes, the write pass's inner pieces)
//         bits from zero_bit (the interval's end) on read as 0, the stop rule unchanged: a symbol
//         that starts in the piece and runs past the interval's data reads libjpeg's zero fill,
//         not the next interval's bits
template <bool WRITE, bool MASK = false, bool CLAMP = false>
__device__ __forceinline__ uint64_t jpg_run(const JpgConst& K, const JpegLds& T, rsrc_t rs,
                                            uint32_t* __restrict__ ring, uint64_t st,
                                            uint32_t end_bit, ChunkOut* cnt, int32_t blk,
                                            int (&pred)[3], int16_t* __restrict__ coef,
                                            uint32_t dc_limit = 0xFFFFFFFFu, bool tail = false,
                                            int badlen = 17, uint32_t* badseen = nullptr,
                                            uint32_t zero_bit = 0xFFFFFFFFu) {
  static_assert(!(MASK && CLAMP), "MASK already zeroes the bits past end_bit");
  uint32_t ndc = 0;
  bool bad_real = false;  // WRITE: a bad code inside the image's blocks
  uint32_t pos = (uint32_t)st, ph = (uint32_t)(st >> 32) & 0xFF, z = (uint32_t)(st >> 40) & 0xFF;
  // ring: words wi .. of groups (wi >> 2) .. (wi >> 2) + JRG - 1 at ring[w & (4 JRG - 1)]; pend =
  // group (wi >> 2) + JRG, raw
  uint32_t wi = pos >> 5;
  {
    const uint32_t g0 = wi >> 2;
#pragma unroll
    for (int k = 0; k < JRG; ++k) {
      const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, (g0 + k) * 16u, 0, 0);
      *reinterpret_cast<v4u*>(ring + ((g0 + k) & (JRG - 1)) * 4) =
          v4u{__builtin_bswap32(v.x), __builtin_bswap32(v.y), __builtin_bswap32(v.z),
              __builtin_bswap32(v.w)};
    }
  }
  v4u pend = __builtin_amdgcn_raw_buffer_load_b128(rs, ((wi >> 2) + JRG) * 16u, 0, 0);
  uint64_t acc = 0;
  int nb = 0;
  // word wix of the stream (MASK: its bits from end_bit on cleared; CLAMP: from zero_bit on)
  auto fetch = [&](uint32_t wix) -> uint32_t {
    const uint32_t v = ring[wix & (4 * JRG - 1)];
    if (!MASK && !CLAMP) return v;
    const int64_t r = (int64_t)(MASK ? end_bit : zero_bit) - 32 * (int64_t)wix;
    return r >= 32 ? v : r <= 0 ? 0u : v & ~(0xFFFFFFFFu >> (uint32_t)r);
  };
  uint32_t nxt = fetch(wi);
  // append word wi (nxt) to acc; a new group retires its predecessor's slot to pend
  auto append = [&](bool need) {
    acc |= need ? (uint64_t)nxt << (32 - nb) : 0ull;
    nb += need ? 32 : 0;
    wi += need ? 1u : 0u;
    if (need && (wi & 3) == 0) {
      *reinterpret_cast<v4u*>(ring + (((wi >> 2) + JRG - 1) & (JRG - 1)) * 4) =
          v4u{__builtin_bswap32(pend.x), __builtin_bswap32(pend.y), __builtin_bswap32(pend.z),
              __builtin_bswap32(pend.w)};
      pend = __builtin_amdgcn_raw_buffer_load_b128(rs, ((wi >> 2) + JRG) * 16u, 0, 0);
    }
    nxt = fetch(wi);
  };
  append(true);
  append(true);
  acc <<= (pos & 31);
  nb -= (int)(pos & 31);
  int16_t* bp = nullptr;
  if (WRITE && z != 0) bp = jpg_block(K, coef, blk, ph, (int)(K.phase_info >> (6 * ph)) & 3);
  int32_t s0 = 0, s1 = 0, s2 = 0, nblk = 0;
  int p0 = pred[0], p1 = pred[1], p2 = pred[2];
  for (;;) {
    const bool dc = z == 0;
    if (MASK) {
      if (dc && ph == 0 && (ndc == dc_limit || pos > end_bit)) break;
    } else {
      if (pos >= end_bit) {
        if (!WRITE || !tail) break;
        const bool go = dc && ph == 0 ? pos == end_bit && (uint32_t)(blk + 1) < K.total_blocks
                                      : (uint32_t)blk < K.total_blocks;
        if (!go) break;
      }
      if (dc && ndc == dc_limit) break;
    }
    append(nb < 32);
    const uint32_t info = (uint32_t)(K.phase_info >> (6 * ph));
    const int c = info & 3;
    int len;
    bool bad = false;
    const int rs8 = jpg_decode(acc, T, dc ? (info >> 2) & 3 : (info >> 4) & 3, &len, badlen, &bad);
    if (WRITE) bad_real |= bad && (uint32_t)(dc ? blk + 1 : blk) < K.total_blocks;
    const int r = rs8 >> 4, s = rs8 & 15;
    const int val = s ? jpg_extend((uint32_t)((acc << len) >> 32) >> (32 - s), s) : 0;
    acc <<= len + s;
    nb -= len + s;
    pos += len + s;
    ndc += dc ? 1u : 0u;
    if (WRITE) {
      if (dc) {
        ++blk;
        const int p = (c == 0 ? p0 : c == 1 ? p1 : p2) + val;
        p0 = c == 0 ? p : p0;
        p1 = c == 1 ? p : p1;
        p2 = c == 2 ? p : p2;
        bp = jpg_block(K, coef, blk, ph, c);
        if (bp) bp[0] = (int16_t)p;
      } else if (s && bp) {
        bp[T.natural[min(z + r, 79u)]] = (int16_t)val;  // libjpeg's overrun guard
      }
    } else {
      nblk += dc ? 1 : 0;
      s0 += dc && c == 0 ? val : 0;
      s1 += dc && c == 1 ? val : 0;
      s2 += dc && c == 2 ? val : 0;
    }
    // next coefficient index: DC -> 1; AC: value r + 1 on, ZRL 16 on, EOB the block's end
    const uint32_t za = s ? z + r + 1 : (r == 15 ? z + 16 : 64u);
    const uint32_t zn = dc ? 1u : za;
    const bool wrap = zn >= 64;
    z = wrap ? 0u : zn;
    ph = wrap ? (ph + 1 == (uint32_t)K.bpm ? 0u : ph + 1) : ph;
  }
  pred[0] = p0;
  pred[1] = p1;
  pred[2] = p2;
  if (WRITE && badseen && bad_real) *badseen = 1u;
  if (!WRITE) {
    cnt->nblk += nblk;
    cnt->dcsum[0] += s0;
    cnt->dcsum[1] += s1;
    cnt->dcsum[2] += s2;
  }
  return jpg_state(pos, ph, z);
}

// stage 1: unstuff, in 16 KiB tiles of the segment (1024 threads x 16 bytes), every tile its own
// workgroup (one workgroup per image walked its tiles in sequence: 0.28 ms for a single 600x1000
// file): count the tile's kept bytes and markers, then each tile writes from the sum of the tiles
// before it (the kept bytes, and every marker's code and unstuffed offset), then per segment the
// length, the zero padding and the restart intervals (jpeg_unstuff_final).
// (DESC: a JpegDev per image, or a JpegScanDev per scan of the scan path: the same fields)
constexpr uint32_t UNS_TILE = 1024 * 16;
constexpr uint32_t JPG_MK_EXTRA = 64;  // marker table room beyond the restart markers
constexpr uint32_t JPG_IV_INHERIT = 0x80000000u;  // interval end flag: see jpeg_unstuff_final
constexpr size_t JPG_MAX_SCAN = ((size_t)1 << 28) - 64;  // bytes: bit positions below the flag

// the thread's 16 bytes [i0, i0 + 16): bit k of keep = byte i0 + k is data, of mkm = byte i0 + k is
// a marker's code (0xFF followed by neither 0x00 nor 0xFF: RSTn or any other marker)
// (the segment starts 16-byte aligned and its buffer is padded to whole 16-byte groups: one
// 16-byte load per thread, plus the bytes either side)
__device__ __forceinline__ void unstuff_masks(const uint8_t* __restrict__ in, uint32_t n,
                                              uint32_t i0, uint32_t& keep, uint32_t& mkm,
                                              uint32_t (&w)[4]) {
  keep = 0;
  mkm = 0;
  const uint4 v = *reinterpret_cast<const uint4*>(in + i0);
  w[0] = v.x;
  w[1] = v.y;
  w[2] = v.z;
  w[3] = v.w;
  uint32_t pv = i0 > 0 ? in[i0 - 1] : 0u;
  const uint32_t after = i0 + 16 < n ? in[i0 + 16] : 0u;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t i = i0 + k;
    const uint32_t b = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
    const uint32_t nx = k < 15 ? (w[(k + 1) >> 2] >> (8 * ((k + 1) & 3))) & 0xFFu : after;
    bool kp;
    if (pv == 0xFF && b == 0x00) {
      kp = false;  // stuffing
    } else if (pv == 0xFF && b != 0xFF) {
      kp = false;  // a marker code
      if (i < n) mkm |= 1u << k;
    } else if (b == 0xFF) {
      kp = i + 1 < n && nx == 0x00;  // data 0xFF (stuffed); else fill / marker prefix
    } else {
      kp = true;
    }
    if (kp && i < n) keep |= 1u << k;
    pv = b;
  }
}

template <typename DESC>
__global__ __launch_bounds__(1024) void jpeg_unstuff_count(const DESC* __restrict__ imgs,
                                                           const uint8_t* __restrict__ scans,
                                                           uint2* __restrict__ tcnt, int mt) {
  const DESC& D = imgs[blockIdx.y];
  const uint32_t base = blockIdx.x * UNS_TILE;
  if (base >= D.scan_len) return;  // uniform
  uint32_t keep = 0, mkm = 0, w[4];
  if (base + threadIdx.x * 16 < D.scan_len)
    unstuff_masks(scans + D.scan_off, D.scan_len, base + threadIdx.x * 16, keep, mkm, w);
  uint32_t a = __popc(keep), r = __popc(mkm);
  for (int o = 32; o > 0; o >>= 1) {
    a += (uint32_t)__shfl_xor((int)a, o);
    r += (uint32_t)__shfl_xor((int)r, o);
  }
  __shared__ uint32_t wa[16], wr[16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    wa[wv] = a;
    wr[wv] = r;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t ta = 0, tr = 0;
    for (int k = 0; k < 16; ++k) {
      ta += wa[k];
      tr += wr[k];
    }
    tcnt[(size_t)blockIdx.y * mt + blockIdx.x] = make_uint2(ta, tr);
  }
}

template <typename DESC>
__global__ __launch_bounds__(1024) void jpeg_unstuff_write(const DESC* __restrict__ imgs,
                                                           const uint8_t* __restrict__ scans,
                                                           const uint2* __restrict__ tcnt, int mt,
                                                           uint8_t* __restrict__ ub,
                                                           uint2* __restrict__ mk) {
  const DESC& D = imgs[blockIdx.y];
  const uint32_t base = blockIdx.x * UNS_TILE;
  if (base >= D.scan_len) return;  // uniform
  __shared__ uint32_t wsum[16], wrst[16], base_s[2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // kept bytes and markers of the tiles before this one
  if (wv == 0) {
    uint32_t a = 0, r = 0;
    for (int k = lane; k < (int)blockIdx.x; k += 64) {
      const uint2 c = tcnt[(size_t)blockIdx.y * mt + k];
      a += c.x;
      r += c.y;
    }
    for (int o = 32; o > 0; o >>= 1) {
      a += (uint32_t)__shfl_xor((int)a, o);
      r += (uint32_t)__shfl_xor((int)r, o);
    }
    if (lane == 0) {
      base_s[0] = a;
      base_s[1] = r;
    }
  }
  const uint8_t* in = scans + D.scan_off;
  const uint32_t i0 = base + threadIdx.x * 16;
  uint32_t keep = 0, mkm = 0, w[4] = {0u, 0u, 0u, 0u};
  if (i0 < D.scan_len) unstuff_masks(in, D.scan_len, i0, keep, mkm, w);
  // block-wide exclusive scans of the kept-byte and marker counts
  const uint32_t cntk = __popc(keep), nr = __popc(mkm);
  uint32_t inc = cntk, rinc = nr;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)inc, o), q = (uint32_t)__shfl_up((int)rinc, o);
    if (lane >= o) {
      inc += t;
      rinc += q;
    }
  }
  if (lane == 63) {
    wsum[wv] = inc;
    wrst[wv] = rinc;
  }
  __syncthreads();
  uint32_t wbase = 0, rbase = 0;
  for (int k = 0; k < wv; ++k) {
    wbase += wsum[k];
    rbase += wrst[k];
  }
  uint32_t o = base_s[0] + wbase + inc - cntk;
  uint32_t orank = base_s[1] + rbase + rinc - nr;
  uint8_t* out = ub + D.ub_off;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t b = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
    if (keep >> k & 1u) out[o++] = (uint8_t)b;
    // a marker: its code and the unstuffed offset where the data before it ends (the table's room
    // holds every restart marker of an intact file plus JPG_MK_EXTRA others)
    if (mkm >> k & 1u) {
      if (orank < D.mk_cap) mk[D.mk_off + orank] = make_uint2(o, b);
      ++orank;
    }
  }
}

// Per segment (one workgroup): its length, the zero padding behind it, and where each restart
// interval's data begins and ends (bits) -- as libjpeg reads them (jdhuff.c process_restart ->
// jdmarker.c read_restart_marker / jpeg_resync_to_restart).  The markers split the data into
// segments; interval 0 reads segment 0.  At each restart the marker ending the current segment is
// the expected RSTn (taken: the interval reads the next segment), or resync decides: action 1
// (the expected RST or one too far away) take it; action 2 (a marker below SOF0 or one of the two
// RSTs before the expected one) skip to the marker after the next segment and decide again;
// action 3 (any other marker, one of the next two RSTs, or none left: the data ended) leave it --
// the interval reads nothing and inherits the out-of-data state (JPG_IV_INHERIT in its end entry).
// An intact file takes the parallel fast path: marker r is RST(r mod 8).  Without restart
// intervals the data simply ends at the first marker: for the chunked decoder ublen says so.
template <typename DESC>
__global__ __launch_bounds__(256) void jpeg_unstuff_final(const DESC* __restrict__ imgs,
                                                          const uint2* __restrict__ tcnt, int mt,
                                                          uint8_t* __restrict__ ub,
                                                          const uint2* __restrict__ mk,
                                                          uint32_t* __restrict__ ivstart,
                                                          uint32_t* __restrict__ ivend,
                                                          uint32_t* __restrict__ ublen,
                                                          uint32_t* __restrict__ overflow) {
  const DESC& D = imgs[blockIdx.x];
  __shared__ uint32_t len_s, nmk_s, bad_s;
  if (threadIdx.x < 64) {
    const int ntiles = (int)((D.scan_len + UNS_TILE - 1) / UNS_TILE);
    uint32_t a = 0, r = 0;
    for (int k = threadIdx.x; k < ntiles; k += 64) {
      const uint2 c = tcnt[(size_t)blockIdx.x * mt + k];
      a += c.x;
      r += c.y;
    }
    for (int o = 32; o > 0; o >>= 1) {
      a += (uint32_t)__shfl_xor((int)a, o);
      r += (uint32_t)__shfl_xor((int)r, o);
    }
    if (threadIdx.x == 0) {
      len_s = a;
      nmk_s = min(r, D.mk_cap);
      bad_s = 0;
      // more markers than the table holds (nintervals + JPG_MK_EXTRA: a damaged file full of
      // stray markers): the dropped ones would resynchronise differently -- the host reports it
      if (r > D.mk_cap) *overflow = 1u;
    }
  }
  __syncthreads();
  const uint32_t len = len_s, M = nmk_s, n = (uint32_t)D.nintervals;
  const uint2* m = mk + D.mk_off;
  // segment s: [start, end) bytes and the marker that ends it (after the last one: EOI)
  auto seg_start = [&](uint32_t s) { return s == 0 ? 0u : m[s - 1].x; };
  auto seg_end = [&](uint32_t s) { return s < M ? m[s].x : len; };
  auto seg_mark = [&](uint32_t s) { return s < M ? m[s].y : 0xD9u; };
  if (n == 1) {  // no restart intervals: the data ends at the first marker
    const uint32_t e = seg_end(0);
    if (threadIdx.x < 64) ub[D.ub_off + e + threadIdx.x] = 0;
    if (threadIdx.x == 0) {
      ublen[blockIdx.x] = e;
      ivstart[D.iv_off] = 0;
      ivend[D.iv_off] = e * 8u;
    }
    return;
  }
  if (threadIdx.x < 64) ub[D.ub_off + len + threadIdx.x] = 0;
  if (threadIdx.x == 0) ublen[blockIdx.x] = len;
  // fast path: every marker is the next RSTn, no more of them than restarts
  for (uint32_t r = threadIdx.x; r < M; r += blockDim.x)
    if (m[r].y != 0xD0u + (r & 7u)) bad_s = 1;
  __syncthreads();
  if (!bad_s && M < n) {
    for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) {
      const bool has = k <= M;  // interval k reads segment k; past the data's end: nothing
      ivstart[D.iv_off + k] = has ? seg_start(k) * 8u : len * 8u;
      ivend[D.iv_off + k] = has ? seg_end(k) * 8u : len * 8u | JPG_IV_INHERIT;
    }
    return;
  }
  if (threadIdx.x != 0) return;
  // a damaged file: libjpeg's restart processing, serially
  uint32_t j = 0, want = 0;
  ivstart[D.iv_off] = 0;
  ivend[D.iv_off] = seg_end(0) * 8u;
  for (uint32_t k = 1; k < n; ++k) {
    uint32_t mc = seg_mark(j);
    int act;
    for (;;) {
      const uint32_t w0 = 0xD0u + want;
      if (mc == w0) act = 1;
      else if (mc < 0xC0u) act = 2;
      else if (mc < 0xD0u || mc > 0xD7u) act = 3;
      else if (mc == 0xD0u + ((want + 1) & 7u) || mc == 0xD0u + ((want + 2) & 7u)) act = 3;
      else if (mc == 0xD0u + ((want - 1) & 7u) || mc == 0xD0u + ((want - 2) & 7u)) act = 2;
      else act = 1;
      if (act == 2 && j < M) {
        ++j;
        mc = seg_mark(j);
        continue;
      }
      break;
    }
    want = (want + 1) & 7u;
    if (act == 1 && j < M) {
      ++j;
      ivstart[D.iv_off + k] = seg_start(j) * 8u;
      ivend[D.iv_off + k] = seg_end(j) * 8u;
    } else {
      ivstart[D.iv_off + k] = len * 8u;
      ivend[D.iv_off + k] = len * 8u | JPG_IV_INHERIT;
    }
  }
}

// Restart intervals go through the same chunked decoder: each interval is cut into its own chunks
// (its first chunk starts at the interval's known state, DC predictors 0; the others synchronise
// as a scan's do), so a file with a few long intervals is not decoded one thread per interval.
// jpeg_chunk_map_kernel (per image with restart intervals, after unstuffing): interval k gets
// max(1, ceil(bits / chunk_bits)) chunks from slot iv_ck[k] on (none if it reads nothing and
// inherits: its first MCU is its predecessor's, see jpeg_write_kernel); ck_iv[slot] names the
// interval (~0: an unused slot).  The host sized the slots for the worst case.
__global__ __launch_bounds__(256) void jpeg_chunk_map_kernel(const JpegDev* __restrict__ imgs,
                                                             const uint32_t* __restrict__ ivstart,
                                                             const uint32_t* __restrict__ ivend,
                                                             uint32_t* __restrict__ iv_ck,
                                                             uint32_t* __restrict__ ck_iv) {
  const JpegDev& D = imgs[blockIdx.x];
  if (!D.restart || D.nscan) return;  // uniform
  __shared__ uint32_t wsum[4], carry_s;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  const uint32_t n = (uint32_t)D.nintervals, cb = D.chunk_bits;
  for (uint32_t k0 = 0; k0 < n; k0 += 256) {
    const uint32_t k = k0 + threadIdx.x;
    uint32_t c = 0;
    if (k < n) {
      const uint32_t ie = ivend[D.iv_off + k];
      if (!(ie & JPG_IV_INHERIT)) c = max(1u, (ie - ivstart[D.iv_off + k] + cb - 1) / cb);
    }
    uint32_t inc = c;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = (uint32_t)__shfl_up((int)inc, o);
      if (lane >= o) inc += t;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t off = carry_s + inc - c;
    for (int w = 0; w < wv; ++w) off += wsum[w];
    if (k < n) {
      iv_ck[D.iv_off + k] = off;
      for (uint32_t q = 0; q < c && off + q < D.nchunks; ++q) ck_iv[D.ch_off + off + q] = k;
    }
    __syncthreads();
    if (threadIdx.x == 0) carry_s += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  for (uint32_t t = carry_s + threadIdx.x; t < D.nchunks; t += 256) ck_iv[D.ch_off + t] = ~0u;
}

// chunk t of image D: its bit range [b0, b1), whether it starts a restart interval (or the image's
// data: a known state) and the interval k; live = false for an unused slot
struct ChunkPos {
  bool live, first;
  uint32_t k, b0, b1, end;  // end: where the interval's (or the image's) data ends
};
__device__ __forceinline__ ChunkPos jpg_chunk_pos(const JpegDev& D, uint32_t t, uint32_t nbits,
                                                  const uint32_t* __restrict__ ck_iv,
                                                  const uint32_t* __restrict__ iv_ck,
                                                  const uint32_t* __restrict__ ivstart,
                                                  const uint32_t* __restrict__ ivend) {
  ChunkPos c;
  if (!D.restart) {
    c.live = t < D.nchunks;
    c.first = t == 0;
    c.k = 0;
    c.end = nbits;
    c.b0 = min(t * D.chunk_bits, nbits);
    c.b1 = min(c.b0 + D.chunk_bits, nbits);
    return c;
  }
  c.k = t < D.nchunks ? ck_iv[D.ch_off + t] : ~0u;
  c.live = c.k != ~0u;
  if (!c.live) {
    c.first = false;
    c.b0 = c.b1 = c.end = 0;
    return c;
  }
  const uint32_t j = t - iv_ck[D.iv_off + c.k];
  c.first = j == 0;
  c.end = ivend[D.iv_off + c.k] & ~JPG_IV_INHERIT;
  c.b0 = min(ivstart[D.iv_off + c.k] + j * D.chunk_bits, c.end);
  c.b1 = min(c.b0 + D.chunk_bits, c.end);
  return c;
}

// stage 2a/2b: sync passes.  grid (max chunks per image, n).  PASS_A: start from the chunk's
// own first bit; else from the predecessor's end state in `prev` (chunk 0: the true start).
// chg_prev / chg_next: per chunk, did its end state change in the previous / this pass.  After
// the first B pass (`all`) a chunk is decoded again only if its predecessor's end state -- its
// start -- changed; otherwise its end state and counts are those of the previous pass.  Only the
// chains still converging cost anything in the later passes.
template <bool PASS_A>
__global__ __launch_bounds__(64) void jpeg_sync_kernel(const JpegDev* __restrict__ imgs,
                                                       const uint8_t* __restrict__ ub,
                                                       const uint32_t* __restrict__ ublen,
                                                       const uint64_t* __restrict__ prev,
                                                       uint64_t* __restrict__ next,
                                                       ChunkOut* __restrict__ cnt,
                                                       uint32_t* __restrict__ changed,
                                                       const uint8_t* __restrict__ chg_prev,
                                                       uint8_t* __restrict__ chg_next, int all,
                                                       uint64_t* __restrict__ ck_st,
                                                       ChunkOut* __restrict__ ck_co,
                                                       const uint32_t* __restrict__ settled,
                                                       int badlen,
                                                       const uint32_t* __restrict__ ck_iv,
                                                       const uint32_t* __restrict__ iv_ck,
                                                       const uint32_t* __restrict__ ivstart,
                                                       const uint32_t* __restrict__ ivend) {
  __shared__ JpegLds T;
  __shared__ __attribute__((aligned(16))) uint32_t ring[64 * JRING_W];
  // the previous pass of this launch round changed nothing: the decode has converged and both
  // state buffers hold the same states (that pass copied every one through), so there is nothing
  // to do -- the host queues a round of passes without reading a flag between them
  if (!PASS_A && settled && *settled == 0u) return;
  const JpegDev& D = imgs[blockIdx.y];
  if (D.nscan || blockIdx.x * 64 >= D.nchunks) return;  // uniform per workgroup
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  const uint32_t nbits = ublen[blockIdx.y] * 8u;
  const ChunkPos cp = jpg_chunk_pos(D, t, nbits, ck_iv, iv_ck, ivstart, ivend);
  bool redo = cp.live;
  if (!PASS_A && !all) {
    redo = cp.live && !cp.first && chg_prev[D.ch_off + t - 1];
    if (cp.live && !redo) {
      next[D.ch_off + t] = prev[D.ch_off + t];
      chg_next[D.ch_off + t] = 0;
    }
    if (__ballot(redo) == 0) return;  // the whole workgroup (one wave) is settled
  }
  jpg_load_tables(T, D);
  __syncthreads();
  if (!redo) return;
  const uint32_t b0 = cp.b0, b1 = cp.b1;
  const uint64_t st = PASS_A || cp.first ? jpg_state(b0, 0, 0) : prev[D.ch_off + t - 1];
  const uint32_t nsub = jpg_nsub(D.chunk_bits);
  uint64_t* cks = ck_st + (size_t)(D.ch_off + t) * nsub;
  ChunkOut* ckc = ck_co + (size_t)(D.ch_off + t) * nsub;
  ChunkOut co{0u, {0, 0, 0}};
  int pred[3] = {0, 0, 0};
  const JpgConst K = jpg_const(D);
  const rsrc_t rs = make_rsrc(ub + D.ub_off, nbits / 8u + 64u);  // past the padding: zeros
  uint64_t e = st;
  for (uint32_t j = 0; j < nsub; ++j) {
    if (!PASS_A && e == cks[j]) {
      // joined the trajectory recorded by this chunk's last decode: its end state stands, the
      // counts from here on shift by the difference at this checkpoint
      const ChunkOut old = ckc[j];
      const int32_t dn = (int32_t)(co.nblk - old.nblk);
      const int32_t d0 = co.dcsum[0] - old.dcsum[0], d1 = co.dcsum[1] - old.dcsum[1],
                    d2 = co.dcsum[2] - old.dcsum[2];
      for (uint32_t k = j; k < nsub; ++k) {
        ChunkOut c = ckc[k];
        c.nblk += (uint32_t)dn;
        c.dcsum[0] += d0;
        c.dcsum[1] += d1;
        c.dcsum[2] += d2;
        ckc[k] = c;
      }
      const ChunkOut tot = cnt[D.ch_off + t];
      co.nblk = tot.nblk + (uint32_t)dn;
      co.dcsum[0] = tot.dcsum[0] + d0;
      co.dcsum[1] = tot.dcsum[1] + d1;
      co.dcsum[2] = tot.dcsum[2] + d2;
      e = prev[D.ch_off + t];
      break;
    }
    cks[j] = e;
    ckc[j] = co;
    const uint32_t sub_end = min(b0 + (j + 1) * JPG_SUB, b1);
    // a state past the sub-chunk (the predecessor ran over it) ends where it starts
    if ((uint32_t)e < sub_end) {
      if (D.restart)  // (uniform per workgroup) the interval's end reads as zero bits
        e = jpg_run<false, false, true>(K, T, rs, ring + threadIdx.x * JRING_W, e, sub_end, &co, 0,
                                        pred, nullptr, 0xFFFFFFFFu, false, badlen, nullptr, cp.end);
      else
        e = jpg_run<false>(K, T, rs, ring + threadIdx.x * JRING_W, e, sub_end, &co, 0, pred,
                           nullptr, 0xFFFFFFFFu, false, badlen);
    }
  }
  next[D.ch_off + t] = e;
  cnt[D.ch_off + t] = co;
  if (PASS_A) {
    chg_next[D.ch_off + t] = 1;
  } else {
    const bool ch = e != prev[D.ch_off + t];
    chg_next[D.ch_off + t] = ch ? 1 : 0;
    if (ch) changed[0] = 1u;
  }
}

// stage 2c: per image, the first block index and DC predictors of every chunk
// one 256-thread workgroup per image: exclusive scan of the chunk counts (block counts and DC
// sums add), 256 chunks per round (a serial walk per image was a ~300-step latency chain),
// segmented at the chunks that start a restart interval (DC sums from 0, blocks from the
// interval's first block)
__global__ __launch_bounds__(256) void jpeg_prefix_kernel(const JpegDev* __restrict__ imgs,
                                                          const ChunkOut* __restrict__ cnt,
                                                          ChunkOut* __restrict__ start, int n,
                                                          const uint32_t* __restrict__ ck_iv,
                                                          const uint32_t* __restrict__ iv_ck) {
  const JpegDev& D = imgs[blockIdx.x];
  if (D.nscan) return;
  __shared__ int32_t sv[4][256];
  __shared__ uint8_t sf[256];
  __shared__ int32_t carry[4];
  if (threadIdx.x < 4) carry[threadIdx.x] = 0;
  for (uint32_t t0 = 0; t0 < D.nchunks; t0 += 256) {
    const uint32_t t = t0 + threadIdx.x;
    ChunkOut c{0u, {0, 0, 0}};
    bool first = t == 0;
    uint32_t k = 0;
    if (t < D.nchunks) {
      c = cnt[D.ch_off + t];
      if (D.restart) {
        k = ck_iv[D.ch_off + t];
        first = k != ~0u && iv_ck[D.iv_off + k] == t;
        if (k == ~0u) c = ChunkOut{0u, {0, 0, 0}};
      }
    }
    const int32_t v[4] = {(int32_t)c.nblk, c.dcsum[0], c.dcsum[1], c.dcsum[2]};
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) sv[q][threadIdx.x] = v[q];
    sf[threadIdx.x] = first ? 1 : 0;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // segmented Hillis-Steele inclusive scan
      int32_t u[4] = {0, 0, 0, 0};
      uint8_t fu = 0;
      if (threadIdx.x >= (unsigned)o) {
#pragma unroll
        for (int q = 0; q < 4; ++q) u[q] = sv[q][threadIdx.x - o];
        fu = sf[threadIdx.x - o];
      }
      const uint8_t fo = sf[threadIdx.x];
      __syncthreads();
      if (!fo)
#pragma unroll
        for (int q = 0; q < 4; ++q) sv[q][threadIdx.x] += u[q];
      sf[threadIdx.x] = fo | fu;
      __syncthreads();
    }
    if (t < D.nchunks) {
      // exclusive = inclusive - own, plus the carry unless a segment started in this round
      const bool seg = sf[threadIdx.x] != 0;
      ChunkOut e;
      e.nblk = (uint32_t)((seg ? 0 : carry[0]) + sv[0][threadIdx.x] - v[0]);
#pragma unroll
      for (int q = 0; q < 3; ++q) e.dcsum[q] = (seg ? 0 : carry[q + 1]) + sv[q + 1][threadIdx.x] - v[q + 1];
      if (D.restart && k != ~0u) {
        // blocks from the interval's first one; the chunks before the interval's own start in
        // this round add nothing (the scan restarted at the interval's first chunk)
        e.nblk += k * (uint32_t)D.restart * (uint32_t)D.bpm;
      }
      start[D.ch_off + t] = e;
    }
    __syncthreads();
    if (threadIdx.x < 4)
      carry[threadIdx.x] = (sf[255] ? 0 : carry[threadIdx.x]) + sv[threadIdx.x][255];
    __syncthreads();
  }
}

// stage 2d: write pass.  Sub-chunks (grid.x over chunks x sub-chunks, from the final
// checkpoints) of images without restart markers and of each restart interval.
__global__ __launch_bounds__(64) void jpeg_write_kernel(const JpegDev* __restrict__ imgs,
                                                        const uint8_t* __restrict__ ub,
                                                        const uint32_t* __restrict__ ublen,
                                                        const uint32_t* __restrict__ ivstart,
                                                        const uint32_t* __restrict__ ivend,
                                                        const uint64_t* __restrict__ ck_st,
                                                        const ChunkOut* __restrict__ ck_co,
                                                        const ChunkOut* __restrict__ start,
                                                        int16_t* __restrict__ coef, int badlen,
                                                        uint32_t* __restrict__ badseen,
                                                        const uint32_t* __restrict__ ck_iv,
                                                        const uint32_t* __restrict__ iv_ck) {
  __shared__ JpegLds T;
  __shared__ __attribute__((aligned(16))) uint32_t ring[64 * JRING_W];
  const JpegDev& D = imgs[blockIdx.y];
  const uint32_t nsub = jpg_nsub(D.chunk_bits);
  const uint32_t nitems = D.nscan ? 0u : D.nchunks * nsub;
  if (blockIdx.x * 64 >= nitems) return;  // uniform per workgroup
  jpg_load_tables(T, D);
  __syncthreads();
  const uint32_t u = blockIdx.x * 64 + threadIdx.x;
  if (u >= nitems) return;
  const uint32_t nbits = ublen[blockIdx.y] * 8u;
  // sub-chunk j of chunk t from its checkpoint: state, first block, DC predictors.  badlen: the
  // bits a bad code takes.  libjpeg's is 17, but the sync passes converge a pass sooner with 16
  // (1.21 against 1.31 ms for a 600x1000 file: bad codes are frequent on the speculative
  // trajectories), so the host decodes with 16 first; the trajectories agree up to the first bad
  // code on the true one, which the write pass then reports (badseen) and the host decodes again
  // with 17 -- only files with a bad code in their data pay for the exact rule
  const uint32_t t = u / nsub, j = u - t * nsub;
  const ChunkPos cp = jpg_chunk_pos(D, t, nbits, ck_iv, iv_ck, ivstart, ivend);
  if (!cp.live) return;
  const uint32_t b1 = min(cp.b1, cp.b0 + (j + 1) * JPG_SUB);
  // the sub-chunk holding the last bit of the data (of the image, or of the restart interval), or
  // the first one without data, finishes the decode where the data ends
  const bool tail = cp.b0 < cp.end ? cp.b1 == cp.end && (cp.end - 1 - cp.b0) / JPG_SUB == j
                                    : cp.first && j == 0;
  const size_t k = (size_t)(D.ch_off + t) * nsub + j;
  const uint64_t st = ck_st[k];
  const ChunkOut c = ck_co[k], s0 = start[D.ch_off + t];
  int pred[3] = {s0.dcsum[0] + c.dcsum[0], s0.dcsum[1] + c.dcsum[1], s0.dcsum[2] + c.dcsum[2]};
  const int32_t blk = (int32_t)(s0.nblk + c.nblk) - 1;
  if ((uint32_t)st >= b1 && !tail) return;
  ChunkOut dummy{0u, {0, 0, 0}};
  JpgConst K = jpg_const(D);
  uint32_t* myring = ring + threadIdx.x * JRING_W;
  const rsrc_t rs = make_rsrc(ub + D.ub_off, nbits / 8u + 64u);
  if (!D.restart) {
    jpg_run<true>(K, T, rs, myring, st, b1, &dummy, blk, pred, coef, 0xFFFFFFFFu, tail, badlen,
                  badseen);
    return;
  }
  // a restart interval: its blocks only (the bits after its last MCU are padding)
  const uint32_t mcus = (uint32_t)(D.mcux * D.mcuy), R = (uint32_t)D.restart;
  const uint32_t bhi = min((cp.k + 1) * R, mcus) * (uint32_t)D.bpm;
  K.total_blocks = bhi;
  if (!tail) {
    jpg_run<true, false, true>(K, T, rs, myring, st, b1, &dummy, blk, pred, coef, 0xFFFFFFFFu,
                               false, badlen, badseen, cp.end);
    return;
  }
  // the interval's end: its MCUs to the last one, the bits past its data 0, an MCU decoded only if
  // the data lasted up to its start; then, if the next interval reads nothing and inherits the
  // out-of-data state and this one did not run out, libjpeg decodes the next one's first MCU from
  // zero bits
  const uint64_t e = jpg_run<true, true>(K, T, rs, myring, st, cp.end, &dummy, blk, pred, coef,
                                         bhi - (uint32_t)(blk + 1), false, badlen, badseen);
  if (cp.k + 1 < (uint32_t)D.nintervals && (ivend[D.iv_off + cp.k + 1] & JPG_IV_INHERIT) &&
      (uint32_t)e <= cp.end && bhi < mcus * (uint32_t)D.bpm) {
    int pz[3] = {0, 0, 0};
    K.total_blocks = min(bhi + R * (uint32_t)D.bpm, mcus * (uint32_t)D.bpm);
    jpg_run<true, true>(K, T, rs, myring, jpg_state(cp.end, 0, 0), cp.end, &dummy,
                        (int32_t)bhi - 1, pz, coef, (uint32_t)D.bpm, false, badlen, badseen);
  }
}

// ---- device: the scan path (progressive / multi-scan files) --------------------------------------
// jdhuff.c's decode_mcu (sequential), decode_mcu_DC_first / _AC_first / _DC_refine / _AC_refine
// (progressive: spectral selection, successive approximation, EOB runs), restated.  One wave per
// image walks the image's scans in file order (a refinement scan reads what the earlier scans
// left in the coefficient blocks); within a scan the lanes take the restart intervals (without
// restart markers lane 0 decodes the scan).  Throughput is not the goal of this path: it makes
// cv2.imread's progressive files decodable bit-exactly (the parallel path is the baseline one).
__device__ __forceinline__ void jpg_load_scan_tables(JpegLdsScan& T, const JpegScanDev& S) {
  const uint32_t* s = reinterpret_cast<const uint32_t*>(&S.lut[0][0]);
  uint32_t* d = reinterpret_cast<uint32_t*>(&T.lut[0][0]);
  for (int k = threadIdx.x; k < (int)(sizeof(T.lut) / 4); k += blockDim.x) d[k] = s[k];
  for (int k = threadIdx.x; k < 8 * 18; k += blockDim.x) {
    (&T.maxcode[0][0])[k] = (&S.maxcode[0][0])[k];
    (&T.valoff[0][0])[k] = (&S.valoff[0][0])[k];
  }
  for (int k = threadIdx.x; k < 8 * 256; k += blockDim.x) (&T.huffval[0][0])[k] = (&S.huffval[0][0])[k];
  for (int k = threadIdx.x; k < 8 * 8; k += blockDim.x) T.mca[k >> 3][k & 7] = jpg_mca(S.maxcode[k >> 3], k & 7);
  for (int k = threadIdx.x; k < 80; k += blockDim.x) T.natural[k] = jpg_natural[k];
}

__device__ __forceinline__ uint32_t jpg_get(BitStream& br, int s) {  // s <= 16
  br.refill();
  return br.bits(s);
}
__device__ __forceinline__ int jpg_huff(BitStream& br, const JpegLdsScan& T, int t) {
  br.refill();
  int len;
  const int sym = jpg_decode(br.acc, T, t, &len);
  br.bits(len);
  return sym;
}
__device__ __forceinline__ int16_t jpg_lshift(int v, int al) { return (int16_t)(int)((uint32_t)v << al); }

// one block of scan component k (slot k: DC table, 4 + k: AC table); eobrun / pred per interval
template <typename SK>
__device__ __forceinline__ void jpg_scan_block(BitStream& br, const JpegLdsScan& T, const SK& S,
                                               int k, int16_t* __restrict__ blk, int& pred,
                                               uint32_t& eobrun) {
  switch (S.kind) {
    case JPG_SEQ: {
      const int s = jpg_huff(br, T, k);
      pred += s ? jpg_extend(jpg_get(br, s), s) : 0;
      blk[0] = (int16_t)pred;
      for (int z = 1; z < 64;) {
        const int rs = jpg_huff(br, T, 4 + k);
        const int r = rs >> 4, sz = rs & 15;
        if (sz) {
          z += r;
          blk[T.natural[min(z, 79)]] = (int16_t)jpg_extend(jpg_get(br, sz), sz);
          ++z;
        } else if (r == 15) {
          z += 16;
        } else {
          break;
        }
      }
      break;
    }
    case JPG_DC_FIRST: {
      const int s = jpg_huff(br, T, k);
      pred += s ? jpg_extend(jpg_get(br, s), s) : 0;
      blk[0] = jpg_lshift(pred, S.Al);
      break;
    }
    case JPG_DC_REFINE:  // OR the bit into the low half of the block's first dword: no load to
                         // wait for (blk is 128-byte aligned, Al <= 13)
      if (jpg_get(br, 1)) atomicOr(reinterpret_cast<unsigned int*>(blk), 1u << S.Al);
      break;
    case JPG_AC_FIRST: {
      if (eobrun) {
        --eobrun;
        break;
      }
      for (int z = S.Ss; z <= S.Se; ++z) {
        const int rs = jpg_huff(br, T, 4);
        const int r = rs >> 4, sz = rs & 15;
        if (sz) {
          z += r;
          blk[T.natural[min(z, 79)]] = jpg_lshift(jpg_extend(jpg_get(br, sz), sz), S.Al);
        } else if (r != 15) {
          eobrun = 1u << r;
          if (r) eobrun += jpg_get(br, r);
          --eobrun;
          break;
        } else {
          z += 15;
        }
      }
      break;
    }
    default: {  // JPG_AC_REFINE
      const int p1 = 1 << S.Al, m1 = -(1 << S.Al);
      int z = S.Ss;
      if (eobrun == 0) {
        for (; z <= S.Se; ++z) {
          const int rs = jpg_huff(br, T, 4);
          int r = rs >> 4, sz = rs & 15;
          if (sz) {
            sz = jpg_get(br, 1) ? p1 : m1;
          } else if (r != 15) {
            eobrun = 1u << r;
            if (r) eobrun += jpg_get(br, r);
            break;
          }
          do {  // refine the nonzero coefficients up to the target zero (r zeros skipped)
            int16_t* c = blk + T.natural[min(z, 79)];
            if (*c != 0) {
              if (jpg_get(br, 1) && (*c & p1) == 0) *c = (int16_t)(*c >= 0 ? *c + p1 : *c + m1);
            } else if (--r < 0) {
              break;
            }
            ++z;
          } while (z <= S.Se);
          if (sz) blk[T.natural[min(z, 79)]] = (int16_t)sz;
        }
      }
      if (eobrun > 0) {  // the band of this block is in an EOB run: refine its nonzeros
        for (; z <= S.Se; ++z) {
          int16_t* c = blk + T.natural[min(z, 79)];
          if (*c != 0 && jpg_get(br, 1) && (*c & p1) == 0) *c = (int16_t)(*c >= 0 ? *c + p1 : *c + m1);
        }
        --eobrun;
      }
    }
  }
}

// a scan's constants, read once per scan: inside the unit loop a read of JpegDev / JpegScanDev
// (component fields at a computed index) was a vector load waited for at every unit
struct ScanK {
  int kind, Ss, Se, Al, ns;
  uint32_t mcux;
  uint32_t wib[4], bw[4], cv[4], ch[4];  // per scan component k
  uint64_t boff[4];                      // its first block
};
__device__ __forceinline__ ScanK jpg_scan_k(const JpegDev& D, const JpegScanDev& S) {
  ScanK K;
  K.kind = S.kind;
  K.Ss = S.Ss;
  K.Se = S.Se;
  K.Al = S.Al;
  K.ns = S.ns;
  K.mcux = (uint32_t)D.mcux;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = k < S.ns ? S.comp[k] : 0;
    K.wib[k] = (uint32_t)D.wib[c];
    K.bw[k] = (uint32_t)D.bw[c];
    K.cv[k] = (uint32_t)D.cv[c];
    K.ch[k] = (uint32_t)D.ch[c];
    K.boff[k] = D.blk_off[c];
  }
  return K;
}
template <typename A>
__device__ __forceinline__ A jpg_pick(const A (&a)[4], int k) {  // (no dynamic register index)
  return k == 0 ? a[0] : k == 1 ? a[1] : k == 2 ? a[2] : a[3];
}

// the scan path's unit u of scan S: an MCU (interleaved) or one block of the scan's component
__device__ __forceinline__ void jpg_scan_unit(BitStream& br, const JpegLdsScan& T, const ScanK& S,
                                              uint32_t u, int16_t* __restrict__ coef,
                                              int (&pred)[4], uint32_t& eobrun) {
  if (S.ns == 1) {  // non-interleaved: the component's own blocks, raster order
    const uint32_t by = u / S.wib[0], bx = u - by * S.wib[0];
    int16_t* blk = coef + (S.boff[0] + (uint64_t)by * S.bw[0] + bx) * 64;
    jpg_scan_block(br, T, S, 0, blk, pred[0], eobrun);
  } else {  // interleaved MCU (sequential, or a progressive DC scan)
    const uint32_t my = u / S.mcux, mx = u - my * S.mcux;
    for (int k = 0; k < S.ns; ++k) {
      const uint32_t cv = jpg_pick(S.cv, k), ch = jpg_pick(S.ch, k), bw = jpg_pick(S.bw, k);
      const uint64_t bo = jpg_pick(S.boff, k);
      for (uint32_t dv = 0; dv < cv; ++dv)
        for (uint32_t dh = 0; dh < ch; ++dh) {
          const uint64_t by = (uint64_t)my * cv + dv, bx = (uint64_t)mx * ch + dh;
          jpg_scan_block(br, T, S, k, coef + (bo + by * bw + bx) * 64, pred[k], eobrun);
        }
    }
  }
}

// One block of an AC refinement scan (jdhuff.c decode_mcu_AC_refine) from its nonzero history h
// (zigzag positions in the band Ss..Se, before this scan) alone: what the decoder reads never
// depends on the coefficient values, only on which are nonzero, and a new coefficient is never
// passed again in its block.  Every history position of the band gets one correction bit, in
// zigzag order (corr: the K = popcount(h) bits, the first read highest); newp / newn: the
// positions that become +-2^Al (newn: negative).  libjpeg's overrun guard writes a value past
// position 63 at 63.  The caller applies it.
struct RefineOut {
  uint64_t corr, newp, newn;
};
__device__ __forceinline__ void jpg_refine_block(BitStream& br, const JpegLdsScan& T, int Ss, int Se,
                                                 uint64_t h, uint32_t& eobrun, RefineOut& out) {
  uint64_t corr = 0, newp = 0, newn = 0;
  auto take = [&](uint64_t nz) {  // the correction bits of the history positions in nz
    for (int k = __popcll(nz); k > 0;) {
      const int s = min(k, 24);
      corr = corr << s | jpg_get(br, s);
      k -= s;
    }
  };
  int z = Ss;
  if (eobrun == 0) {
    while (z <= Se) {
      const int rs = jpg_huff(br, T, 4);
      const int r = rs >> 4, sz = rs & 15;
      bool neg = false;
      if (sz) {
        neg = jpg_get(br, 1) == 0;
      } else if (r != 15) {
        eobrun = 1u << r;
        if (r) eobrun += jpg_get(br, r);
        break;
      }
      // the (r + 1)-th position without history from z on (Se + 1 if the band runs out first)
      uint64_t zs = ~h & (~0ull << z) & (Se == 63 ? ~0ull : (1ull << (Se + 1)) - 1);
      for (int i = 0; i < r && zs; ++i) zs &= zs - 1;
      const int t = zs ? __builtin_ctzll(zs) : Se + 1;
      take(h & (~0ull << z) & (t >= 64 ? ~0ull : (1ull << t) - 1));
      if (sz) {
        const int zt = min(t, 63);
        newp |= 1ull << zt;
        newn |= (uint64_t)neg << zt;
      }
      z = t + 1;
    }
  }
  if (eobrun > 0) {
    if (z <= Se) take(h & (~0ull << z));
    --eobrun;
  }
  out = RefineOut{corr, newp, newn};
}

// Out of data (jdhuff.c insufficient_data): a unit is decoded only while the interval's data lasted
// up to its start (a skipped unit keeps what the earlier scans left); an interval that reads
// nothing and inherits the out-of-data state is the predecessor's lane's: it decodes the first unit
// from zero bits if the predecessor did not run out (see jpeg_unstuff_final).
// A non-interleaved scan without restart intervals (every AC scan) decodes on one lane into blocks
// the wave stages JPG_PT at a time in LDS (loaded, decoded into, written back): an AC refinement
// read every block's earlier coefficients as it went, a dependent HBM round trip each, and on gfx9
// the bit reader's waits for its loads (vmcnt) also waited for every coefficient store before.
constexpr uint32_t JPG_PT = 256;
__global__ __launch_bounds__(64) void jpeg_prog_kernel(const JpegDev* __restrict__ imgs,
                                                       const JpegScanDev* __restrict__ scans,
                                                       const uint8_t* __restrict__ ub,
                                                       const uint32_t* __restrict__ ivstart,
                                                       const uint32_t* __restrict__ ivend,
                                                       const uint32_t* __restrict__ ublen_s,
                                                       int16_t* __restrict__ coef) {
  __shared__ JpegLdsScan T;
  __shared__ uint4 tile[JPG_PT * 8];  // JPG_PT blocks of 64 coefficients
  __shared__ uint64_t ref_hist[JPG_PT];
  __shared__ RefineOut ref_out[JPG_PT];
  __shared__ __attribute__((aligned(16))) uint32_t bring[64 * JRING_S];
  uint32_t* myring = bring + threadIdx.x * JRING_S;
  const JpegDev& D = imgs[blockIdx.x];
  const uint32_t nscan = D.nscan;
  if (nscan == 0 || D.arith) return;  // uniform: a parallel-path or arithmetic-coded image
  for (uint32_t si = 0; si < nscan; ++si) {
    const JpegScanDev& S = scans[D.scan0 + si];
    // the previous scan's coefficient stores visible to every lane, its table reads done
    __threadfence();
    __syncthreads();
    jpg_load_scan_tables(T, S);
    __syncthreads();
    const rsrc_t rs = make_rsrc(ub + S.ub_off, ublen_s[D.scan0 + si] + 64u);
    const ScanK K = jpg_scan_k(D, S);
    if (S.ns == 1 && S.nintervals == 1) {  // (interval 0 never inherits)
      const uint32_t ie = ivend[S.iv_off];
      const int c = S.comp[0];
      const uint32_t wib = (uint32_t)D.wib[c], bw = (uint32_t)D.bw[c];
      int16_t* cb = coef + D.blk_off[c] * 64;
      const uint64_t band = (S.Se == 63 ? ~0ull : (1ull << (S.Se + 1)) - 1) & (~0ull << S.Ss);
      const int p1 = 1 << S.Al, m1 = -(1 << S.Al);
      const bool refine = S.kind == JPG_AC_REFINE;
      BitStream br;
      if (threadIdx.x == 0) br.start(rs, myring, ivstart[S.iv_off], ie);
      uint32_t eobrun = 0;
      int pred = 0;
      for (uint32_t t0 = 0; t0 < S.nunits; t0 += JPG_PT) {
        const uint32_t nt = min(JPG_PT, S.nunits - t0);
        // 16-byte piece k of the tile: part k % 8 of its block k / 8
        for (uint32_t k = threadIdx.x; k < nt * 8; k += 64) {
          const uint32_t u = t0 + k / 8, by = u / wib, bx = u - by * wib;
          tile[k] = reinterpret_cast<const uint4*>(cb + ((uint64_t)by * bw + bx) * 64)[k % 8];
        }
        __syncthreads();
        if (!refine) {  // the other kinds read nothing back: the blocks in LDS, one lane
          if (threadIdx.x == 0)
            for (uint32_t u = 0; u < nt && br.pos <= ie; ++u)
              jpg_scan_block(br, T, K, 0, reinterpret_cast<int16_t*>(tile + 8 * u), pred, eobrun);
        }
        const int16_t* tb = reinterpret_cast<const int16_t*>(tile);
        for (uint32_t u = threadIdx.x; u < nt && refine; u += 64) {  // nonzero history, zigzag
          uint64_t h = 0;
          for (int zz = 0; zz < 64; ++zz) h |= (uint64_t)(tb[u * 64 + T.natural[zz]] != 0) << zz;
          ref_hist[u] = h & band;
        }
        __syncthreads();
        if (threadIdx.x == 0 && refine) {
          uint32_t u = 0;
          for (; u < nt && br.pos <= ie; ++u)
            jpg_refine_block(br, T, S.Ss, S.Se, ref_hist[u], eobrun, ref_out[u]);
          for (; u < nt; ++u) ref_out[u] = RefineOut{0ull, 0ull, 0ull};  // out of data: unchanged
        }
        __syncthreads();
        for (uint32_t u = threadIdx.x; u < nt && refine; u += 64) {  // corrections, then new ones
          int16_t* blk = reinterpret_cast<int16_t*>(tile + 8 * u);
          const RefineOut o = ref_out[u];
          uint64_t h = ref_hist[u];
          for (int j = __popcll(h) - 1; h; h &= h - 1, --j) {
            if (!((o.corr >> j) & 1u)) continue;
            int16_t* cp = blk + T.natural[__builtin_ctzll(h)];
            if ((*cp & p1) == 0) *cp = (int16_t)(*cp >= 0 ? *cp + p1 : *cp + m1);
          }
          for (uint64_t nw = o.newp; nw; nw &= nw - 1) {
            const int zz = __builtin_ctzll(nw);
            blk[T.natural[zz]] = (int16_t)((o.newn >> zz) & 1u ? m1 : p1);
          }
        }
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < nt * 8; k += 64) {
          const uint32_t u = t0 + k / 8, by = u / wib, bx = u - by * wib;
          reinterpret_cast<uint4*>(cb + ((uint64_t)by * bw + bx) * 64)[k % 8] = tile[k];
        }
        __syncthreads();
      }
      continue;
    }
    for (int t = threadIdx.x; t < S.nintervals; t += 64) {
      const uint32_t ie = ivend[S.iv_off + t];
      if (ie & JPG_IV_INHERIT) continue;
      const uint32_t u0 = S.restart ? (uint32_t)t * (uint32_t)S.restart : 0u;
      const uint32_t u1 = S.restart ? min(u0 + (uint32_t)S.restart, S.nunits) : S.nunits;
      BitStream br;
      br.start(rs, myring, ivstart[S.iv_off + t], ie);
      int pred[4] = {0, 0, 0, 0};
      uint32_t eobrun = 0;
      for (uint32_t u = u0; u < u1 && br.pos <= ie; ++u) jpg_scan_unit(br, T, K, u, coef, pred, eobrun);
      if (t + 1 < S.nintervals && (ivend[S.iv_off + t + 1] & JPG_IV_INHERIT) && br.pos <= ie &&
          u1 < S.nunits) {
        int pz[4] = {0, 0, 0, 0};
        uint32_t ez = 0;
        br.start(rs, myring, ie, ie);
        jpg_scan_unit(br, T, K, u1, coef, pz, ez);
      }
    }
  }
}

// ---- device: arithmetic-coded scans (jdarith.c, libjpeg 9d) ------------------------------------
// The QM-coder (ITU-T T.81 Annex D) over each restart interval's unstuffed bytes, with libjpeg's
// statistics per table (DC: 64 bins, AC: 256) reset at every interval, the DC conditioning of
// the DAC parameters (L, U) and the AC split K, restated: decode_mcu (sequential) and
// decode_mcu_DC_first / _AC_first / _DC_refine / _AC_refine.  The structure is the scan path's:
// one wave per image, scans in file order, lanes over restart intervals (one lane without them:
// an arithmetic-coded file decodes serially -- correct, not fast; such files are rare).
#include "jpeg_aritab.inc"  // jpg_aritab[114]: T.81 Table D.2 + the fixed 0.5 state 113

constexpr int JAR_DC = 64, JAR_AC = 256, JAR_LANE = 4 * JAR_DC + 4 * JAR_AC;  // stats bytes per lane

struct ArithDec {
  const uint8_t* p;
  uint32_t i, end;  // byte cursor and the interval's end (past it libjpeg reads 0)
  long long c;      // libjpeg's INT32 registers (long)
  int a, ct;
  bool bad;         // JWRN_ARITH_BAD_CODE: the rest of the interval decodes nothing
};

__device__ __forceinline__ int jar_decode(ArithDec& e, uint8_t* st) {
  while (e.a < 0x8000) {  // renormalisation and data input (D.2.6)
    if (--e.ct < 0) {
      const int data = e.i < e.end ? (int)e.p[e.i] : 0;
      ++e.i;
      e.c = (e.c << 8) | data;
      if ((e.ct += 8) < 0 && ++e.ct == 0) e.a = 0x8000;  // 2 initial bytes: a = 0x10000 below
    }
    e.a <<= 1;
  }
  int sv = *st;
  const uint32_t qv = jpg_aritab[sv & 0x7F];
  const int nl = (int)(qv & 0xFF), nm = (int)((qv >> 8) & 0xFF), qe = (int)(qv >> 16);
  const int temp = e.a - qe;
  e.a = temp;
  const long long t2 = (long long)temp << e.ct;
  if (e.c >= t2) {  // LPS path, with the conditional exchange (D.2.4 / D.2.5)
    e.c -= t2;
    if (e.a < qe) {
      e.a = qe;
      *st = (uint8_t)((sv & 0x80) ^ nm);
    } else {
      e.a = qe;
      *st = (uint8_t)((sv & 0x80) ^ nl);
      sv ^= 0x80;
    }
  } else if (e.a < 0x8000) {  // MPS path, conditional exchange
    if (e.a < qe) {
      *st = (uint8_t)((sv & 0x80) ^ nl);
      sv ^= 0x80;
    } else {
      *st = (uint8_t)((sv & 0x80) ^ nm);
    }
  }
  return sv >> 7;
}

// a DC difference (Figures F.19, F.21-F.24), updating the component's conditioning ctx
__device__ int jar_dc_diff(ArithDec& e, uint8_t* dcs, int& ctx, int L, int U) {
  uint8_t* st = dcs + ctx;
  if (jar_decode(e, st) == 0) {
    ctx = 0;
    return 0;
  }
  const int sign = jar_decode(e, st + 1);
  st += 2 + sign;
  int m = jar_decode(e, st);
  if (m) {
    st = dcs + 20;  // X1
    while (jar_decode(e, st)) {
      if ((m <<= 1) == 0x8000) {
        e.bad = true;
        return 0;
      }
      ++st;
    }
  }
  if (m < ((1 << L) >> 1)) ctx = 0;
  else if (m > ((1 << U) >> 1)) ctx = 12 + sign * 4;
  else ctx = 4 + sign * 4;
  int v = m;
  st += 14;
  while (m >>= 1)
    if (jar_decode(e, st)) v |= m;
  v += 1;
  return sign ? -v : v;
}

// an AC coefficient's value once its position k is known (st: the bins of its run, 3 (k - 1))
__device__ int jar_ac_value(ArithDec& e, uint8_t* acs, uint8_t* st, int k, int K, uint8_t* fixed) {
  const int sign = jar_decode(e, fixed);
  st += 2;
  int m = jar_decode(e, st);
  if (m && jar_decode(e, st)) {
    m <<= 1;
    st = acs + (k <= K ? 189 : 217);
    while (jar_decode(e, st)) {
      if ((m <<= 1) == 0x8000) {
        e.bad = true;
        return 0;
      }
      ++st;
    }
  }
  int v = m;
  st += 14;
  while (m >>= 1)
    if (jar_decode(e, st)) v |= m;
  v += 1;
  return sign ? -v : v;
}

// one block of scan component k
__device__ void jar_block(ArithDec& e, const JpegScanDev& S, int k, uint8_t* dcs, uint8_t* acs,
                          uint8_t* fixed, int16_t* __restrict__ blk, int& last, int& ctx,
                          const uint8_t* nat) {
  const bool prog = S.kind != JPG_SEQ;
  if (S.kind == JPG_SEQ || S.kind == JPG_DC_FIRST) {
    last += jar_dc_diff(e, dcs, ctx, S.aL[k], S.aU[k]);
    if (e.bad) return;
    blk[0] = jpg_lshift(last, prog ? S.Al : 0);
    if (prog) return;
    int z = 0;  // sequential: AC 1..63
    while (z < 63) {
      uint8_t* st = acs + 3 * z;
      if (jar_decode(e, st)) break;  // EOB
      for (;;) {
        ++z;
        if (jar_decode(e, st + 1)) break;
        st += 3;
        if (z >= 63) {
          e.bad = true;
          return;
        }
      }
      const int v = jar_ac_value(e, acs, st, z, S.aK[k], fixed);
      if (e.bad) return;
      blk[nat[z]] = (int16_t)v;
    }
  } else if (S.kind == JPG_DC_REFINE) {
    if (jar_decode(e, fixed)) blk[0] = (int16_t)(blk[0] | (1 << S.Al));
  } else if (S.kind == JPG_AC_FIRST) {
    int z = S.Ss - 1;
    while (z < S.Se) {
      uint8_t* st = acs + 3 * z;
      if (jar_decode(e, st)) break;
      for (;;) {
        ++z;
        if (jar_decode(e, st + 1)) break;
        st += 3;
        if (z >= S.Se) {
          e.bad = true;
          return;
        }
      }
      const int v = jar_ac_value(e, acs, st, z, S.aK[k], fixed);
      if (e.bad) return;
      blk[nat[z]] = jpg_lshift(v, S.Al);
    }
  } else {  // AC refine
    const int p1 = 1 << S.Al, m1 = -(1 << S.Al);
    int kex = S.Se;  // the previous stage's end of block
    while (kex > 0 && blk[nat[kex]] == 0) --kex;
    int z = S.Ss - 1;
    while (z < S.Se) {
      uint8_t* st = acs + 3 * z;
      if (z >= kex && jar_decode(e, st)) break;
      for (;;) {
        int16_t* c = blk + nat[++z];
        if (*c) {  // previously nonzero: a correction bit
          if (jar_decode(e, st + 2)) *c = (int16_t)(*c < 0 ? *c + m1 : *c + p1);
          break;
        }
        if (jar_decode(e, st + 1)) {  // newly nonzero
          *c = (int16_t)(jar_decode(e, fixed) ? m1 : p1);
          break;
        }
        st += 3;
        if (z >= S.Se) {
          e.bad = true;
          return;
        }
      }
    }
  }
}

__global__ __launch_bounds__(64) void jpeg_arith_kernel(const JpegDev* __restrict__ imgs,
                                                        const JpegScanDev* __restrict__ scans,
                                                        const uint8_t* __restrict__ ub,
                                                        const uint32_t* __restrict__ ivstart,
                                                        const uint32_t* __restrict__ ivend,
                                                        int16_t* __restrict__ coef) {
  __shared__ uint8_t stats[64 * JAR_LANE];
  __shared__ uint8_t nat[80];  // jpg_natural in LDS
  for (int k = threadIdx.x; k < 80; k += 64) nat[k] = jpg_natural[k];
  const JpegDev& D = imgs[blockIdx.x];
  const uint32_t nscan = D.nscan;
  if (nscan == 0 || !D.arith) return;  // uniform
  uint8_t* mine = stats + threadIdx.x * JAR_LANE;
  for (uint32_t si = 0; si < nscan; ++si) {
    const JpegScanDev& S = scans[D.scan0 + si];
    // the previous scan's coefficient stores visible to every lane
    __threadfence();
    __syncthreads();
    for (int t = threadIdx.x; t < S.nintervals; t += 64) {
      const uint32_t u0 = S.restart ? (uint32_t)t * (uint32_t)S.restart : 0u;
      const uint32_t u1 = S.restart ? min(u0 + (uint32_t)S.restart, S.nunits) : S.nunits;
      for (int k = 0; k < JAR_LANE; k += 16) *reinterpret_cast<uint4*>(mine + k) = make_uint4(0, 0, 0, 0);
      ArithDec e;
      e.p = ub + S.ub_off;
      // (jdarith.c has no out-of-data state: past its data an interval decodes zeros)
      e.i = ivstart[S.iv_off + t] >> 3;
      e.end = (ivend[S.iv_off + t] & ~JPG_IV_INHERIT) >> 3;
      e.c = 0;
      e.a = 0;
      e.ct = -16;
      e.bad = false;
      uint8_t fixed = 113;
      int last[4] = {0, 0, 0, 0}, ctx[4] = {0, 0, 0, 0};
      for (uint32_t u = u0; u < u1 && !e.bad; ++u) {
        if (S.ns == 1) {
          const int c = S.comp[0];
          const uint32_t by = u / (uint32_t)D.wib[c], bx = u - by * (uint32_t)D.wib[c];
          int16_t* blk = coef + (D.blk_off[c] + (uint64_t)by * D.bw[c] + bx) * 64;
          jar_block(e, S, 0, mine + S.td[0] * JAR_DC, mine + 4 * JAR_DC + S.ta[0] * JAR_AC, &fixed,
                    blk, last[0], ctx[0], nat);
        } else {
          const uint32_t my = u / (uint32_t)D.mcux, mx = u - my * (uint32_t)D.mcux;
          for (int k = 0; k < S.ns && !e.bad; ++k) {
            const int c = S.comp[k];
            for (int dv = 0; dv < D.cv[c]; ++dv)
              for (int dh = 0; dh < D.ch[c] && !e.bad; ++dh) {
                const uint64_t by = (uint64_t)my * D.cv[c] + dv, bx = (uint64_t)mx * D.ch[c] + dh;
                int16_t* blk = coef + (D.blk_off[c] + by * D.bw[c] + bx) * 64;
                jar_block(e, S, k, mine + S.td[k] * JAR_DC, mine + 4 * JAR_DC + S.ta[k] * JAR_AC,
                          &fixed, blk, last[k], ctx[k], nat);
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

// 16-point IDCT kernel of jidctint.c's jpeg_idct_16x16 / jpeg_idct_16x8 (libjpeg 9, cK =
// sqrt(2) cos(K pi / 32)): 8 coefficients -> 16 samples.  Pass 1 (columns) descales by
// CONST_BITS - PASS1_BITS, pass 2 (ROW) by CONST_BITS + PASS1_BITS + 3; libjpeg 9 folds the
// rounding fudge (and the range centre) into the DC term, which equals rounding at the end.
template <bool ROW>
__device__ __forceinline__ void jpg_idct16(const int (&x)[8], int (&o)[16]) {
  // even part
  int tmp0 = x[0] * (1 << JCB);
  int z1 = x[4];
  int tmp1 = z1 * 10703;   // FIX(1.306562965)   c4[16] = c2[8]
  int tmp2 = z1 * 4433;    // FIX_0_541196100    c12[16] = c6[8]
  int tmp10 = tmp0 + tmp1, tmp11 = tmp0 - tmp1, tmp12 = tmp0 + tmp2, tmp13 = tmp0 - tmp2;
  z1 = x[2];
  int z2 = x[6];
  int z3 = z1 - z2;
  int z4 = z3 * 2260;      // FIX(0.275899379)   c14[16] = c7[8]
  z3 = z3 * 11363;         // FIX(1.387039845)   c2[16] = c1[8]
  tmp0 = z3 + z2 * 20995;  // FIX_2_562915447    (c6+c2)[16]
  tmp1 = z4 + z1 * 7373;   // FIX_0_899976223    (c6-c14)[16]
  tmp2 = z3 - z1 * 4926;   // FIX(0.601344887)   (c2-c10)[16]
  int tmp3 = z4 - z2 * 4176;  // FIX(0.509795579) (c10-c14)[16]
  const int tmp20 = tmp10 + tmp0, tmp27 = tmp10 - tmp0;
  const int tmp21 = tmp12 + tmp1, tmp26 = tmp12 - tmp1;
  const int tmp22 = tmp13 + tmp2, tmp25 = tmp13 - tmp2;
  const int tmp23 = tmp11 + tmp3, tmp24 = tmp11 - tmp3;
  // odd part
  z1 = x[1];
  z2 = x[3];
  z3 = x[5];
  z4 = x[7];
  tmp11 = z1 + z3;
  tmp1 = (z1 + z2) * 11086;  // FIX(1.353318001) c3
  tmp2 = tmp11 * 10217;      // FIX(1.247225013) c5
  tmp3 = (z1 + z4) * 8956;   // FIX(1.093201867) c7
  tmp10 = (z1 - z4) * 7350;  // FIX(0.897167586) c9
  tmp11 = tmp11 * 5461;      // FIX(0.666655658) c11
  tmp12 = (z1 - z2) * 3363;  // FIX(0.410524528) c13
  tmp0 = tmp1 + tmp2 + tmp3 - z1 * 18730;     // FIX(2.286341144) c7+c5+c3-c1
  tmp13 = tmp10 + tmp11 + tmp12 - z1 * 15038; // FIX(1.835730603) c9+c11+c13-c15
  z1 = (z2 + z3) * 1136;                      // FIX(0.138617169) c15
  tmp1 += z1 + z2 * 589;                      // FIX(0.071888074) c9+c11-c3-c15
  tmp2 += z1 - z3 * 9222;                     // FIX(1.125726048) c5+c7+c15-c3
  z1 = (z3 - z2) * 11529;                     // FIX(1.407403738) c1
  tmp11 += z1 - z3 * 6278;                    // FIX(0.766367282) c1+c11-c9-c13
  tmp12 += z1 + z2 * 16154;                   // FIX(1.971951411) c1+c5+c13-c7
  z2 += z4;
  z1 = z2 * -5461;                            // -c11
  tmp1 += z1;
  tmp3 += z1 + z4 * 8728;                     // FIX(1.065388962) c3+c11+c15-c7
  z2 = z2 * -10217;                           // -c5
  tmp10 += z2 + z4 * 25733;                   // FIX(3.141271809) c1+c5+c9-c13
  tmp12 += z2;
  z2 = (z3 + z4) * -11086;                    // -c3
  tmp2 += z2;
  tmp3 += z2;
  z2 = (z4 - z3) * 3363;                      // c13
  tmp10 += z2;
  tmp11 += z2;
  constexpr int SH = ROW ? JCB + JP1 + 3 : JCB - JP1;
  o[0] = jpg_descale(tmp20 + tmp0, SH);
  o[15] = jpg_descale(tmp20 - tmp0, SH);
  o[1] = jpg_descale(tmp21 + tmp1, SH);
  o[14] = jpg_descale(tmp21 - tmp1, SH);
  o[2] = jpg_descale(tmp22 + tmp2, SH);
  o[13] = jpg_descale(tmp22 - tmp2, SH);
  o[3] = jpg_descale(tmp23 + tmp3, SH);
  o[12] = jpg_descale(tmp23 - tmp3, SH);
  o[4] = jpg_descale(tmp24 + tmp10, SH);
  o[11] = jpg_descale(tmp24 - tmp10, SH);
  o[5] = jpg_descale(tmp25 + tmp11, SH);
  o[10] = jpg_descale(tmp25 - tmp11, SH);
  o[6] = jpg_descale(tmp26 + tmp12, SH);
  o[9] = jpg_descale(tmp26 - tmp12, SH);
  o[7] = jpg_descale(tmp27 + tmp13, SH);
  o[8] = jpg_descale(tmp27 - tmp13, SH);
}

// libjpeg 9d block smoothing (jdcoefct.c decompress_smooth_data) of block (bx, by) of component
// c, on its dequantised coefficients x: a coefficient among AC01 AC10 AC20 AC11 AC02 whose
// coef_bits latch Al != 0 and whose value is still 0 is estimated from the quantised DC values
// DC1..DC9 of the 3x3 blocks around it (rows above / own / below; edge blocks repeat at the
// image's data edges, width_in_blocks x height_in_blocks):
//   num = mult Q00 term,  pred = ((Qk << 7) + |num|) / (Qk << 8), capped at 2^Al - 1 for Al > 0,
//   signed as num, stored as a 16-bit JCOEF; then dequantised like the coded coefficients.
// The estimates never feed a neighbour (libjpeg smooths a copy of each block).
__device__ __forceinline__ void jpg_smooth(const JpegDev& D, int c, const int16_t* cc, int bx,
                                           int by, const uint16_t* q, int (&x)[64]) {
  const int bw = D.bw[c], xl = D.wib[c] - 1, yl = D.hib[c] - 1;
  const int xs[3] = {max(bx - 1, 0), bx, min(bx + 1, xl)};
  const int ys[3] = {max(by - 1, 0), by, min(by + 1, yl)};
  long long dc[9];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int k = 0; k < 3; ++k) dc[3 * r + k] = cc[((size_t)ys[r] * bw + xs[k]) * 64];
  const long long q00 = q[0];
  auto est = [&](int z, int pos, long long num) {
    const int al = D.cbits[c][z];
    if (al == 0 || x[pos] != 0) return;  // q[pos] != 0 (smoothing_ok): x == 0 iff the coefficient is
    const long long qk = q[pos];
    long long pred = ((qk << 7) + (num >= 0 ? num : -num)) / (qk << 8);
    if (al > 0 && pred >= (1ll << al)) pred = (1ll << al) - 1;
    if (num < 0) pred = -pred;
    x[pos] = (int)(int16_t)pred * (int)qk;
  };
  est(1, 1, 36 * q00 * (dc[3] - dc[5]));                      // AC01: DC4 - DC6
  est(2, 8, 36 * q00 * (dc[1] - dc[7]));                      // AC10: DC2 - DC8
  est(3, 16, 9 * q00 * (dc[1] + dc[7] - 2 * dc[4]));          // AC20
  est(4, 9, 5 * q00 * (dc[0] - dc[2] - dc[6] + dc[8]));       // AC11
  est(5, 2, 9 * q00 * (dc[3] + dc[5] - 2 * dc[4]));           // AC02
}

// one thread per coefficient block of components whose IDCT output is (8 SV) x (8 SH) samples;
// blocks of all components of all images in one flat index space (blocks of other scales exit)
template <int SV, int SH>
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
  if (D.sv[c] != SV || D.sh[c] != SH) return;
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
  if (D.smooth && bx < D.wib[c] && by < D.hib[c])
    jpg_smooth(D, c, coef + D.blk_off[c] * 64, bx, by, q, x);
  constexpr int R = 8 * SV, C = 8 * SH;  // output rows, columns
  int ws[R * 8];
#pragma unroll
  for (int col = 0; col < 8; ++col) {  // pass 1: columns (the all-zero-AC shortcut is exact)
    if constexpr (SV == 1) {
      int o[8];
      jpg_idct1<false>(x[col], x[8 + col], x[16 + col], x[24 + col], x[32 + col], x[40 + col],
                       x[48 + col], x[56 + col], o);
#pragma unroll
      for (int r = 0; r < 8; ++r) ws[8 * r + col] = o[r];
    } else {
      const int xi[8] = {x[col], x[8 + col], x[16 + col], x[24 + col], x[32 + col], x[40 + col],
                         x[48 + col], x[56 + col]};
      int o[16];
      jpg_idct16<false>(xi, o);
#pragma unroll
      for (int r = 0; r < 16; ++r) ws[8 * r + col] = o[r];
    }
  }
  const int pw = D.pw[c];
  uint8_t* out = planes + D.pl_off[c] + (uint64_t)(by * R) * pw + bx * C;
#pragma unroll
  for (int r = 0; r < R; ++r) {  // pass 2: rows
    int o[C];
    if constexpr (SH == 1) {
      jpg_idct1<true>(ws[8 * r], ws[8 * r + 1], ws[8 * r + 2], ws[8 * r + 3], ws[8 * r + 4],
                      ws[8 * r + 5], ws[8 * r + 6], ws[8 * r + 7], o);
    } else {
      const int xi[8] = {ws[8 * r], ws[8 * r + 1], ws[8 * r + 2], ws[8 * r + 3], ws[8 * r + 4],
                         ws[8 * r + 5], ws[8 * r + 6], ws[8 * r + 7]};
      jpg_idct16<true>(xi, o);
    }
    uint32_t wd[C / 4];
#pragma unroll
    for (int j = 0; j < C / 4; ++j)
      wd[j] = jpg_range(o[4 * j]) | jpg_range(o[4 * j + 1]) << 8 | jpg_range(o[4 * j + 2]) << 16 |
              jpg_range(o[4 * j + 3]) << 24;
    uint8_t* orow = out + (uint64_t)r * pw;
    if constexpr (SH == 1) {
      reinterpret_cast<uint2*>(orow)[0] = make_uint2(wd[0], wd[1]);
    } else {
      reinterpret_cast<uint4*>(orow)[0] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    }
  }
}

// ---- device: upsampling + colour ---------------------------------------------------------------
__device__ __forceinline__ uint32_t jpg_clamp(int v) { return (uint32_t)min(max(v, 0), 255); }

// 8 consecutive pixels of a row per thread from dword loads: Y 2 dwords, each chroma row 2 dwords
// (full-size planes) or 3 dwords (the samples the 8 outputs' fancy upsampling needs, columns
// x0/2 - 1 .. x0/2 + 4 for turbo's h2 forms); jdsample.c's h2v1 / h2v2 formulas on the extracted
// samples, jdcolor.c's integer tables.
__device__ __forceinline__ uint32_t ld_dw(const uint8_t* __restrict__ row, int col4, int pw) {
  return (col4 >= 0 && col4 < pw) ? *reinterpret_cast<const uint32_t*>(row + col4) : 0u;
}
// the 12 samples of chroma row r at columns cb .. cb + 11 (cb = x0/2 - 4, dword aligned)
struct C12 {
  uint32_t d[3];
  __device__ __forceinline__ int at(int k) const { return (int)((d[k >> 2] >> (8 * (k & 3))) & 0xFFu); }
};
template <int HS, int VS>  // chroma subsampling factors (1 or 2)
__device__ __forceinline__ void jpg_chroma8(const uint8_t* __restrict__ P, int pw, int dw, int dh,
                                            int x0, int y, int (&out)[8]) {
  if constexpr (HS == 1) {  // 4:4:4
    const uint8_t* r = P + (int64_t)y * pw;
    const uint32_t a = ld_dw(r, x0, pw), b = ld_dw(r, x0 + 4, pw);
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = (int)(((k < 4 ? a : b) >> (8 * (k & 3))) & 0xFFu);
    return;
  }
  const int cb = x0 / 2 - 4;  // x0 % 8 == 0: dword aligned
  const int inrow = VS == 2 ? y >> 1 : y;
  C12 r0, r1;
  const uint8_t* p0 = P + (int64_t)inrow * pw;
#pragma unroll
  for (int j = 0; j < 3; ++j) r0.d[j] = ld_dw(p0, cb + 4 * j, pw);
  if constexpr (VS == 2) {
    const int other = min(max((y & 1) ? inrow + 1 : inrow - 1, 0), dh - 1);
    const uint8_t* p1 = P + (int64_t)other * pw;
#pragma unroll
    for (int j = 0; j < 3; ++j) r1.d[j] = ld_dw(p1, cb + 4 * j, pw);
  }
  // column sum of sample k (k = col - cb): h2v1 the sample, h2v2 3 * nearer + further row
  auto cs = [&](int k) { return VS == 2 ? r0.at(k) * 3 + r1.at(k) : r0.at(k); };
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int col = x0 / 2 + (i >> 1), k = 4 + (i >> 1);
    const int t = cs(k);
    if constexpr (VS == 2) {
      if ((i & 1) == 0) out[i] = col == 0 ? (t * 4 + 8) >> 4 : (t * 3 + cs(k - 1) + 8) >> 4;
      else out[i] = col == dw - 1 ? (t * 4 + 7) >> 4 : (t * 3 + cs(k + 1) + 7) >> 4;
    } else {
      if ((i & 1) == 0) out[i] = col == 0 ? t : (t * 3 + cs(k - 1) + 1) >> 2;
      else out[i] = col == dw - 1 ? t : (t * 3 + cs(k + 1) + 2) >> 2;
    }
  }
}

template <int HS, int VS, bool GRAY>
__device__ __forceinline__ void jpg_color8(const JpegDev& D, const uint8_t* __restrict__ planes,
                                           int x0, int y, uint32_t (&o)[6]) {
  const int pw0 = D.pw[0];
  const uint8_t* yr = planes + D.pl_off[0] + (int64_t)y * pw0;
  const uint32_t ya = ld_dw(yr, x0, pw0), yb = ld_dw(yr, x0 + 4, pw0);
  int cbv[8], crv[8];
  if constexpr (!GRAY) {
    jpg_chroma8<HS, VS>(planes + D.pl_off[1], D.pw[1], D.dw[1], D.dh[1], x0, y, cbv);
    jpg_chroma8<HS, VS>(planes + D.pl_off[2], D.pw[2], D.dw[2], D.dh[2], x0, y, crv);
  }
  uint32_t px[24];
  const int cbg = D.cb_g;  // jdcolor.c build_ycc_rgb_table (SCALEBITS 16)
  uint32_t ka = 0, kb = 0;  // a fourth component (K), sampled as the first
  if (!GRAY && D.ncomp == 4) {
    const int pw3 = D.pw[3];
    const uint8_t* kr = planes + D.pl_off[3] + (int64_t)y * pw3;
    ka = ld_dw(kr, x0, pw3);
    kb = ld_dw(kr, x0 + 4, pw3);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int Y = (int)(((i < 4 ? ya : yb) >> (8 * (i & 3))) & 0xFFu);
    if constexpr (GRAY) {
      px[3 * i] = px[3 * i + 1] = px[3 * i + 2] = (uint32_t)Y;
    } else if (D.rgb == 1) {  // jdcolor.c rgb_convert: a copy (components R, G, B -> BGR)
      px[3 * i + 0] = (uint32_t)crv[i];
      px[3 * i + 1] = (uint32_t)cbv[i];
      px[3 * i + 2] = (uint32_t)Y;
    } else if (D.rgb >= 2) {
      // libjpeg's CMYK output: the components as stored (CMYK), or jdcolor.c ycck_cmyk_convert
      // (YCCK: 255 minus the YCbCr -> RGB conversion, K unchanged); then OpenCV's
      // icvCvt_CMYK2BGR_8u_C4C3R (grfmt_jpeg.cpp: Adobe-inverted CMYK), c' = k - ((255 - c) k >> 8)
      int c0 = Y, c1 = cbv[i], c2 = crv[i];
      if (D.rgb == 3) {
        const int xb = cbv[i] - 128, xr = crv[i] - 128;
        c0 = 255 - (int)jpg_clamp(Y + ((91881 * xr + 32768) >> 16));
        c1 = 255 - (int)jpg_clamp(Y + ((-46802 * xr + (-cbg * xb + 32768)) >> 16));
        c2 = 255 - (int)jpg_clamp(Y + ((116130 * xb + 32768) >> 16));
      }
      const int k = (int)(((i < 4 ? ka : kb) >> (8 * (i & 3))) & 0xFFu);
      px[3 * i + 0] = (uint32_t)(k - (((255 - c2) * k) >> 8));
      px[3 * i + 1] = (uint32_t)(k - (((255 - c1) * k) >> 8));
      px[3 * i + 2] = (uint32_t)(k - (((255 - c0) * k) >> 8));
    } else {
      const int xb = cbv[i] - 128, xr = crv[i] - 128;
      px[3 * i + 0] = jpg_clamp(Y + ((116130 * xb + 32768) >> 16));                  // FIX(1.772)
      px[3 * i + 1] = jpg_clamp(Y + ((-46802 * xr + (-cbg * xb + 32768)) >> 16));  // FIX(0.714136286)
      px[3 * i + 2] = jpg_clamp(Y + ((91881 * xr + 32768) >> 16));                   // FIX(1.402)
    }
  }
#pragma unroll
  for (int j = 0; j < 6; ++j)
    o[j] = px[4 * j] | px[4 * j + 1] << 8 | px[4 * j + 2] << 16 | px[4 * j + 3] << 24;
}

// grid (tiles of 256 x 8 decoded pixels, n); (h, w) is the batch's output size, which is the
// decoded size turned by each image's EXIF orientation (D.orient, OpenCV 3.4.2 loadsave.cpp
// ApplyExifOrientation: 2 flip(1), 3 flip(-1), 4 flip(0), 5 transpose, 6 transpose + flip(1),
// 7 transpose + flip(-1), 8 transpose + flip(0)).  Decoded pixel (y, x) of an H x W image goes to
// the output position below; orientation 1 keeps the coalesced 24-byte row stores
__global__ __launch_bounds__(256) void jpeg_color8_kernel(const JpegDev* __restrict__ imgs,
                                                          const uint8_t* __restrict__ planes,
                                                          uint8_t* __restrict__ dst, int h, int w,
                                                          int64_t row_stride) {
  const JpegDev& D = imgs[blockIdx.y];
  const int H = D.height, W = D.width;  // as decoded
  const int ow = (W + 7) / 8;
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= (int64_t)H * ow) return;
  const int y = (int)(q / ow), x0 = 8 * (int)(q - (int64_t)y * ow);
  uint32_t o[6];
  if (D.ncomp == 1) jpg_color8<1, 1, true>(D, planes, x0, y, o);
  else if (D.up == 0) jpg_color8<1, 1, false>(D, planes, x0, y, o);
  else if (D.up == 1) jpg_color8<2, 1, false>(D, planes, x0, y, o);
  else jpg_color8<2, 2, false>(D, planes, x0, y, o);
  uint8_t* const img = dst + (int64_t)blockIdx.y * h * row_stride;
  if (D.orient > 1) {
    const int t = D.orient;
    for (int k = 0; k < 8 && x0 + k < W; ++k) {
      const int x = x0 + k;
      int oy, ox;
      if (t <= 4) {
        oy = (t == 3 || t == 4) ? H - 1 - y : y;
        ox = (t == 2 || t == 3) ? W - 1 - x : x;
      } else {  // transposed: (x, y), then the flip of the W x H result
        oy = (t == 7 || t == 8) ? W - 1 - x : x;
        ox = (t == 6 || t == 7) ? H - 1 - y : y;
      }
      uint8_t* p = img + (int64_t)oy * row_stride + (int64_t)ox * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int b = 3 * k + c;
        p[c] = (uint8_t)(o[b >> 2] >> (8 * (b & 3)));
      }
    }
    return;
  }
  uint8_t* p = img + (int64_t)y * row_stride + (int64_t)x0 * 3;
  if (x0 + 8 <= w && ((uintptr_t)p & 7) == 0) {
    uint2* p2 = reinterpret_cast<uint2*>(p);
    p2[0] = make_uint2(o[0], o[1]);
    p2[1] = make_uint2(o[2], o[3]);
    p2[2] = make_uint2(o[4], o[5]);
  } else if (x0 + 8 <= w && ((uintptr_t)p & 3) == 0) {
    uint32_t* p4 = reinterpret_cast<uint32_t*>(p);
#pragma unroll
    for (int j = 0; j < 6; ++j) p4[j] = o[j];
  } else {
    for (int k = 0; k < 24 && x0 + k / 3 < w; ++k) p[k] = (uint8_t)(o[k >> 2] >> (8 * (k & 3)));
  }
}

// the colour space libjpeg assigns a file (jdapimin.c default_decompress_parms; the caller asks
// for RGB, or CMYK for 4 components): 0 YCbCr (converted), 1 RGB (copied), 2 CMYK (copied), 3 YCCK
// (converted to CMYK), -1 one that is not restated.
// libjpeg 9 looks at the component IDs first -- (1, 2, 3) YCbCr, (1, 0x22, 0x23) big-gamut YCC,
// 'R' 'G' 'B' RGB, 'r' 'g' 'b' big-gamut RGB -- then a JFIF marker (YCbCr), then Adobe's transform
// (0 RGB, else YCbCr), else YCbCr.  libjpeg-turbo (6b's order) looks at JFIF, then Adobe, then the
// IDs 'R' 'G' 'B', else YCbCr.
static int jpg_color_space(const JpegHost& J, bool turbo) {
  if (J.ncomp == 4)  // CMYK stored as is, or YCCK: Adobe's transform 0 / 2 (else YCCK; no marker: CMYK)
    return J.adobe && J.adobe_transform != 0 ? 3 : 2;
  if (J.ncomp != 3) return 0;
  const int a = J.cid[0], b = J.cid[1], c = J.cid[2];
  const bool rgb_ids = a == 'R' && b == 'G' && c == 'B';
  const int adobe = J.adobe_transform == 0 ? 1 : 0;
  if (!turbo) {
    if (a == 1 && b == 2 && c == 3) return 0;
    if ((a == 1 && b == 0x22 && c == 0x23) || (a == 'r' && b == 'g' && c == 'b')) return -1;
    if (rgb_ids) return 1;
    if (J.jfif) return 0;
    return J.adobe ? adobe : 0;
  }
  if (J.jfif) return 0;
  if (J.adobe) return adobe;
  return rgb_ids ? 1 : 0;
}

// ---- host: batch plan ---------------------------------------------------------------------------
struct JpegPlan {
  std::vector<JpegDev> dev;
  std::vector<uint64_t> blk_end;
  std::vector<size_t> scan_begin;
  std::vector<JpegScanDev> scans;   // the scan path's scans, image by image
  std::vector<size_t> scan_src;     // their first byte in the file
  uint64_t scan_bytes = 0, nblk = 0, plane_bytes = 0, ub_bytes = 0;
  uint32_t nintervals = 0, nchunks = 0, max_items = 1, max_items_w = 1, nsub = 1;
  uint64_t nmk = 0;  // marker table entries
  int mt_img = 1, mt_scan = 1;  // most unstuffing tiles of an image / of a scan
  bool any_chunked = false, any_restart = false;
  bool any_huff_scan = false, any_arith = false;  // scan-path images of each coding
  bool scales[2][2] = {};  // IDCT output scales present: [sv - 1][sh - 1]
  size_t off_imgs = 0, off_blkend = 0, off_scans = 0, off_scan = 0, off_coef = 0, off_planes = 0;
  size_t off_ub = 0, off_iv = 0, off_ivend = 0, off_mk = 0, off_ublen = 0, off_ublen_s = 0, off_s0 = 0, off_s1 = 0,
         off_cnt = 0, off_start = 0, off_flag = 0, off_chg0 = 0, off_chg1 = 0, off_ck_st = 0,
         off_ck_co = 0, off_tcnt = 0, off_ck_iv = 0, off_iv_ck = 0, total = 0;
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// flags: IDN_JPEG_TURBO selects libjpeg-turbo's decode (else libjpeg 9d's); bits 8..23 = entropy
// chunk size in bits (0: the batch-dependent default; else a multiple of 64, >= 512)
static int jpeg_plan(const uint8_t* const* files, const size_t* lens, int n, int h, int w,
                     int flags, JpegPlan& P, std::string* err, bool tables = true) {
  const bool turbo = (flags & IDN_JPEG_TURBO) != 0;
  const bool orient = (flags & IDN_JPEG_IGNORE_ORIENTATION) == 0;
  const uint32_t chunk_req = (uint32_t)(flags >> 8) & 0xFFFFu;
  if ((flags & ~(IDN_JPEG_TURBO | IDN_JPEG_IGNORE_ORIENTATION | (0xFFFF << 8))) != 0 ||
      (chunk_req != 0 && (chunk_req < 512 || chunk_req % 64 != 0))) {
    if (err) *err = "bad flags";
    return IDN_EINVAL;
  }
  uint64_t chunked_bits = 0;  // entropy bits of the images the chunked decoder takes
  P.dev.assign(n, JpegDev{});
  P.blk_end.assign(n, 0);
  P.scan_begin.assign(n, 0);
  for (int i = 0; i < n; ++i) {
    JpegHost J;
    if (!files[i]) return jpg_fail(err, "null file pointer");
    int rc = jpeg_parse(files[i], lens[i], J, err);
    if (rc != IDN_OK) return rc;
    const int ori = orient ? jpg_exif_orientation(files[i], lens[i]) : 1;
    const bool tr = ori >= 5;  // the output is the transposed size
    if ((h > 0 && (tr ? J.width : J.height) != h) || (w > 0 && (tr ? J.height : J.width) != w)) {
      if (err) *err = "image size differs from the batch size";
      return IDN_EINVAL;
    }
    JpegDev& D = P.dev[i];
    memset(&D, 0, sizeof(D));
    D.orient = ori;
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
      for (int c = 0; c < J.ncomp; ++c) {
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
      // jdmaster.c (libjpeg >= 7, do_fancy_upsampling): the IDCT size doubles while the doubled
      // component still divides the maximum sampling factor (at most 16 = 2 x DCTSIZE); the two
      // directions never differ by more than 2x, which holds for factors 1 and 2
      D.sh[c] = (!turbo && D.hmax % (2 * D.ch[c]) == 0) ? 2 : 1;
      D.sv[c] = (!turbo && D.vmax % (2 * D.cv[c]) == 0) ? 2 : 1;
      D.pw[c] = D.bw[c] * 8 * D.sh[c];
      // libjpeg: downsampled size = ceil(image size * samp * idct size / (max samp * 8))
      D.dw[c] = (J.width * D.ch[c] * D.sh[c] + D.hmax - 1) / D.hmax;
      D.dh[c] = (J.height * D.cv[c] * D.sv[c] + D.vmax - 1) / D.vmax;
      P.scales[D.sv[c] - 1][D.sh[c] - 1] = true;
      D.blk_off[c] = P.nblk;
      P.nblk += (uint64_t)D.bw[c] * D.bh[c];
      D.pl_off[c] = P.plane_bytes;
      P.plane_bytes += (uint64_t)D.pw[c] * D.bh[c] * 8 * D.sv[c];
    }
    // what the colour pass still has to upsample (the chroma planes' remaining factor)
    D.up = 0;
    if (J.ncomp >= 3) {
      const int fh = D.hmax / (D.ch[1] * D.sh[1]), fv = D.vmax / (D.cv[1] * D.sv[1]);
      if (fh != D.hmax / (D.ch[2] * D.sh[2]) || fv != D.vmax / (D.cv[2] * D.sv[2]) ||
          D.ch[0] * D.sh[0] != D.hmax || D.cv[0] * D.sv[0] != D.vmax ||
          (J.ncomp == 4 && (D.ch[3] * D.sh[3] != D.hmax || D.cv[3] * D.sv[3] != D.vmax)))
        return jpg_fail(err, "unsupported chroma sampling");
      if (fh == 1 && fv == 1) D.up = 0;
      else if (fh == 2 && fv == 1) D.up = 1;
      else if (fh == 2 && fv == 2) D.up = 2;
      else return jpg_fail(err, "unsupported chroma sampling");
    }
    D.cb_g = turbo ? 22554 : 22553;  // FIX(0.34414) / FIX(0.344136286), SCALEBITS 16
    P.blk_end[i] = P.nblk;
    D.bpm = 0;
    for (int c = 0; c < J.ncomp; ++c)
      for (int v = 0; v < D.cv[c]; ++v)
        for (int hh = 0; hh < D.ch[c]; ++hh) {
          D.ph_comp[D.bpm] = (uint8_t)c;
          D.ph_dv[D.bpm] = (uint8_t)v;
          D.ph_dh[D.bpm] = (uint8_t)hh;
          ++D.bpm;
        }
    D.total_blocks = (uint32_t)mcus * D.bpm;
    for (int c = 0; c < J.ncomp; ++c) {  // jdinput.c: ceil(ceil(size * samp / max samp) / 8)
      const int cw = (J.width * D.ch[c] + D.hmax - 1) / D.hmax;
      const int chh = (J.height * D.cv[c] + D.vmax - 1) / D.vmax;
      D.wib[c] = (cw + 7) / 8;
      D.hib[c] = (chh + 7) / 8;
    }
    for (int t = 0; t < 4; ++t) memcpy(D.q[t], J.q[t], sizeof(D.q[t]));
    if (J.smooth && turbo)  // libjpeg-turbo >= 2.1: 9 coefficients from a 5x5 DC neighbourhood
      return jpg_fail(err, "libjpeg-turbo block smoothing (progressive file with imprecise AC) "
                           "not supported");
    D.smooth = J.smooth ? 1 : 0;
    D.arith = J.arith ? 1 : 0;
    D.rgb = jpg_color_space(J, turbo);
    if (D.rgb < 0) return jpg_fail(err, "big-gamut (BG_YCC / BG_RGB) JPEG not supported");
    memcpy(D.cbits, J.cbits, sizeof(D.cbits));
    if (!J.scans.empty()) {  // the scan path: one descriptor per scan, its bytes in this image's
                             // stretch of the batch scan buffer; the parallel path sees no data
      D.scan_off = P.scan_bytes;
      D.scan_len = 0;
      P.scan_begin[i] = 0;
      D.ub_off = P.ub_bytes;
      P.ub_bytes += 64;
      D.iv_off = P.nintervals;
      D.nintervals = 1;
      P.nintervals += 1;
      D.mk_off = P.nmk;
      D.mk_cap = 0;
      D.restart = 0;
      D.nchunks = 0;
      D.scan0 = (uint32_t)P.scans.size();
      D.nscan = (uint32_t)J.scans.size();
      (J.arith ? P.any_arith : P.any_huff_scan) = true;
      for (const ScanHost& S : J.scans) {
        JpegScanDev SD;
        memset(&SD, 0, sizeof(SD));
        SD.img = i;
        SD.ns = S.ns;
        for (int k = 0; k < S.ns; ++k) SD.comp[k] = S.comp[k];
        SD.Ss = S.Ss;
        SD.Se = S.Se;
        SD.Ah = S.Ah;
        SD.Al = S.Al;
        SD.restart = S.restart;
        SD.kind = !J.progressive ? JPG_SEQ
                  : S.Ss == 0     ? (S.Ah ? JPG_DC_REFINE : JPG_DC_FIRST)
                                  : (S.Ah ? JPG_AC_REFINE : JPG_AC_FIRST);
        SD.nunits = S.ns == 1 ? (uint32_t)D.wib[S.comp[0]] * (uint32_t)D.hib[S.comp[0]]
                              : (uint32_t)mcus;
        SD.nintervals = S.restart ? (int)((SD.nunits + S.restart - 1) / S.restart) : 1;
        if (SD.nintervals < 1) SD.nintervals = 1;
        SD.arith = J.arith ? 1 : 0;
        for (int k = 0; k < 4; ++k) {
          SD.td[k] = S.td[k];
          SD.ta[k] = S.ta[k];
          SD.aL[k] = S.aL[k];
          SD.aU[k] = S.aU[k];
          SD.aK[k] = S.aK[k];
        }
        for (int sl = 0; sl < 8; ++sl)
          for (int k = 0; k < 18; ++k) SD.maxcode[sl][k] = -1;
        for (int k = 0; k < S.ns && tables && !J.arith; ++k) {
          const bool dc = SD.kind == JPG_SEQ || SD.kind == JPG_DC_FIRST;
          const bool ac = SD.kind == JPG_SEQ || SD.kind == JPG_AC_FIRST || SD.kind == JPG_AC_REFINE;
          if (dc) {
            rc = jpeg_build_huff(S.dc[k], true, SD.lut[k], SD.maxcode[k], SD.valoff[k], SD.huffval[k], err);
            if (rc != IDN_OK) return rc;
          }
          if (ac) {
            rc = jpeg_build_huff(S.ac[k], false, SD.lut[4 + k], SD.maxcode[4 + k], SD.valoff[4 + k],
                                 SD.huffval[4 + k], err);
            if (rc != IDN_OK) return rc;
          }
        }
        const size_t len = S.end - S.begin;
        if (len >= JPG_MAX_SCAN) return jpg_fail(err, "scan too large");
        SD.scan_off = P.scan_bytes;
        SD.scan_len = (uint32_t)len;
        P.scan_bytes += (len + 15) & ~(size_t)15;
        SD.ub_off = P.ub_bytes;
        P.ub_bytes += (len + 64 + 15) & ~(size_t)15;
        SD.iv_off = P.nintervals;
        P.nintervals += (uint32_t)SD.nintervals;
        SD.mk_off = P.nmk;
        SD.mk_cap = (uint32_t)SD.nintervals + JPG_MK_EXTRA;
        P.nmk += SD.mk_cap;
        P.scans.push_back(SD);
        P.scan_src.push_back(S.begin);
      }
      continue;
    }
    for (int t = 0; t < 4 && tables; ++t) {
      for (int k = 0; k < 18; ++k) D.maxcode[t][k] = -1;
      const HuffSpec& H = t < 2 ? J.dc[t] : J.ac[t - 2];
      if (!H.present) continue;
      rc = jpeg_build_huff(H, t < 2, D.lut[t], D.maxcode[t], D.valoff[t], D.huffval[t], err);
      if (rc != IDN_OK) return rc;
    }
    D.scan_off = P.scan_bytes;
    D.scan_len = (uint32_t)(J.scan_end - J.scan_begin);
    P.scan_begin[i] = J.scan_begin;
    if (J.scan_end - J.scan_begin >= JPG_MAX_SCAN) return jpg_fail(err, "scan too large");
    P.scan_bytes += (D.scan_len + 15) & ~15u;
    D.ub_off = P.ub_bytes;
    P.ub_bytes += (D.scan_len + 64 + 15) & ~15u;
    D.iv_off = P.nintervals;
    P.nintervals += (uint32_t)D.nintervals;
    D.mk_off = P.nmk;
    D.mk_cap = (uint32_t)D.nintervals + JPG_MK_EXTRA;
    P.nmk += D.mk_cap;
    if (!D.restart) chunked_bits += (uint64_t)D.scan_len * 8;
  }
  // entropy chunks (the self-synchronising decoder's threads).  Default size: about 100k chunks
  // in the batch, within [1536, 6144] bits in steps of 512 -- a single 600x1000 q90 file decodes
  // in 1.41 ms at 1536-bit chunks against 1.62 at 4096, a batch of 256 in 7.07 ms at 6144
  // against 7.27 (profiles/r05/jpeg/chunk_sweep.txt): short chunks shorten every pass when the
  // batch cannot fill the chip, long ones need fewer B passes when it can
  const uint32_t chunk_bits =
      chunk_req ? chunk_req
                : (uint32_t)std::min<uint64_t>(
                      6144, std::max<uint64_t>(1536, (chunked_bits / 100000 + 511) / 512 * 512));
  for (int i = 0; i < n; ++i) {
    JpegDev& D = P.dev[i];
    D.ch_off = P.nchunks;
    D.chunk_bits = chunk_bits;
    if (D.nscan) continue;  // the scan path: no chunks
    // (restart intervals: each its own chunks, jpeg_chunk_map_kernel; room for the worst case)
    D.nchunks = (uint32_t)(((uint64_t)D.scan_len * 8 + D.chunk_bits - 1) / D.chunk_bits) +
                (D.restart ? (uint32_t)D.nintervals : 0u);
    if (D.nchunks == 0) D.nchunks = 1;
    P.nchunks += D.nchunks;
    P.any_chunked = true;
    P.any_restart |= D.restart != 0;
    P.max_items = std::max(P.max_items, D.nchunks);
    P.max_items_w = std::max(P.max_items_w, D.nchunks * jpg_nsub(chunk_bits));
  }
  P.off_imgs = 0;
  P.off_blkend = align256(P.off_imgs + sizeof(JpegDev) * (size_t)n);
  P.off_scans = align256(P.off_blkend + sizeof(uint64_t) * (size_t)n);
  P.off_scan = align256(P.off_scans + sizeof(JpegScanDev) * P.scans.size());
  P.off_coef = align256(P.off_scan + P.scan_bytes + 16);
  P.off_planes = align256(P.off_coef + P.nblk * 128);
  P.off_ub = align256(P.off_planes + P.plane_bytes);
  P.off_iv = align256(P.off_ub + P.ub_bytes);
  P.off_ivend = align256(P.off_iv + sizeof(uint32_t) * (size_t)P.nintervals);
  P.off_mk = align256(P.off_ivend + sizeof(uint32_t) * (size_t)P.nintervals);
  P.off_ublen = align256(P.off_mk + sizeof(uint2) * (size_t)P.nmk);
  P.off_ublen_s = align256(P.off_ublen + sizeof(uint32_t) * (size_t)n);
  P.off_s0 = align256(P.off_ublen_s + sizeof(uint32_t) * (P.scans.size() + 1));
  P.off_s1 = align256(P.off_s0 + sizeof(uint64_t) * (size_t)P.nchunks);
  P.off_cnt = align256(P.off_s1 + sizeof(uint64_t) * (size_t)P.nchunks);
  P.off_start = align256(P.off_cnt + sizeof(ChunkOut) * (size_t)P.nchunks);
  P.off_flag = align256(P.off_start + sizeof(ChunkOut) * (size_t)P.nchunks);
  P.off_chg0 = align256(P.off_flag + 256);
  P.off_chg1 = align256(P.off_chg0 + (size_t)P.nchunks);
  P.nsub = jpg_nsub(chunk_bits);
  P.off_ck_st = align256(P.off_chg1 + (size_t)P.nchunks);
  P.off_ck_co = align256(P.off_ck_st + sizeof(uint64_t) * (size_t)P.nchunks * P.nsub);
  for (const JpegDev& D : P.dev)
    P.mt_img = std::max(P.mt_img, (int)((D.scan_len + UNS_TILE - 1) / UNS_TILE));
  for (const JpegScanDev& S : P.scans)
    P.mt_scan = std::max(P.mt_scan, (int)((S.scan_len + UNS_TILE - 1) / UNS_TILE));
  P.off_ck_iv = align256(P.off_ck_co + sizeof(ChunkOut) * (size_t)P.nchunks * P.nsub);
  P.off_iv_ck = align256(P.off_ck_iv + sizeof(uint32_t) * (size_t)P.nchunks);
  P.off_tcnt = align256(P.off_iv_ck + sizeof(uint32_t) * (size_t)P.nintervals);
  const size_t ntc = std::max((size_t)n * P.mt_img, P.scans.size() * (size_t)P.mt_scan);
  P.total = align256(P.off_tcnt + sizeof(uint2) * ntc);
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
  const bool tr = jpg_exif_orientation(file, len) >= 5;  // cv2.imread's shape: after the turn
  *height = tr ? J.width : J.height;
  *width = tr ? J.height : J.width;
  *components = J.ncomp;
  return IDN_OK;
}

extern "C" int idn_jpeg_orientation(const uint8_t* file, size_t len, int* orientation) {
  IDN_CHECK_ARG(file && orientation, "idn_jpeg_orientation: null pointer");
  *orientation = jpg_exif_orientation(file, len);
  return IDN_OK;
}

extern "C" size_t idn_jpeg_workspace_size(const uint8_t* const* files, const size_t* lens, int n,
                                          int flags) {
  if (!files || !lens || n <= 0) return 0;
  JpegPlan P;
  if (jpeg_plan(files, lens, n, 0, 0, flags, P, nullptr) != IDN_OK) return 0;  // tables checked
  return P.total;
}

extern "C" int idn_jpeg_decode_u8(const uint8_t* const* files, const size_t* lens, int n,
                                  uint8_t* dst, int h, int w, int64_t row_stride, int flags,
                                  void* workspace, size_t ws_bytes, void* stream) {
  IDN_CHECK_ARG(n >= 0 && (n == 0 || (files && lens && dst)), "idn_jpeg_decode_u8: null pointer");
  IDN_CHECK_ARG(h > 0 && w > 0 && row_stride >= (int64_t)w * 3,
                "idn_jpeg_decode_u8: bad output shape");
  IDN_CHECK_ARG(n <= 65535, "idn_jpeg_decode_u8: batch too large");
  if (n == 0) return IDN_OK;
  JpegPlan P;
  std::string err;
  const int rc = jpeg_plan(files, lens, n, h, w, flags, P, &err);
  if (rc != IDN_OK) return set_error(rc, "idn_jpeg_decode_u8: %s", err.c_str());
  if (!workspace || ws_bytes < P.total)
    return set_error(IDN_EWORKSPACE, "idn_jpeg_decode_u8: needs %zu workspace bytes (got %zu)",
                     P.total, ws_bytes);
  hipStream_t st = as_stream(stream);
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  // one pinned host staging buffer (kept per thread, grown as needed; the call is synchronous, so
  // the next call may reuse it) -> one copy: descriptors, block ends, entropy segments
  static thread_local uint8_t* pin = nullptr;
  static thread_local size_t pin_cap = 0;
  if (pin_cap < P.off_coef) {
    if (pin) (void)hipHostFree(pin);
    pin = nullptr;
    pin_cap = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&pin), P.off_coef, 0) != hipSuccess)
      return set_error(IDN_EHIP, "idn_jpeg_decode_u8: pinned staging alloc failed");
    pin_cap = P.off_coef;
  }
  uint8_t* host = pin;
  memcpy(host + P.off_imgs, P.dev.data(), sizeof(JpegDev) * (size_t)n);
  memcpy(host + P.off_blkend, P.blk_end.data(), sizeof(uint64_t) * (size_t)n);
  if (!P.scans.empty())
    memcpy(host + P.off_scans, P.scans.data(), sizeof(JpegScanDev) * P.scans.size());
  bool copy_ok = hipMemcpyAsync(ws, host, P.off_scan, hipMemcpyHostToDevice, st) == hipSuccess;
  {
    // the entropy segments, gathered by a few host threads in NPART parts of the batch; each
    // part's host-to-device copy is issued as soon as the part is complete, so the DMA of part
    // k overlaps the gathering of part k + 1
    constexpr int MAXPART = 16;
    const int nt = std::max(1, std::min(8, n / 8));
    const int npart = std::max(1, std::min(std::min(4, MAXPART), n / 16));
    std::atomic<int> done[MAXPART];
    for (int q = 0; q < MAXPART; ++q) done[q].store(0);
    auto first = [&](int q) { return (int)((int64_t)n * q / npart); };
    // image i's entropy bytes: its one segment, or its scans' segments (the scan path)
    auto gather = [&](int i) {
      const JpegDev& D = P.dev[i];
      if (D.nscan == 0) {
        memcpy(host + P.off_scan + D.scan_off, files[i] + P.scan_begin[i], D.scan_len);
        return;
      }
      for (uint32_t k = D.scan0; k < D.scan0 + D.nscan; ++k)
        memcpy(host + P.off_scan + P.scans[k].scan_off, files[i] + P.scan_src[k],
               P.scans[k].scan_len);
    };
    auto worker = [&](int k) {
      for (int q = 0; q < npart; ++q) {
        for (int i = first(q) + k; i < first(q + 1); i += nt) gather(i);
        done[q].fetch_add(1, std::memory_order_release);
      }
    };
    std::vector<std::thread> th;
    for (int k = 1; k < nt; ++k) th.emplace_back(worker, k);
    for (int q = 0; q < npart; ++q) {  // the calling thread: its share, then the part's copy
      for (int i = first(q); i < first(q + 1); i += nt) gather(i);
      done[q].fetch_add(1, std::memory_order_release);
      while (done[q].load(std::memory_order_acquire) < nt) std::this_thread::yield();
      const size_t b0 = P.dev[first(q)].scan_off;
      const size_t b1 = q + 1 < npart ? (size_t)P.dev[first(q + 1)].scan_off : P.scan_bytes;
      if (b1 > b0)
        copy_ok = copy_ok && hipMemcpyAsync(ws + P.off_scan + b0, host + P.off_scan + b0,
                                            b1 - b0, hipMemcpyHostToDevice, st) == hipSuccess;
    }
    for (auto& t : th) t.join();
  }
  if (!copy_ok) return set_error(IDN_EHIP, "idn_jpeg_decode_u8: staging copy failed");
  const JpegDev* dimg = reinterpret_cast<const JpegDev*>(ws + P.off_imgs);
  int16_t* coef = reinterpret_cast<int16_t*>(ws + P.off_coef);
  uint8_t* ub = ws + P.off_ub;
  uint32_t* ivs = reinterpret_cast<uint32_t*>(ws + P.off_iv);
  uint32_t* ive = reinterpret_cast<uint32_t*>(ws + P.off_ivend);
  uint2* mk = reinterpret_cast<uint2*>(ws + P.off_mk);
  uint32_t* ublen = reinterpret_cast<uint32_t*>(ws + P.off_ublen);
  uint64_t* S[2] = {reinterpret_cast<uint64_t*>(ws + P.off_s0),
                    reinterpret_cast<uint64_t*>(ws + P.off_s1)};
  ChunkOut* cnt = reinterpret_cast<ChunkOut*>(ws + P.off_cnt);
  ChunkOut* cstart = reinterpret_cast<ChunkOut*>(ws + P.off_start);
  uint32_t* flag = reinterpret_cast<uint32_t*>(ws + P.off_flag);
  uint64_t* ck_st = reinterpret_cast<uint64_t*>(ws + P.off_ck_st);
  ChunkOut* ck_co = reinterpret_cast<ChunkOut*>(ws + P.off_ck_co);
  uint8_t* chg[2] = {reinterpret_cast<uint8_t*>(ws + P.off_chg0),
                     reinterpret_cast<uint8_t*>(ws + P.off_chg1)};
  uint2* tcnt = reinterpret_cast<uint2*>(ws + P.off_tcnt);
  uint32_t* ck_iv = reinterpret_cast<uint32_t*>(ws + P.off_ck_iv);
  uint32_t* iv_ck = reinterpret_cast<uint32_t*>(ws + P.off_iv_ck);
  uint32_t* mk_over = flag + 33;  // marker table overflow (jpeg_unstuff_final)
  if (hipMemsetAsync(mk_over, 0, 4, st) != hipSuccess)
    return set_error(IDN_EHIP, "idn_jpeg_decode_u8: memset failed");
  {
    const dim3 g((unsigned)P.mt_img, (unsigned)n);
    hipLaunchKernelGGL(jpeg_unstuff_count<JpegDev>, g, dim3(1024), 0, st, dimg, ws + P.off_scan,
                       tcnt, P.mt_img);
    hipLaunchKernelGGL(jpeg_unstuff_write<JpegDev>, g, dim3(1024), 0, st, dimg, ws + P.off_scan,
                       tcnt, P.mt_img, ub, mk);
    hipLaunchKernelGGL(jpeg_unstuff_final<JpegDev>, dim3(n), dim3(256), 0, st, dimg, tcnt,
                       P.mt_img, ub, mk, ivs, ive, ublen, mk_over);
  }
  if (P.any_restart)
    hipLaunchKernelGGL(jpeg_chunk_map_kernel, dim3(n), dim3(256), 0, st, dimg, ivs, ive, iv_ck,
                       ck_iv);
  const JpegScanDev* dscan = reinterpret_cast<const JpegScanDev*>(ws + P.off_scans);
  if (!P.scans.empty()) {
    // (after the images' unstuffing: the tile counts reuse the same array)
    const unsigned ns = (unsigned)P.scans.size();
    const dim3 g((unsigned)P.mt_scan, ns);
    hipLaunchKernelGGL(jpeg_unstuff_count<JpegScanDev>, g, dim3(1024), 0, st, dscan,
                       ws + P.off_scan, tcnt, P.mt_scan);
    hipLaunchKernelGGL(jpeg_unstuff_write<JpegScanDev>, g, dim3(1024), 0, st, dscan,
                       ws + P.off_scan, tcnt, P.mt_scan, ub, mk);
    hipLaunchKernelGGL(jpeg_unstuff_final<JpegScanDev>, dim3(ns), dim3(256), 0, st, dscan, tcnt,
                       P.mt_scan, ub, mk, ivs, ive, reinterpret_cast<uint32_t*>(ws + P.off_ublen_s),
                       mk_over);
  }
  const dim3 gitems((P.max_items + 63) / 64, n);
  uint32_t* badseen = flag + 32;  // (past the sync passes' flags)
  // entropy decoding to the output; badlen: see jpeg_write_kernel
  auto decode = [&](int badlen) -> int {
    if (hipMemsetAsync(ws + P.off_coef, 0, P.nblk * 128, st) != hipSuccess ||
        hipMemsetAsync(badseen, 0, 4, st) != hipSuccess)
      return set_error(IDN_EHIP, "idn_jpeg_decode_u8: memset failed");
    int cur = 0;
    if (P.any_chunked) {
      // pass A, then pass B until no chunk's end state changes (a batch takes ~4-6 passes, a
      // single large file ~8-9).  The B passes are launched JPG_BROUND at a time with one flag each
      // and one host read per round: the pass after the first one that changed nothing returns at
      // once (its predecessor's flag), so a round costs the passes that work plus a launch each for
      // the rest -- every host round trip (a D2H read and a stream synchronisation, ~30-40 us)
      // was a gap in a single file's decode
      constexpr int JPG_BROUND = 12;
      hipLaunchKernelGGL(jpeg_sync_kernel<true>, gitems, dim3(64), 0, st, dimg, ub, ublen, S[1],
                         S[0], cnt, flag, chg[1], chg[0], 1, ck_st, ck_co, nullptr, badlen, ck_iv,
                         iv_ck, ivs, ive);
      for (uint32_t it = 0;; it += JPG_BROUND) {
        if (hipMemsetAsync(flag, 0, 4 * JPG_BROUND, st) != hipSuccess)
          return set_error(IDN_EHIP, "idn_jpeg_decode_u8: memset failed");
        for (int k = 0; k < JPG_BROUND; ++k) {
          hipLaunchKernelGGL(jpeg_sync_kernel<false>, gitems, dim3(64), 0, st, dimg, ub, ublen,
                             S[cur], S[cur ^ 1], cnt, flag + k, chg[cur], chg[cur ^ 1],
                             it + k == 0 ? 1 : 0, ck_st, ck_co, k > 0 ? flag + k - 1 : nullptr,
                             badlen, ck_iv, iv_ck, ivs, ive);
          cur ^= 1;
        }
        uint32_t changed[JPG_BROUND] = {};
        if (hipMemcpyAsync(changed, flag, sizeof(changed), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
          return set_error(IDN_EHIP, "idn_jpeg_decode_u8: sync pass failed");
        if (!changed[JPG_BROUND - 1]) break;  // the round's last pass changed nothing
        if (it > P.max_items + 2)
          return set_error(IDN_EHIP, "idn_jpeg_decode_u8: entropy decoding did not converge");
      }
      hipLaunchKernelGGL(jpeg_prefix_kernel, dim3(n), dim3(256), 0, st, dimg, cnt, cstart, n, ck_iv,
                         iv_ck);
    }
    const dim3 gwrite((P.max_items_w + 63) / 64, n);
    hipLaunchKernelGGL(jpeg_write_kernel, gwrite, dim3(64), 0, st, dimg, ub, ublen, ivs, ive, ck_st,
                       ck_co, cstart, coef, badlen, badseen, ck_iv, iv_ck);
    if (!P.scans.empty()) {
      if (P.any_huff_scan)
        hipLaunchKernelGGL(jpeg_prog_kernel, dim3(n), dim3(64), 0, st, dimg, dscan, ub, ivs, ive,
                           reinterpret_cast<const uint32_t*>(ws + P.off_ublen_s), coef);
      if (P.any_arith)
        hipLaunchKernelGGL(jpeg_arith_kernel, dim3(n), dim3(64), 0, st, dimg, dscan, ub, ivs, ive,
                           coef);
    }
    const uint64_t gb = (P.nblk + 255) / 256;
    IDN_CHECK_ARG(gb < 0x7FFFFFFF, "idn_jpeg_decode_u8: batch too large");
    const uint64_t* bend = reinterpret_cast<const uint64_t*>(ws + P.off_blkend);
    if (P.scales[0][0])
      hipLaunchKernelGGL((jpeg_idct_kernel<1, 1>), dim3((unsigned)gb), dim3(256), 0, st, dimg, bend,
                         n, P.nblk, coef, ws + P.off_planes);
    if (P.scales[0][1])
      hipLaunchKernelGGL((jpeg_idct_kernel<1, 2>), dim3((unsigned)gb), dim3(256), 0, st, dimg, bend,
                         n, P.nblk, coef, ws + P.off_planes);
    if (P.scales[1][1])
      hipLaunchKernelGGL((jpeg_idct_kernel<2, 2>), dim3((unsigned)gb), dim3(256), 0, st, dimg, bend,
                         n, P.nblk, coef, ws + P.off_planes);
    {
      // decoded 8-pixel groups per image: h x ceil(w / 8), or w x ceil(h / 8) for a transposed one
      const int64_t groups = std::max((int64_t)h * ((w + 7) / 8), (int64_t)w * ((h + 7) / 8));
      const int64_t gx = (groups + 255) / 256;
      hipLaunchKernelGGL(jpeg_color8_kernel, dim3((unsigned)gx, (unsigned)n), dim3(256), 0, st, dimg,
                         ws + P.off_planes, dst, h, w, row_stride);
    }
    return IDN_OK;
  };
  int drc = decode(P.any_chunked ? 16 : 17);
  if (drc != IDN_OK) return drc;
  uint32_t bad_over[2] = {0u, 0u};  // badseen, mk_over (adjacent words)
  if (hipMemcpyAsync(bad_over, badseen, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return set_error(IDN_EHIP, "idn_jpeg_decode_u8: decode failed");
  if (bad_over[1])
    return set_error(IDN_EUNSUPPORTED, "idn_jpeg_decode_u8: more markers in an entropy-coded "
                                       "segment than restart intervals + %u (damaged file)",
                     JPG_MK_EXTRA);
  // a bad code on a true trajectory: decode again with libjpeg's rule
  if (P.any_chunked && bad_over[0] && (drc = decode(17)) != IDN_OK) return drc;
  // the staging buffer is reused by the next call: finish here
  if (hipStreamSynchronize(st) != hipSuccess)
    return set_error(IDN_EHIP, "idn_jpeg_decode_u8: decode failed");
  IDN_CHECK_LAUNCH("idn_jpeg_decode_u8");
  return IDN_OK;
}
