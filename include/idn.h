/*
 * idn.h — C-ABI of the MI355X-native noise-injection + denoising filter bank.
 *
 * One shared library (image-denoising_amd/idn/libidn_hip.so, hipcc --offload-arch=gfx950)
 * exports every function below with C linkage.  No torch types cross this boundary:
 * plain device pointers, sizes and a hipStream_t passed as `void*`.
 *
 * Conventions (all entry points)
 *   - Images are uint8 HxWxC, channel-interleaved (cv2.imread layout: BGR, C=3), row pitch
 *     `row_stride` bytes (>= W*C), a batch of `n` images laid back to back with image pitch
 *     h*row_stride.  f64 arrays use the same element order with pitch W*C elements.
 *   - Pointers are DEVICE pointers owned by the caller; nothing is allocated inside a call.
 *     Calls that need scratch take (workspace, ws_bytes) and expose idn_*_workspace_size().
 *   - Every call is stream-ordered on `stream` (NULL = default stream) and capture-safe
 *     (no sync, no malloc; idn_jpeg_decode_u8 and the one-time Poisson table build are the
 *     documented exceptions).  The RNG position is explicit: Philox4x32 keyed by (seed ^ a per-
 *     mode tag), counter = (element group, stream tag, image id) with image id = offset + i (or
 *     an explicit id array), so results do not depend on how a batch is split across launches,
 *     ranks or memory layouts.  Streams (csrc/noise.hip, noise_apply.hpp):
 *       gaussian / speckle, u8-only output  Philox4x32-7, one block per 8 elements: 16-bit
 *         uniforms, fp32 Box-Muller (the extreme radius cell refined to 32 bits from a second
 *         block, |z| <= 6.66), U8 computed as floor(clip(v + 255 n)) / floor(clip(v + v n)) in
 *         fp32 on the 0..255 scale
 *       gaussian / speckle, float64 output  Philox4x32-10, one block per 2 elements: 53-bit
 *         uniforms, fp64 Box-Muller, numpy's float64 apply; U8 = trunc(255 * out) of it
 *       s&p      Philox4x32-7, one block per 4 elements: 16-bit `flipped` / `salted` uniforms
 *                against integer thresholds (|P - p| < 2^-16)
 *       poisson  Philox4x32-7, one block per 4 elements, 32-bit words inverted through the
 *                exact CDF of Poisson(img_as_float(v) * vals)
 *     The tuning knobs of the kernels are compile-time constants: this library reads no
 *     environment variable.
 *   - Return IDN_OK (0) or a negative idn_status; idn_last_error() returns a thread-local
 *     message for the last failing call on the calling thread.
 *
 * Reference interfaces replaced (paths relative to the reference repo):
 *   cv2.GaussianBlur / cv2.blur / cv2.medianBlur / cv2.bilateralFilter calls inside the noise
 *   closures and the post-dispatch denoise hook: lib/model/test.py:193-1607,1787-1831 and
 *   lib/roi_data_layer/minibatch.py:87-1516,1636-1673; skimage random_noise calls at the same
 *   sites; lib/utils/blob.py:17-47 (prep_im_for_blob / im_list_to_blob).
 */
#ifndef IDN_H_
#define IDN_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum idn_status {
  IDN_OK = 0,
  IDN_EINVAL = -1,        /* bad shape / stride / parameter                         */
  IDN_EUNSUPPORTED = -2,  /* valid but unsupported combination (e.g. ksize 7)        */
  IDN_EHIP = -3,          /* HIP runtime error (launch failure, ...)                */
  IDN_EWORKSPACE = -4     /* workspace missing or too small                         */
} idn_status;

/* noise kinds for idn_noise_u8 (skimage.util.random_noise modes used on the path) */
typedef enum idn_noise_kind {
  IDN_NOISE_GAUSSIAN = 0, /* out = clip(x + N(mean, sqrt(var)), 0, 1)                */
  IDN_NOISE_SPECKLE = 1,  /* out = clip(x + x*N(mean, sqrt(var)), 0, 1)              */
  IDN_NOISE_SAP = 2,      /* salt & pepper, amount = p0, salt_vs_pepper = p1          */
  IDN_NOISE_POISSON = 3   /* out = clip(Poisson(x*vals)/vals, 0, 1), vals per image    */
} idn_noise_kind;

/* wavelet families for idn_wavelet_denoise_u8 */
typedef enum idn_wavelet {
  IDN_WAVELET_DB1 = 0,    /* Haar ('db1', skimage default)                           */
  IDN_WAVELET_BIOR15 = 1  /* 'bior1.5' (the reference's in-branch choice)             */
} idn_wavelet;

/* ---- library ------------------------------------------------------------------------- */
/* ABI version of this header; idn_abi_version() returns the library's.  A caller (the ctypes
 * binding idn/_lib.py) refuses a library whose number differs.  History:
 *   3  idn_jpeg_workspace_size / idn_jpeg_decode_u8 gained `flags` before `workspace`
 *      (IDN_JPEG_TURBO); the default decode became IJG libjpeg 9d's; idn_noise_filter_u8
 *      (the fused noise -> 3x3 / 5x5 filter) was removed: compose idn_noise_u8 and the filter
 *   4  idn_abi_version added (no signature changed)
 *   5  idn_noise_ycc_u8 and idn_wavelet_denoise_ycc added (no signature changed)
 *   6  cv2.imread's EXIF orientation: idn_jpeg_decode_u8 turns each image by it (flag
 *      IDN_JPEG_IGNORE_ORIENTATION keeps the decoded layout), idn_jpeg_info reports the turned
 *      size, idn_jpeg_orientation added */
#define IDN_ABI_VERSION 6
int idn_abi_version(void);
const char* idn_version(void);
const char* idn_last_error(void);
/* Test hook, not part of the ABI (exported, deliberately undeclared): the bilateral output
 * step's reciprocal, idn_internal_bl_recip_check, used by tests/test_filters_gpu.py only. */

/* ---- denoising filters (u8 -> u8, src != dst) ------------------------------------------ */

/* cv2.GaussianBlur(img, (ksize, ksize), 0), ksize in {3, 5}, BORDER_REFLECT_101.
 * Replaces e.g. lib/model/test.py:224, lib/roi_data_layer/minibatch.py:1636-1639. Bit-exact. */
int idn_gaussian_blur_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                         int64_t row_stride, int ksize, void* stream);

/* cv2.blur(img, (ksize, ksize)), ksize = 3, BORDER_REFLECT_101.
 * Replaces lib/model/test.py:241,1767, lib/roi_data_layer/minibatch.py:1640-1643. Bit-exact. */
int idn_box_blur_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                    int64_t row_stride, int ksize, void* stream);

/* cv2.medianBlur(img, ksize), ksize in {3, 5}, BORDER_REPLICATE.
 * Replaces lib/model/test.py:259, lib/roi_data_layer/minibatch.py:1644-1648. Bit-exact. */
int idn_median_blur_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                       int64_t row_stride, int ksize, void* stream);

/* cv2.bilateralFilter(img, d, sigma_color, sigma_space, borderType=BORDER_CONSTANT), c = 3
 * (or 1).  Replaces lib/model/test.py:278, lib/roi_data_layer/minibatch.py:1658-1663.
 * <= 1 LSB vs OpenCV (fp32 summation order). */
int idn_bilateral_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                     int64_t row_stride, int d, double sigma_color, double sigma_space,
                     void* stream);

/* ---- noise generators (skimage.util.random_noise, as called on the path) --------------- */

/* Apply one random_noise mode to a batch of u8 images.
 *   out_u8  (nullable): U8(255*out)  == (255*out).astype(np.uint8), the denoise-branch input
 *   out_f64 (nullable): out itself (float64 in [0,1]), what the "plain" branches return
 *   p0, p1: GAUSSIAN/SPECKLE: mean, var; SAP: amount, salt_vs_pepper; POISSON: unused
 *   replay  (nullable): caller-provided random field, which makes the result bit-exact with
 *     numpy's legacy stream:  GAUSSIAN/SPECKLE: f64 N(mean,sqrt(var)) field (n*h*w*c);
 *     SAP: f64 [2][n*h*w*c] = (random_sample for `flipped`, random_sample for `salted`);
 *     POISSON: f64 per-element Poisson draws (n*h*w*c).  NULL = Philox stream (seed, offset).
 *   workspace: POISSON needs idn_noise_workspace_size() bytes (per-image `vals`); else unused.
 *     (POISSON's CDF / level tables are built once per device by the library and kept.)
 * Replaces skimage random_noise at lib/model/test.py:193-590, minibatch.py:87-490. */
int idn_noise_u8(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n, int h, int w,
                 int c, int64_t row_stride, int kind, double p0, double p1, uint64_t seed,
                 uint64_t offset, const double* replay, void* workspace, size_t ws_bytes,
                 void* stream);
size_t idn_noise_workspace_size(int kind, int n);
/* Diagnostics for the POISSON flat kernel: builds (once per device) the per-vals level tables
 * (vals = 1 .. 256) and copies to ntab_out[9] the thresholds each level holds; a value above
 * cap_out[0] (the LDS capacity) means that level's draws would bisect the global CDF rows
 * instead of the LDS tables.  Synchronous on `stream`. */
int idn_poisson_levels(uint32_t* ntab_out, uint32_t* cap_out, void* stream);
/* As idn_noise_u8 (Philox stream only) with an explicit device array of n image ids instead of
 * offset + i: a mixed batch's images of one noise type (any ids) run as one launch and draw
 * exactly what per-image calls with offset = id would.  Replaces the per-image dispatch of the
 * mix lists (test.py:1611-1677, minibatch.py:1518-1574). */
int idn_noise_ids_u8(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n, int h, int w,
                     int c, int64_t row_stride, int kind, double p0, double p1, uint64_t seed,
                     const uint64_t* image_ids, void* workspace, size_t ws_bytes, void* stream);
/* As idn_noise_ids_u8, addressing the batch through a device array of n slots (int64): image i
 * of the launch reads src image slots[i] and writes out_u8 / out_f64 image slots[i] (compact
 * h*w*c images; row_stride must be w*c).  A mixed batch's per-type group then runs in place in
 * the full batch with no gather / scatter of its images. */
int idn_noise_slots_u8(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n, int h, int w,
                       int c, int64_t row_stride, int kind, double p0, double p1, uint64_t seed,
                       const uint64_t* image_ids, const int64_t* slots, void* workspace,
                       size_t ws_bytes, void* stream);

/* The live test path's float64 gaussian / speckle noise (random_noise(..., 'gaussian') returned as
 * float64 straight into denoise_wavelet: lib/model/test.py:1678-1684 -> 1807-1810), fused with
 * the wavelet's colour range: as idn_noise_u8 (kind GAUSSIAN or SPECKLE, c = 3, compact rows,
 * out_f64 required, out_u8 nullable; the float64 Philox stream, or numpy's field in `replay`;
 * image ids offset + i, or image_ids[i] when image_ids is non-NULL) -- the same bytes -- and per
 * image i the fp64 min and max of skimage rgb2ycbcr's Y, Cb, Cr over out_f64, as order-preserving
 * u64 keys in ycc_keys[6 i .. 6 i + 2] (min) and [6 i + 3 .. 6 i + 5] (max), written whole by the
 * call, for idn_wavelet_denoise_ycc: the wavelet then does not read the float64 image an extra
 * time for its colour range.  IDN_EUNSUPPORTED for an odd pixel count or misaligned buffers
 * (u8 2-byte, float64 16-byte aligned). */
int idn_noise_ycc_u8(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n, int h, int w,
                     int kind, double p0, double p1, uint64_t seed, uint64_t offset,
                     const uint64_t* image_ids, const double* replay, uint64_t* ycc_keys,
                     void* stream);

/* The reference's own additive noises (not skimage), SURVEY §8f:
 *   IDN_NOISE_UNIFORM   p0 = high   out = img_as_float(x) + U(0, high)         (test.py:767-903)
 *   IDN_NOISE_GAMMA     p0 = shape, p1 = scale: out = x + gamma.rvs(shape, scale) (1300-1437)
 *   IDN_NOISE_RAYLEIGH  p0 = scale  out = x + rayleigh.rvs(scale)               (1439-1572)
 *   IDN_NOISE_BROWNIAN  p0 = dt     out_u8 = sat(img + U8(255 * B)),
 *                       B = concat([0], cumsum(sqrt(dt) * N(0,1)[h*w*c - 1]))  (905-1126)
 * cv2.add(float64, float64) is a plain add, so out is unclipped; out_u8 = U8(255*out) wraps
 * modulo 256 ((uint8)(int32)trunc, |y| >= 2^31 -> 0); out_f64 = out (brownian: the walk B).
 * replay (float64, N*h*w*c, optional): numpy's unit draws -- random_sample, standard_gamma(shape),
 * sqrt(chisquare(2)), or for brownian the normals with element e holding z[e-1] (element 0
 * unused).  Brownian needs idn_noise_add_workspace_size() bytes of workspace. */
typedef enum idn_noise_add_kind {
  IDN_NOISE_UNIFORM = 4,
  IDN_NOISE_GAMMA = 5,
  IDN_NOISE_RAYLEIGH = 6,
  IDN_NOISE_BROWNIAN = 7
} idn_noise_add_kind;
int idn_noise_add_u8(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n, int h, int w,
                     int c, int64_t row_stride, int kind, double p0, double p1, uint64_t seed,
                     uint64_t offset, const double* replay, void* workspace, size_t ws_bytes,
                     void* stream);
size_t idn_noise_add_workspace_size(int kind, int n, int h, int w, int c);
/* As idn_noise_add_u8 (Philox stream only) with a device array of n image ids (see
 * idn_noise_ids_u8). */
int idn_noise_add_ids_u8(const uint8_t* src, uint8_t* out_u8, double* out_f64, int n, int h,
                         int w, int c, int64_t row_stride, int kind, double p0, double p1,
                         uint64_t seed, const uint64_t* image_ids, void* workspace,
                         size_t ws_bytes, void* stream);

/* Periodic noise pattern of add_periodic_noise (lib/model/test.py:1128-1298):
 * pattern[i] = U8(255*sin(t_i)), t = np.linspace(-A, A, h*w*c), written as u8 HxWxC (pitch w*c).
 * Image independent: build once per (h, w, c, A) and reuse. */
int idn_periodic_pattern_u8(uint8_t* pattern, int h, int w, int c, double amplitude,
                            void* stream);

/* cv2.add(img, pattern) on u8 (saturating), pattern broadcast over the batch. */
int idn_add_pattern_u8(const uint8_t* src, const uint8_t* pattern, uint8_t* dst, int n, int h,
                       int w, int c, int64_t row_stride, void* stream);
/* idn_add_pattern_u8 on the batch images slots[0..n) (compact h*w*c images, see
 * idn_noise_slots_u8). */
int idn_add_pattern_slots_u8(const uint8_t* src, const uint8_t* pattern, uint8_t* dst, int n,
                             int h, int w, int c, const int64_t* slots, void* stream);
/* dst image slots[i] = src image slots[i] for i < n (per_img bytes per image): the noise-free
 * ("original") members of a mixed batch. */
int idn_copy_slots_u8(const uint8_t* src, uint8_t* dst, int n, int64_t per_img,
                      const int64_t* slots, void* stream);

/* ---- quant noise (colour quantisation by k-means in 8-bit Lab) ---------------------------- */

/* Per image: lab = cv2.cvtColor(img, COLOR_BGR2LAB); k-means with k clusters on the Lab pixels;
 * out = cv2.cvtColor(centres.astype(uint8)[labels], COLOR_LAB2BGR).  Replaces the
 * MiniBatchKMeans(n_clusters=k).fit_predict blocks of lib/model/test.py:592-765 and
 * lib/roi_data_layer/minibatch.py:492-667.  C = 3 (BGR), 1 <= k <= 16, h*w >= k.
 *   centers_in == NULL: device fit -- greedy k-means++ seeding + Lloyd to a fixed point on up to
 *     8192 Lab samples of the image (all pixels when h*w <= 8192, else Philox draws keyed by
 *     (seed, image id = offset + i or image_ids[i])), best of 3 restarts by sample inertia
 *     (sklearn's n_init = 3; the restarts run as separate workgroups).
 *   centers_in != NULL: replay -- the caller's fitted centres (double [n][k][3], e.g. sklearn's
 *     cluster_centers_): labels = argmin_j ||c_j||^2 - 2 x.c_j in float64 (sklearn's
 *     _labels_inertia), bit-exact given the centres.
 * labels_out (nullable): uint8 [n][h][w] cluster index per pixel.  centers_out (nullable):
 * double [n][k][3], the centres used.  8-bit Lab follows OpenCV's integer RGB2Lab_b /
 * Lab2RGBinteger paths (parity vs cv2 unpinned: no cv2 in the build container). */
int idn_quant_u8(const uint8_t* src, uint8_t* dst, uint8_t* labels_out, int n, int h, int w,
                 int64_t row_stride, int k, uint64_t seed, uint64_t offset,
                 const uint64_t* image_ids, const double* centers_in, double* centers_out,
                 void* workspace, size_t ws_bytes, void* stream);
size_t idn_quant_workspace_size(int n, int k);
/* cv2.cvtColor(img, COLOR_BGR2LAB) / (lab, COLOR_LAB2BGR) on 8-bit 3-channel images. */
int idn_bgr2lab_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int64_t row_stride,
                   void* stream);
int idn_lab2bgr_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int64_t row_stride,
                   void* stream);

/* ---- fused steps (one pass over HBM instead of two) ------------------------------------------ */

/* cv2.GaussianBlur(img, (ksize, ksize), 0) then prep_im_for_blob at scale 1.0
 * (lib/utils/blob.py:33-47): blob = float32(float64(v) - mean[ch]), dense (n, h, w, c) float32
 * written by the filter kernel (the filtered u8 image never reaches HBM).  mean: host double[3].
 * IDN_EUNSUPPORTED unless C = 3 and compact rows of 8k <= 3024 bytes. */
int idn_gaussian_blob_f32(const uint8_t* src, float* blob, int n, int h, int w, int c,
                          int64_t row_stride, int ksize, const double* mean, void* stream);

/* Flat copy of nbytes (multiple of 16, 16-byte aligned pointers).  policy 0 = default cache
 * policy, 1 = nontemporal loads and stores.  Not a reference interface: the bench's same-run
 * copy ceiling (SURVEY §8d "also report a measured copy-kernel peak"). */
int idn_copy_u8(const uint8_t* src, uint8_t* dst, int64_t nbytes, int policy, void* stream);

/* ---- wavelet denoise (skimage 0.14.2 denoise_wavelet, BayesShrink, soft, YCbCr) -------- */

/* out_u8 = (255*denoise_wavelet(img, method='BayesShrink', mode='soft', wavelet=wavelet,
 *           multichannel=True, convert2ycbcr=True, wavelet_levels=levels)).astype(uint8),
 * c = 3.  levels <= 0 selects skimage's default max(dwt_max_level - 3, 1).  in_f64 (nullable)
 * replaces src when the caller holds a float image in [0,1] (the reference's f64 branches, dense
 * n*h*w*3).  out_f32 (nullable) receives the float result before the U8 cast (dense n*h*w*3).
 * Precision: Haar computes its statistics exactly (integer moments / fp64) and, on the fused
 * path, its level-1 synthesis stage in fp32.  bior1.5 keeps pywt's fp64 op order where an exact
 * value matters -- the normalisation (exact quotient), the level-1 column highpass and the finest
 * dd (whose exact zeros and median give sigma, bit-identical to an all-fp64 run: the median
 * recomputes its candidates' exact dd from the input), and the sums of squares -- and runs the
 * lowpass outputs (aa / ad / da), the deeper levels and the synthesis in fp32; intermediate bands
 * live in the workspace as fp32 (the coarsest aa as fp64): |out - reference| <= 1e-5 before the
 * cast (tests: <= 2e-6 from the all-fp64 form).
 * Replaces lib/model/test.py:197-201,1807-1810, minibatch.py:1653-1656,
 * minibatch_before_curvelet.py:85-87. */
int idn_wavelet_denoise_u8(const uint8_t* src, const double* in_f64, uint8_t* out_u8,
                           float* out_f32, int n, int h, int w, int64_t row_stride, int wavelet,
                           int levels, void* workspace, size_t ws_bytes, void* stream);
/* As idn_wavelet_denoise_u8 on float64 input (dense n*h*w*3) whose colour range idn_noise_ycc_u8
 * already reduced into ycc_keys: the same outputs bit for bit, one pass over the input fewer. */
int idn_wavelet_denoise_ycc(const double* in_f64, const uint64_t* ycc_keys, uint8_t* out_u8,
                            float* out_f32, int n, int h, int w, int wavelet, int levels,
                            void* workspace, size_t ws_bytes, void* stream);
size_t idn_wavelet_workspace_size(int n, int h, int w, int wavelet, int levels);
/* diagnostics: byte offset in the workspace of the per-image statistics blocks (256 doubles per
 * image: channel sums of squared details, sigma medians, thresholds) after a call */
size_t idn_wavelet_stats_offset(int n, int h, int w, int wavelet, int levels);

/* ---- float64 filters (the reference's quirk branches blur random_noise's float64 output) -- */

/* cv2.GaussianBlur / cv2.blur on CV_64F images (dense n*h*w*c doubles), BORDER_REFLECT_101.
 * Reached by train_v0 post hooks after a "plain" noise branch (minibatch.py:1636-1643) and by
 * test_v0's default branch (test.py:1757-1768).  Within 1e-12 of the double reference. */
int idn_gaussian_blur_f64(const double* src, double* dst, int n, int h, int w, int c, int ksize,
                          void* stream);
int idn_box_blur_f64(const double* src, double* dst, int n, int h, int w, int c, int ksize,
                     void* stream);

/* ---- shader / bloom noise types ---------------------------------------------------------- */

/* add_shader (test.py:1595-1601): np.array(ImageEnhance.Brightness(PIL image).enhance(factor)).
 * src is the BGR image; dst is written in PIL's RGB channel order, as the reference returns it. */
int idn_shader_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                  int64_t row_stride, double factor, void* stream);

/* add_bloom -> Automold add_sun_flare (tools/Automold.py:588-627): per image `ncirc` steps of
 * {filled LINE_8 circle on the overlay, cv2.addWeighted(overlay, a, out, b, 0)}.
 * circles: device int32 [n][ncirc][8] = {cx, cy, radius, c0, c1, c2, reset_overlay, 0};
 * weights: device float [n][ncirc][2] = {a, b}; spans: device int16 half-width table of radius R
 * at row offset t stored at R*(R+1)/2 + t (idn/automold.py).  <= 1 LSB (float blend order). */
int idn_bloom_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c, int64_t row_stride,
                 const int32_t* circles, const float* weights, int ncirc, const int16_t* spans,
                 void* stream);

/* ---- blob epilogue (lib/utils/blob.py:17-47) -------------------------------------------- */

/* blob[i, y, x, ch] = float32(float64(img[i,y,x,ch]) - mean[ch]) for y<h, x<w; zero elsewhere
 * in the (n, out_h, out_w, 3) float32 NHWC blob (im_list_to_blob's zero padding).  flip != 0
 * mirrors x (minibatch.py:1676-1677).  c must be 3.  Scale 1.0 only (the 600x1000 case). */
int idn_blob_f32(const uint8_t* src, float* blob, int n, int h, int w, int c,
                 int64_t row_stride, int out_h, int out_w, const double mean[3], int flip,
                 void* stream);

/* blob from a float64 image (dense n*h*w*3): float32(float64(float32(x)) - mean[ch]) -- what
 * prep_im_for_blob does with the float64 output of the "plain" noise branches. */
int idn_blob_from_f64(const double* src, float* blob, int n, int h, int w, int out_h, int out_w,
                      const double mean[3], int flip, void* stream);

/* cv2.resize(im_f32, None, None, fx, fy, INTER_LINEAR) on dense n*h*w*c float32 images
 * (prep_im_for_blob when the image is not already 600 x 1000: lib/utils/blob.py:44-45,
 * lib/model/test.py:75-76).  out_h/out_w = round(h*fy), round(w*fx) as cv2 computes them. */
int idn_resize_linear_f32(const float* src, float* dst, int n, int h, int w, int c, int out_h,
                          int out_w, double fx, double fy, void* stream);

/* ---- decode front-end (cv2.imread: lib/model/test.py:191, minibatch.py:85) --------------- */

/* Header of one JPEG file in host memory (SOI .. EOI): height, width, components (1, 3 or 4).
 * Taken: Huffman-coded baseline, extended sequential and progressive files (SOF0 / SOF1 / SOF2),
 * arithmetic-coded sequential and progressive files (SOF9 / SOF10, DAC conditioning), one or
 * several scans, restart intervals, 4:4:4 / 4:2:2 / 4:2:0 or grayscale; a progressive
 * file whose last scan leaves AC 1..5 imprecise is block-smoothed as libjpeg 9d smooths it
 * (jdcoefct.c smoothing_ok / decompress_smooth_data); three components are YCbCr or RGB as
 * libjpeg decides it (component IDs, JFIF / Adobe markers); four are CMYK or YCCK (Adobe's
 * transform; K sampled as the first component), decoded to libjpeg's CMYK and converted to BGR
 * as OpenCV does (icvCvt_CMYK2BGR_8u_C4C3R).  IDN_EUNSUPPORTED for anything else (lossless,
 * hierarchical, 12-bit, big-gamut colour, DHP / EXP / JPGn / LSE markers, other sampling).
 * height x width is the size cv2.imread returns: after the file's EXIF orientation
 * (idn_jpeg_orientation), so orientations 5..8 report the decoded size transposed. */
int idn_jpeg_info(const uint8_t* file, size_t len, int* height, int* width, int* components);

/* The EXIF orientation (1..8; 1 = none) OpenCV 3.4.2's imread applies to this file after decoding
 * (loadsave.cpp ApplyExifOrientation, unless IMREAD_IGNORE_ORIENTATION): exif.cpp's ExifReader
 * reads Orientation (0x0112) from IFD0 of the FIRST APP1 segment (little- or big-endian TIFF);
 * a marker its walk does not know, or a malformed IFD0 (any offset past the data, a bad tag
 * value among the tags it parses), means 1, as does a value outside 1..8.  The decode applies
 * it: 2 flip(1), 3 flip(-1), 4 flip(0), 5 transpose, 6 transpose + flip(1), 7 transpose +
 * flip(-1), 8 transpose + flip(0) (cv::flip codes).  Restated from OpenCV's published source
 * (parity vs cv2 unpinned: cv2 is not importable where this was built; the decoded pixels are
 * pinned by the real libjpeg 9d, the geometry by Pillow's reading of the tag). */
int idn_jpeg_orientation(const uint8_t* file, size_t len, int* orientation);

/* idn_jpeg_decode_u8 flags.  Default (0): the decode of the reference's pinned libjpeg 9d
 * (requirements.txt:74, linked by its OpenCV 3.4.2): 8x8 ISLOW IDCT for full-size components,
 * libjpeg 9's scaled 16x16 / 16x8 IDCT for 4:2:0 / 4:2:2 chroma (no upsampling pass), libjpeg 9's
 * YCbCr tables.  IDN_JPEG_TURBO: libjpeg-turbo's decode (8x8 IDCT, fancy h2v1 / h2v2
 * upsampling), what a turbo-linked OpenCV or PIL produce (a file libjpeg-turbo would
 * block-smooth is IDN_EUNSUPPORTED in this mode: turbo's smoothing is not restated).  Bits 8..23:
 * entropy chunk size in bits
 * for the self-synchronising decoder (0 = the default: ~100k chunks per batch, 1536..6144 bits;
 * else a multiple of 64, >= 512; does not
 * change the output). */
#define IDN_JPEG_TURBO 1
/* cv2.IMREAD_IGNORE_ORIENTATION: store every image as decoded (h x w is then the decoded size) */
#define IDN_JPEG_IGNORE_ORIENTATION 2
/* device workspace for decoding these files with these flags (0 if any is unsupported) */
size_t idn_jpeg_workspace_size(const uint8_t* const* files, const size_t* lens, int n, int flags);
/* cv2.imread(path) (IMREAD_COLOR) of n JPEG files held in host memory (any mix of the kinds
 * idn_jpeg_info takes: baseline / extended sequential files on the parallel path, progressive and
 * multi-scan files on the scan path), all h x w, into
 * the device u8 BGR NHWC batch dst (row_stride bytes per row), bit-exact with the library the
 * flags name (replaces cv2.imread at lib/model/test.py:191, lib/roi_data_layer/minibatch.py:85).
 * Damaged entropy-coded data decodes as libjpeg decodes it (it only warns): a file cut short (an
 * EOI appended, or none), bit errors, bad Huffman codes, lost / renumbered restart markers and
 * stray markers -- the data runs out, the rest of its restart interval stays gray, restart
 * markers resynchronise as jdmarker.c's jpeg_resync_to_restart does.
 * Each image is turned by its EXIF orientation (idn_jpeg_orientation) unless the flags say
 * IDN_JPEG_IGNORE_ORIENTATION; h x w is the size after that turn.
 * Speed: baseline / extended sequential files (the reference's VOC images) take the parallel
 * self-synchronising entropy decoder (600 x 1000 q90: ~1.3 ms alone, ~28 us each in a batch of
 * 256; one host core with libjpeg 9d: ~14 ms).
 * PROGRESSIVE AND ARITHMETIC-CODED FILES DECODE SLOWER THAN ONE HOST CORE.  They take the scan
 * path, which is serial within a restart interval (one lane per interval).  Measured on MI355X
 * for a 600 x 1000 file without restart markers: progressive 229 ms, arithmetic-coded 796 ms
 * (72.5 ms with a restart marker per MCU row), against ~22 ms for libjpeg 9d on one host core
 * (JPEG section).  The output is still bit-exact; use this path for correctness
 * or for large batches of such files, which run one wave per image side by side.
 * The entropy-coded segments are copied to the workspace in one transfer; synchronous on
 * `stream`. */
int idn_jpeg_decode_u8(const uint8_t* const* files, const size_t* lens, int n, uint8_t* dst,
                       int h, int w, int64_t row_stride, int flags, void* workspace,
                       size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* IDN_H_ */
