// Blob epilogue: lib/utils/blob.py:17-47 (prep_im_for_blob at scale 1.0 + im_list_to_blob),
// test-side lib/model/test.py:49-83, flip from lib/roi_data_layer/minibatch.py:1676-1677.
//
//   blob[i, y, x, ch] = float32(float64(img[i, y, x', ch]) - PIXEL_MEANS[ch])   y < h, x < w
//                     = 0                                                        padding
// x' = w-1-x when flipped.  numpy computes `im.astype(f32); im -= PIXEL_MEANS(f64)` in float64
// and rounds once to float32 (naive f32 arithmetic differs in 384 of the 768 (ch, v) cases,
// SURVEY §8a row a13), so the kernel does the same: one f64 subtract, one round-to-nearest cvt.
// One thread per output pixel: 3 bytes in, 12 bytes out (HBM bound: 15 B/pixel).
#include "idn_common.hpp"

namespace idn {

struct BlobArgs {
  double m0, m1, m2;
};

__global__ __launch_bounds__(256) void blob_kernel(const uint8_t* __restrict__ src,
                                                   float* __restrict__ blob, int n, int h, int w,
                                                   int64_t row_stride, int out_h, int out_w,
                                                   BlobArgs m, int flip) {
  const int64_t per_img = (int64_t)out_h * out_w;
  const int64_t total = per_img * n;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int img = (int)(p / per_img);
    const int64_t q = p - (int64_t)img * per_img;
    const int y = (int)(q / out_w), x = (int)(q - (int64_t)y * out_w);
    float v0 = 0.f, v1 = 0.f, v2 = 0.f;
    if (y < h && x < w) {
      const int xs = flip ? (w - 1 - x) : x;
      const uint8_t* s = src + (int64_t)img * h * row_stride + (int64_t)y * row_stride + (int64_t)xs * 3;
      v0 = __double2float_rn(__dsub_rn((double)s[0], m.m0));
      v1 = __double2float_rn(__dsub_rn((double)s[1], m.m1));
      v2 = __double2float_rn(__dsub_rn((double)s[2], m.m2));
    }
    float* o = blob + p * 3;
    o[0] = v0;
    o[1] = v1;
    o[2] = v2;
  }
}

}  // namespace idn

extern "C" int idn_blob_f32(const uint8_t* src, float* blob, int n, int h, int w, int c,
                            int64_t row_stride, int out_h, int out_w, const double mean[3],
                            int flip, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(src && blob && mean, "idn_blob_f32: null pointer");
  IDN_CHECK_ARG(c == 3, "idn_blob_f32: the blob is 3-channel (got c=%d)", c);
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0, "idn_blob_f32: bad shape");
  IDN_CHECK_ARG(out_h >= h && out_w >= w, "idn_blob_f32: blob (%d x %d) smaller than image", out_h,
                out_w);
  IDN_CHECK_ARG(row_stride >= (int64_t)w * c, "idn_blob_f32: row_stride < w*c");
  if (n == 0) return IDN_OK;
  const int64_t total = (int64_t)n * out_h * out_w;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  BlobArgs m{mean[0], mean[1], mean[2]};
  hipLaunchKernelGGL(blob_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), src, blob,
                     n, h, w, row_stride, out_h, out_w, m, flip);
  IDN_CHECK_LAUNCH("idn_blob_f32");
  return IDN_OK;
}
