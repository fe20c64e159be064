// Remaining elementwise / per-pixel stages of the dispatcher:
//   shader  add_shader (lib/model/test.py:1595-1601, minibatch.py:1505-1511):
//           np.array(ImageEnhance.Brightness(PIL.Image.open(path)).enhance(3)) -- an RGB array
//   bloom   add_bloom -> Automold add_sun_flare (tools/Automold.py:588-627, add_sun_process 575-586,
//           flare_source 553-563): 48 sequential cv2.circle + cv2.addWeighted passes, evaluated per
//           pixel in one pass (the circles are host-drawn span tables, see idn/automold.py)
//   blob    from a float64 image (test_v0 / train_v0 "plain" branches hand random_noise's float64
//           output to prep_im_for_blob: f32(f64(f32(x)) - mean))
#include "idn_common.hpp"

namespace idn {

// Pillow ImagingBlend(black, image, alpha): interpolation for 0 <= alpha <= 1, clipped
// extrapolation otherwise; float arithmetic, truncating casts.  Output channel order is RGB.
__global__ __launch_bounds__(256) void shader_kernel(const uint8_t* __restrict__ src,
                                                     uint8_t* __restrict__ dst, int n, int h, int w,
                                                     int64_t row_stride, float alpha, int extrap) {
  const int64_t total = (int64_t)n * h * w;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(p % w);
    const int64_t t = p / w;
    const int y = (int)(t % h);
    const int img = (int)(t / h);
    const int64_t off = (int64_t)img * h * row_stride + (int64_t)y * row_stride + (int64_t)x * 3;
    const uint8_t* s = src + off;
    uint8_t* d = dst + off;
    uint8_t o[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float v = (float)s[2 - k];  // BGR (cv2.imread) -> RGB (PIL)
      const float temp = 0.0f + alpha * (v - 0.0f);
      if (extrap) o[k] = temp <= 0.0f ? 0 : (temp >= 255.0f ? 255 : (uint8_t)temp);
      else o[k] = (uint8_t)(int)temp;
    }
    d[0] = o[0];
    d[1] = o[1];
    d[2] = o[2];
  }
}

// circles: per image ncirc records of 8 int32 {cx, cy, radius, b, g, r, reset_overlay, 0};
// weights: per image ncirc {alpha, beta} floats (cv2.addWeighted's float-cast scalars);
// spans: half-width of a filled LINE_8 circle of radius R at row offset t, at spans[R*(R+1)/2 + t]
__global__ __launch_bounds__(256) void bloom_kernel(const uint8_t* __restrict__ src,
                                                    uint8_t* __restrict__ dst, int n, int h, int w,
                                                    int64_t row_stride,
                                                    const int32_t* __restrict__ circles,
                                                    const float* __restrict__ weights, int ncirc,
                                                    const int16_t* __restrict__ spans) {
  const int64_t total = (int64_t)n * h * w;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(p % w);
    const int64_t t = p / w;
    const int y = (int)(t % h);
    const int img = (int)(t / h);
    const int64_t off = (int64_t)img * h * row_stride + (int64_t)y * row_stride + (int64_t)x * 3;
    float ov[3], out[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) ov[k] = out[k] = (float)src[off + k];
    const int32_t* cr = circles + (int64_t)img * ncirc * 8;
    const float* wt = weights + (int64_t)img * ncirc * 2;
    for (int c = 0; c < ncirc; ++c) {
      const int32_t* q = cr + 8 * c;
      if (q[6]) {  // flare_source starts a new overlay from the current output
        ov[0] = out[0];
        ov[1] = out[1];
        ov[2] = out[2];
      }
      const int dy = y - q[1], R = q[2];
      const int ady = dy < 0 ? -dy : dy;
      if (ady <= R) {
        const int half = spans[R * (R + 1) / 2 + ady];
        const int dx = x - q[0];
        if (dx >= -half && dx <= half) {
          ov[0] = (float)q[3];
          ov[1] = (float)q[4];
          ov[2] = (float)q[5];
        }
      }
      const float a = wt[2 * c], b = wt[2 * c + 1];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        // cv2.addWeighted(overlay, a, output, b, 0): saturate_cast<uchar>(s1*a + s2*b + 0)
        const float v = ov[k] * a + out[k] * b + 0.0f;
        float r = __builtin_rintf(v);
        r = r < 0.f ? 0.f : (r > 255.f ? 255.f : r);
        out[k] = r;
      }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) dst[off + k] = (uint8_t)out[k];
  }
}

struct BlobMean {
  double m0, m1, m2;
};

__global__ __launch_bounds__(256) void blob_f64_kernel(const double* __restrict__ src,
                                                       float* __restrict__ blob, int n, int h, int w,
                                                       int out_h, int out_w, BlobMean m, int flip) {
  const int64_t per_img = (int64_t)out_h * out_w;
  const int64_t total = per_img * n;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int img = (int)(p / per_img);
    const int64_t q = p - (int64_t)img * per_img;
    const int y = (int)(q / out_w), x = (int)(q - (int64_t)y * out_w);
    float v[3] = {0.f, 0.f, 0.f};
    if (y < h && x < w) {
      const int xs = flip ? (w - 1 - x) : x;
      const double* s = src + (((int64_t)img * h + y) * w + xs) * 3;
      const double mm[3] = {m.m0, m.m1, m.m2};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        // im.astype(np.float32); im -= PIXEL_MEANS  ->  f32(f64(f32(x)) - mean)
        const double xf = (double)__double2float_rn(s[k]);
        v[k] = __double2float_rn(__dsub_rn(xf, mm[k]));
      }
    }
    float* o = blob + p * 3;
    o[0] = v[0];
    o[1] = v[1];
    o[2] = v[2];
  }
}

static unsigned blocks_for(int64_t work) {
  int64_t b = (work + 255) / 256;
  if (b < 1) b = 1;
  return (unsigned)(b > 65536 ? 65536 : b);
}

}  // namespace idn

extern "C" int idn_shader_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                             int64_t row_stride, double factor, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(src && dst, "idn_shader_u8: null pointer");
  IDN_CHECK_ARG(c == 3, "idn_shader_u8: needs 3 channels");
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0 && row_stride >= (int64_t)w * 3, "idn_shader_u8: bad shape");
  if (n == 0) return IDN_OK;
  const float alpha = (float)factor;
  const int extrap = !(alpha >= 0.f && alpha <= 1.0f);
  hipLaunchKernelGGL(shader_kernel, dim3(blocks_for((int64_t)n * h * w)), dim3(256), 0,
                     as_stream(stream), src, dst, n, h, w, row_stride, alpha, extrap);
  IDN_CHECK_LAUNCH("idn_shader_u8");
  return IDN_OK;
}

extern "C" int idn_bloom_u8(const uint8_t* src, uint8_t* dst, int n, int h, int w, int c,
                            int64_t row_stride, const int32_t* circles, const float* weights,
                            int ncirc, const int16_t* spans, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(src && dst && circles && weights && spans, "idn_bloom_u8: null pointer");
  IDN_CHECK_ARG(c == 3, "idn_bloom_u8: needs 3 channels");
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0 && row_stride >= (int64_t)w * 3 && ncirc >= 0,
                "idn_bloom_u8: bad shape");
  if (n == 0) return IDN_OK;
  hipLaunchKernelGGL(bloom_kernel, dim3(blocks_for((int64_t)n * h * w)), dim3(256), 0,
                     as_stream(stream), src, dst, n, h, w, row_stride, circles, weights, ncirc, spans);
  IDN_CHECK_LAUNCH("idn_bloom_u8");
  return IDN_OK;
}

extern "C" int idn_blob_from_f64(const double* src, float* blob, int n, int h, int w, int out_h,
                                 int out_w, const double mean[3], int flip, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(src && blob && mean, "idn_blob_from_f64: null pointer");
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0 && out_h >= h && out_w >= w, "idn_blob_from_f64: bad shape");
  if (n == 0) return IDN_OK;
  BlobMean m{mean[0], mean[1], mean[2]};
  hipLaunchKernelGGL(blob_f64_kernel, dim3(blocks_for((int64_t)n * out_h * out_w)), dim3(256), 0,
                     as_stream(stream), src, blob, n, h, w, out_h, out_w, m, flip);
  IDN_CHECK_LAUNCH("idn_blob_from_f64");
  return IDN_OK;
}

// ---- cv2.resize(f32, fx, fy, INTER_LINEAR) (lib/utils/blob.py:44-45, lib/model/test.py:75-76) ----
// OpenCV 3.4.2 resizeGeneric_ float path: fx = (float)((dx + 0.5) * scale_x - 0.5), sx = floor,
// coefficients (1 - f, f) in float, source index clamped at the borders (where the tap weight is 0
// or the single tap is copied), horizontal pass then vertical pass, float arithmetic.
namespace idn {
__device__ __forceinline__ void lin_coef(int d, double scale, int n, int& s0, int& s1, float& a0,
                                         float& a1) {
  float f = (float)((d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f -= (float)s;
  if (s < 0) {
    f = 0.f;
    s = 0;
  }
  if (s >= n - 1) {
    f = 0.f;
    s = n - 1;
  }
  s0 = s;
  s1 = s + 1 < n ? s + 1 : n - 1;
  a0 = 1.f - f;
  a1 = f;
}

__global__ __launch_bounds__(256) void resize_linear_f32_kernel(const float* __restrict__ src,
                                                                float* __restrict__ dst, int n,
                                                                int h, int w, int c, int oh, int ow,
                                                                double scale_x, double scale_y) {
  const int64_t total = (int64_t)n * oh * ow;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int dx = (int)(p % ow);
    const int64_t t = p / ow;
    const int dy = (int)(t % oh);
    const int img = (int)(t / oh);
    int x0, x1, y0, y1;
    float ax0, ax1, by0, by1;
    lin_coef(dx, scale_x, w, x0, x1, ax0, ax1);
    lin_coef(dy, scale_y, h, y0, y1, by0, by1);
    const bool xcopy = (ax1 == 0.f && x0 == w - 1);  // OpenCV copies S[xofs] past xmax
    const float* s = src + (int64_t)img * h * w * c;
    for (int ch = 0; ch < c; ++ch) {
      const float* r0 = s + ((int64_t)y0 * w) * c + ch;
      const float* r1 = s + ((int64_t)y1 * w) * c + ch;
      const float h0 = xcopy ? r0[(int64_t)x0 * c] : r0[(int64_t)x0 * c] * ax0 + r0[(int64_t)x1 * c] * ax1;
      const float h1 = xcopy ? r1[(int64_t)x0 * c] : r1[(int64_t)x0 * c] * ax0 + r1[(int64_t)x1 * c] * ax1;
      dst[(((int64_t)img * oh + dy) * ow + dx) * c + ch] = h0 * by0 + h1 * by1;
    }
  }
}
}  // namespace idn

extern "C" int idn_resize_linear_f32(const float* src, float* dst, int n, int h, int w, int c,
                                     int out_h, int out_w, double fx, double fy, void* stream) {
  using namespace idn;
  IDN_CHECK_ARG(src && dst, "idn_resize_linear_f32: null pointer");
  IDN_CHECK_ARG(n >= 0 && h > 0 && w > 0 && c > 0 && out_h > 0 && out_w > 0 && fx > 0 && fy > 0,
                "idn_resize_linear_f32: bad shape");
  if (n == 0) return IDN_OK;
  hipLaunchKernelGGL(resize_linear_f32_kernel, dim3(blocks_for((int64_t)n * out_h * out_w)),
                     dim3(256), 0, as_stream(stream), src, dst, n, h, w, c, out_h, out_w, 1.0 / fx,
                     1.0 / fy);
  IDN_CHECK_LAUNCH("idn_resize_linear_f32");
  return IDN_OK;
}
