// Post-process effects: the 12 compute shaders of src/shaders/compute/*.wgsl run as a
// chain (rendering/post_processor.rs:101-129) on RGBA8 images, one HIP pass per effect,
// ping-ponging two device buffers like the reference's two intermediate textures.
//
// Where WGSL leaves behaviour to the implementation, the build defines it (DESIGN.md
// §4.10): u8 -> f32 is u / 255 (IEEE division); f32 -> u8 is rint(clamp(x, 0, 1) * 255)
// (round half to even); loads outside the image read (0, 0, 0, 0); stores outside it
// are dropped and the destination is cleared before every pass; f32 expressions are
// evaluated as written, left to right, without contraction. oracle/post_ref.py restates
// every effect in numpy and tests/test_post.py compares them bit for bit.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "internal.h"

namespace fr {
namespace {

__device__ __forceinline__ float4 load_px(const uchar4* __restrict__ src, int x, int y, int w, int h) {
  if (x < 0 || y < 0 || x >= w || y >= h) return make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  const uchar4 c = src[static_cast<size_t>(y) * w + x];
  return make_float4(static_cast<float>(c.x) / 255.0f, static_cast<float>(c.y) / 255.0f,
                     static_cast<float>(c.z) / 255.0f, static_cast<float>(c.w) / 255.0f);
}

__device__ __forceinline__ uint8_t to_unorm8(float v) {
  const float c = fminf(fmaxf(v, 0.0f), 1.0f);  // NaN -> 0 (fmax/fmin ignore NaN)
  return static_cast<uint8_t>(__builtin_rintf(c * 255.0f));
}

__device__ __forceinline__ void store_px(uchar4* __restrict__ dst, int x, int y, int w, int h, float4 c) {
  if (x < 0 || y < 0 || x >= w || y >= h) return;
  dst[static_cast<size_t>(y) * w + x] = make_uchar4(to_unorm8(c.x), to_unorm8(c.y), to_unorm8(c.z), to_unorm8(c.w));
}

__device__ __forceinline__ float fract(float v) { return v - floorf(v); }

__device__ __forceinline__ float luma(float4 c) { return (c.x * 0.299f + c.y * 0.587f) + c.z * 0.114f; }

// watercolor.comp.wgsl:7-10
__device__ __forceinline__ float hash_wc(float px, float py) {
  const float ax = fract(px * 0.1031f), ay = fract(py * 0.1031f), az = fract(px * 0.1031f);
  const float d = (ax * (ay + 33.333f) + ay * (az + 33.333f)) + az * (ax + 33.333f);  // dot(p3, p3.yzx + 33.333)
  return fract((ax + ay) * d);
}

// noise.comp.wgsl:28-33
__device__ __forceinline__ float hash_noise(uint32_t x, uint32_t y, float time) {
  const float fx = static_cast<float>(x) / 10.0f, fy = static_cast<float>(y) / 10.0f;
  const float vx = fx * 0.3183099f + time * 0.05f, vy = fy * 0.3678794f + time * 0.05f;
  return fract(23.0f * fract((vx * vy) * (vx + vy)));
}

__global__ __launch_bounds__(256) void fx_kernel(int effect, float time, const uchar4* __restrict__ src,
                                                 uchar4* __restrict__ dst, int w, int h) {
  const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (x >= w || y >= h) return;  // `if (id.x >= dims.x || id.y >= dims.y) return;`
  const float4 c = load_px(src, x, y, w, h);
  float4 o = c;
  switch (effect) {
    case FR_FX_NONE: break;
    case FR_FX_NOISE: {  // noise.comp.wgsl:16-26
      const float n = hash_noise(x, y, time) / 20.0f;
      o = make_float4(c.x + n, c.y + n, c.z + n, 1.0f);
      break;
    }
    case FR_FX_PIXELATE:  // pixelate.comp.wgsl:9-23, PIXEL_SIZE 8
      o = load_px(src, (x / 8) * 8, (y / 8) * 8, w, h);
      break;
    case FR_FX_INVERT_COLOR: o = make_float4(1.0f - c.x, 1.0f - c.y, 1.0f - c.z, 1.0f); break;
    case FR_FX_WAVE: {  // wave.comp.wgsl:9-27
      const float l = luma(c);
      o = make_float4(l, l, l, 1.0f);
      if (c.x > 0.4f) o = make_float4(1.0f, c.y, 0.1f * c.z, 1.0f);
      if (c.y > 0.4f) o = make_float4(0.1f, c.y, 0.1f * c.z, 1.0f);
      if (c.z > 0.4f) o = make_float4(0.1f * c.x, c.y, 1.0f, 1.0f);
      break;
    }
    case FR_FX_INTERLACE: {  // interlace.comp.wgsl: select(1.0, 0.0, y % 2 == 0)
      const float f = (y % 2) == 0 ? 0.0f : 1.0f;
      o = make_float4(c.x * f, c.y * f, c.z * f, c.w);
      break;
    }
    case FR_FX_FLIP_AXIS:  // flip_axis.comp.wgsl: stored at (y, x)
      store_px(dst, y, x, w, h, c);
      return;
    case FR_FX_GRAYSCALE: {
      const float l = luma(c);
      o = make_float4(l, l, l, c.w);
      break;
    }
    case FR_FX_STEP: {  // step.comp.wgsl: floor(y / 0.2) * 0.2
      const float b = floorf(luma(c) / 0.2f) * 0.2f;
      o = make_float4(b, b, b, c.w);
      break;
    }
    case FR_FX_WATERCOLOR: {  // watercolor.comp.wgsl:13-54
      const float px = static_cast<float>(x), py = static_cast<float>(y);
      const float qw = static_cast<float>(w) / 4.0f, qh = static_cast<float>(h) / 4.0f;
      for (int i = 0; i < 50; ++i) {
        const float fi = static_cast<float>(i);
        const float csx = fi * 123.45f, csy = 67.89f;
        const float rsx = fi * 234.56f, rsy = 78.9f;
        const float ksx = fi * 345.67f, ksy = 89.01f;
        const float cx = qw + (hash_wc(csx, csy) * qw) * 2.0f;
        const float cy = qh + (hash_wc(csx + 1.0f, csy) * qh) * 2.0f;
        const float radius = 10.0f + hash_wc(rsx, rsy) * 200.0f;
        const float r = hash_wc(ksx, ksy);
        const float dx = px - cx, dy = py - cy;
        if (sqrtf(dx * dx + dy * dy) <= radius) {
          o.x = o.x + r * 0.05f;
          o.y = o.y + 0.0f * 0.05f;
          o.z = o.z + 0.0f * 0.05f;
          o.w = o.w + 1.0f * 0.05f;
        }
      }
      break;
    }
    case FR_FX_CHROMOSTEREOPSIS: {  // saturate(sign(r - b))
      const float diff = c.x - c.z;
      const float r = diff > 0.0f ? 1.0f : 0.0f;
      o = make_float4(r, 0.0f, 1.0f - r, 1.0f);
      break;
    }
    case FR_FX_ANAGLYPH: {  // anaglyph.comp.wgsl: offset 10 pixels
      const float r = load_px(src, x - 10, y, w, h).x;
      const float b = load_px(src, x + 10, y, w, h).z;
      o = make_float4(r, 0.0f, b, 1.0f);
      break;
    }
    default: break;
  }
  store_px(dst, x, y, w, h, o);
}

__global__ __launch_bounds__(256) void rgb_to_rgba_kernel(const uint8_t* __restrict__ rgb, uchar4* __restrict__ rgba,
                                                          size_t n) {
  const size_t i = static_cast<size_t>(blockIdx.x) * 256u + threadIdx.x;
  if (i < n) rgba[i] = make_uchar4(rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2], 255);
}

#define PCHK(x)                                                                                  \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) return set_error(FR_EHIP, "%s: %s", #x, hipGetErrorString(e_));       \
  } while (0)

// Runs the chain on device buffers a (input) and b (scratch); returns which holds the result.
int run_chain(const int* effects, uint32_t n, float time, uchar4* a, uchar4* b, uint32_t w, uint32_t h,
              hipStream_t st, uchar4** result) {
  const dim3 grid((w + 15) / 16, (h + 15) / 16);
  uchar4* src = a;
  uchar4* dst = b;
  for (uint32_t k = 0; k < n; ++k) {
    PCHK(hipMemsetAsync(dst, 0, static_cast<size_t>(w) * h * 4, st));
    hipLaunchKernelGGL(fx_kernel, grid, dim3(256), 0, st, effects[k], time, src, dst, static_cast<int>(w),
                       static_cast<int>(h));
    PCHK(hipGetLastError());
    uchar4* t = src;
    src = dst;
    dst = t;
  }
  *result = src;
  return FR_OK;
}

}  // namespace
}  // namespace fr

using namespace fr;

extern "C" {

int fr_post_process(int device, const int* effects, uint32_t n_effects, float time, uint32_t width, uint32_t height,
                    const uint8_t* rgba_in, uint8_t* rgba_out) {
  if ((n_effects && !effects) || !rgba_in || !rgba_out || width == 0 || height == 0)
    return set_error(FR_EARG, "fr_post_process: bad arguments");
  for (uint32_t k = 0; k < n_effects; ++k)
    if (effects[k] < FR_FX_NONE || effects[k] > FR_FX_ANAGLYPH)
      return set_error(FR_EARG, "fr_post_process: unknown effect %d", effects[k]);
  PCHK(hipSetDevice(device));
  const size_t bytes = static_cast<size_t>(width) * height * 4;
  uchar4* buf = nullptr;
  PCHK(hipMalloc(&buf, 2 * bytes));
  int rc = FR_OK;
  uchar4* res = nullptr;
  if (hipMemcpy(buf, rgba_in, bytes, hipMemcpyHostToDevice) != hipSuccess) {
    rc = set_error(FR_EHIP, "fr_post_process: upload failed");
  } else {
    rc = run_chain(effects, n_effects, time, buf, buf + static_cast<size_t>(width) * height, width, height, 0, &res);
    if (rc == FR_OK && hipMemcpy(rgba_out, res, bytes, hipMemcpyDeviceToHost) != hipSuccess)
      rc = set_error(FR_EHIP, "fr_post_process: download failed");
  }
  (void)hipFree(buf);
  return rc;
}

int fr_rgb_to_rgba_device(void* stream, const uint8_t* d_rgb, uint8_t* d_rgba, size_t pixels) {
  if (!d_rgb || !d_rgba) return set_error(FR_EARG, "fr_rgb_to_rgba_device: null buffer");
  if (pixels)
    hipLaunchKernelGGL(rgb_to_rgba_kernel, dim3(static_cast<uint32_t>((pixels + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), d_rgb, reinterpret_cast<uchar4*>(d_rgba), pixels);
  PCHK(hipGetLastError());
  return FR_OK;
}

int fr_post_process_device(void* stream, const int* effects, uint32_t n_effects, float time, uint32_t width,
                           uint32_t height, uint8_t* d_rgba, uint8_t* d_scratch) {
  if ((n_effects && !effects) || !d_rgba || !d_scratch || width == 0 || height == 0)
    return set_error(FR_EARG, "fr_post_process_device: bad arguments");
  for (uint32_t k = 0; k < n_effects; ++k)
    if (effects[k] < FR_FX_NONE || effects[k] > FR_FX_ANAGLYPH)
      return set_error(FR_EARG, "fr_post_process_device: unknown effect %d", effects[k]);
  hipStream_t st = static_cast<hipStream_t>(stream);
  uchar4* res = nullptr;
  int rc = run_chain(effects, n_effects, time, reinterpret_cast<uchar4*>(d_rgba), reinterpret_cast<uchar4*>(d_scratch),
                     width, height, st, &res);
  if (rc) return rc;
  if (res != reinterpret_cast<uchar4*>(d_rgba))
    PCHK(hipMemcpyAsync(d_rgba, res, static_cast<size_t>(width) * height * 4, hipMemcpyDeviceToDevice, st));
  return FR_OK;
}

}  // extern "C"
