// On-device input preprocessing: decoded camera frames (uint8 HWC, e.g. the
// 1920x1200 SPEED images, grayscale replicated to RGB by utils.py:215) -> torchvision Resize(img_size)
// (speed.py:66-69) = Pillow's BILINEAR ImagingResample, bit-exactly, on the GPU. ToTensor's /255 stays fused
// into the network's stem, so the output is the uint8 NHWC frame spef_forward takes.
//
// Two separable passes with Pillow's integer coefficient tables (PRECISION_BITS = 22, computed on the host
// exactly as precompute_coeffs + normalize_coeffs_8bpc do): horizontal over the source rows the vertical pass
// needs, into an 8-bit temporary image, then vertical. One thread per output pixel (3 channels). HBM-bound:
// the horizontal pass streams the full-resolution frame once.
#include "spef_common.hpp"
#include "spef_kernels.hpp"

namespace spef {

__device__ __forceinline__ uint32_t clip8(int v) {
  v >>= 22;
  return (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// in: [B][Hin][Win][3]; tmp: [B][Ht][Wo][3] from source rows y0 .. y0 + Ht
__global__ __launch_bounds__(256) void resize_h_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ tmp,
                                                       const int* __restrict__ bounds, const int* __restrict__ kk,
                                                       int ksize, int B, int Hin, int Win, int y0, int Ht, int Wo) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)B * Ht * Wo) return;
  const int x = (int)(t % Wo);
  const int64_t r = t / Wo;                 // b * Ht + row
  const int row = (int)(r % Ht), b = (int)(r / Ht);
  const int xmin = bounds[2 * x], n = bounds[2 * x + 1];
  const uint8_t* src = in + (((size_t)b * Hin + y0 + row) * Win + xmin) * 3;
  const int* k = kk + (size_t)x * ksize;
  int s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
  for (int i = 0; i < n; ++i) {
    const int w = k[i];
    s0 += (int)src[3 * i] * w;
    s1 += (int)src[3 * i + 1] * w;
    s2 += (int)src[3 * i + 2] * w;
  }
  uint8_t* dst = tmp + t * 3;
  dst[0] = (uint8_t)clip8(s0);
  dst[1] = (uint8_t)clip8(s1);
  dst[2] = (uint8_t)clip8(s2);
}

// tmp: [B][Ht][Wo][3] -> out [B][Ho][Wo][3]
__global__ __launch_bounds__(256) void resize_v_kernel(const uint8_t* __restrict__ tmp, uint8_t* __restrict__ out,
                                                       const int* __restrict__ bounds, const int* __restrict__ kk,
                                                       int ksize, int B, int Ht, int Ho, int Wo) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)B * Ho * Wo) return;
  const int x = (int)(t % Wo);
  const int64_t r = t / Wo;
  const int y = (int)(r % Ho), b = (int)(r / Ho);
  const int ymin = bounds[2 * y], n = bounds[2 * y + 1];
  const uint8_t* src = tmp + (((size_t)b * Ht + ymin) * Wo + x) * 3;
  const int* k = kk + (size_t)y * ksize;
  const size_t rs = (size_t)Wo * 3;
  int s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
  for (int i = 0; i < n; ++i) {
    const int w = k[i];
    s0 += (int)src[i * rs] * w;
    s1 += (int)src[i * rs + 1] * w;
    s2 += (int)src[i * rs + 2] * w;
  }
  uint8_t* dst = out + t * 3;
  dst[0] = (uint8_t)clip8(s0);
  dst[1] = (uint8_t)clip8(s1);
  dst[2] = (uint8_t)clip8(s2);
}

hipError_t launch_resize_h(const uint8_t* in, uint8_t* tmp, const int* bounds, const int* kk, int ksize, int B,
                           int Hin, int Win, int y0, int Ht, int Wo, hipStream_t s) {
  const int64_t n = (int64_t)B * Ht * Wo, nb = (n + 255) / 256;
  if (nb > 0x7fffffff) return hipErrorInvalidValue;
  if (n > 0) resize_h_kernel<<<(unsigned)nb, 256, 0, s>>>(in, tmp, bounds, kk, ksize, B, Hin, Win, y0, Ht, Wo);
  return hipGetLastError();
}

hipError_t launch_resize_v(const uint8_t* tmp, uint8_t* out, const int* bounds, const int* kk, int ksize, int B,
                           int Ht, int Ho, int Wo, hipStream_t s) {
  const int64_t n = (int64_t)B * Ho * Wo, nb = (n + 255) / 256;
  if (nb > 0x7fffffff) return hipErrorInvalidValue;
  if (n > 0) resize_v_kernel<<<(unsigned)nb, 256, 0, s>>>(tmp, out, bounds, kk, ksize, B, Ht, Ho, Wo);
  return hipGetLastError();
}

}  // namespace spef
