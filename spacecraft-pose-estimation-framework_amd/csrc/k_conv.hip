// Backbone kernels for MobileNet-V2 (src/modeling/backbone/mobilenet_v2.py:232-271) on gfx950.
//
//   stem_kernel     ConvBnAct 3->32 3x3/s2 (pytorch_layers.py:35-62), VALU fp32, input u8 NHWC or f32 NCHW
//   pw_kernel       1x1 ConvBnAct / projection (+residual add, pytorch_layers.py:78-96) as an MFMA GEMM
//   dw_kernel       depthwise 3x3 ConvBnAct (pytorch_layers.py:82-83), VALU fp32 over 8-channel vectors
//   pw_pool_kernel  last 1x1 ConvBnAct 320->1280 fused with URSONetHead's mean([2,3]) (ursonet.py:30)
//
// BatchNorm is folded into the conv weights/bias at build time (spef_amd/blob.py).
#include "spef_common.hpp"
#include "spef_kernels.hpp"

namespace spef {

// ------------------------------------------------------------------------------------------ stem
template <typename DT, int LAYOUT>
__global__ __launch_bounds__(256) void stem_kernel(const void* __restrict__ in, const float* __restrict__ w,
                                                   const float* __restrict__ bias, typename DT::T* __restrict__ y,
                                                   int B, int H, int W, int OH, int OW) {
  using T = typename DT::T;
  __shared__ float sw[27 * 32];
  __shared__ float sb[32];
  for (int i = threadIdx.x; i < 27 * 32; i += 256) sw[i] = w[i];
  if (threadIdx.x < 32) sb[threadIdx.x] = bias[threadIdx.x];
  __syncthreads();
  // grid = output rows x ceil(OW * 4 / 256) blocks per row (workgroup-uniform row split, as dw_kernel)
  const int RW = OW * 4, nbx = (RW + 255) >> 8;
  const int row = (int)blockIdx.x / nbx, t = ((int)blockIdx.x - row * nbx) * 256 + (int)threadIdx.x;
  if (t >= RW) return;
  const int g = t & 3, ox = t >> 2;
  const int oy = row % OH, b = row / OH;

  float xin[27];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = 2 * oy - 1 + ky;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int ix = 2 * ox - 1 + kx;
      const bool v = (iy >= 0) && (iy < H) && (ix >= 0) && (ix < W);
#pragma unroll
      for (int ci = 0; ci < 3; ++ci) {
        float val = 0.0f;
        if (v) {
          if (LAYOUT == IN_U8_NHWC) {
            const uint8_t* src = (const uint8_t*)in;
            // ToTensor(): uint8 / 255 in fp32 (datasets/speed.py:66-69)
            val = (float)src[(((int64_t)b * H + iy) * W + ix) * 3 + ci] / 255.0f;
          } else {
            const float* src = (const float*)in;
            val = src[(((int64_t)b * 3 + ci) * H + iy) * W + ix];
          }
        }
        xin[ky * 9 + kx * 3 + ci] = val;
      }
    }
  }
  float acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = 0.0f;
#pragma unroll
  for (int k = 0; k < 27; ++k) {
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = fmaf(xin[k], sw[k * 32 + 8 * g + c], acc[c]);
  }
  typename DT::x8 o;
#pragma unroll
  for (int c = 0; c < 8; ++c) o[c] = (T)fmaxf(acc[c] + sb[8 * g + c], 0.0f);
  *reinterpret_cast<typename DT::x8*>(y + (((int64_t)b * OH + oy) * OW + ox) * 32 + 8 * g) = o;
}

// ------------------------------------------------------------------------------------------ pointwise
// C^T[n][m] = sum_k W[n][k] X[m][k]: output channels on the MFMA row axis (A = weights), pixels on the
// column axis (B = activations). Each lane loads 16 contiguous bytes of an NHWC pixel row (B fragment) and
// stores 4 consecutive output channels of one pixel (8 bytes) -- no LDS transpose needed.
// A wave owns NT channel tiles x MT pixel tiles (16x16 each); a 256-thread workgroup = 4 waves on
// 4*MT*16 consecutive pixels; channel chunks of NT*16 are the fastest-varying logical id so the chunks of
// one pixel tile run back to back on one XCD and re-read X from its L2.
template <typename DT, int NT, int MT, int EPI>
__global__ __launch_bounds__(256) void pw_kernel(const typename DT::T* __restrict__ X, const typename DT::T* __restrict__ Wt,
                                                 const float* __restrict__ bias, const typename DT::T* __restrict__ R,
                                                 typename DT::T* __restrict__ Y, int64_t M, int K, int N, int Kp,
                                                 int n_chunks, uint32_t nwg) {
  using T = typename DT::T;
  using x8 = typename DT::x8;
  using x4 = typename DT::x4;
  const uint32_t L = xcd_remap(blockIdx.x, nwg);
  const int chunk = (int)(L % (uint32_t)n_chunks);
  const int64_t ptile = L / (uint32_t)n_chunks;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  const int n0 = chunk * 16 * NT;
  const int64_t m0 = ptile * (64 * MT) + (int64_t)wave * 16 * MT;

  f32x4 acc[NT][MT];   // accumulators start at the folded-BN bias
#pragma unroll
  for (int a = 0; a < NT; ++a) {
    const float4 bb = *reinterpret_cast<const float4*>(bias + n0 + 16 * a + 4 * kg);
#pragma unroll
    for (int b = 0; b < MT; ++b) acc[a][b] = f32x4{bb.x, bb.y, bb.z, bb.w};
  }

  const T* wp = Wt + (size_t)(n0 + r16) * Kp + 8 * kg;
  const T* xp[MT];
  bool mv[MT];
#pragma unroll
  for (int b = 0; b < MT; ++b) {
    const int64_t m = m0 + 16 * b + r16;
    mv[b] = m < M;
    xp[b] = X + (size_t)(mv[b] ? m : 0) * K + 8 * kg;
  }
  const int KS = Kp >> 5;
#pragma unroll 2
  for (int ks = 0; ks < KS; ++ks) {
    const bool kv = (ks * 32 + 8 * kg) < K;
    x8 av[NT], bv[MT];
#pragma unroll
    for (int a = 0; a < NT; ++a) av[a] = load8<DT>(wp + (size_t)a * 16 * Kp + ks * 32);
#pragma unroll
    for (int b = 0; b < MT; ++b) bv[b] = (kv && mv[b]) ? load8<DT>(xp[b] + ks * 32) : zero8<DT>();
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int b = 0; b < MT; ++b) acc[a][b] = DT::mfma(av[a], bv[b], acc[a][b]);
  }

#pragma unroll
  for (int a = 0; a < NT; ++a) {
    const int i = n0 + 16 * a + 4 * kg;
    if (i >= N) continue;
#pragma unroll
    for (int b = 0; b < MT; ++b) {
      const int64_t m = m0 + 16 * b + r16;
      if (m >= M) continue;
      f32x4 v = acc[a][b];
      if (EPI == EPI_RELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.0f);
      }
      if (EPI == EPI_RES) {
        const x4 rr = *reinterpret_cast<const x4*>(R + (size_t)m * N + i);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (float)rr[e];
      }
      x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (T)v[e];
      *reinterpret_cast<x4*>(Y + (size_t)m * N + i) = o;
    }
  }
}

// ------------------------------------------------------------------------------------------ depthwise
template <typename DT, int S, int MODE = DW_FP32>
__global__ __launch_bounds__(256) void dw_kernel(const typename DT::T* __restrict__ X, const typename DT::DW* __restrict__ W9,
                                                 const float* __restrict__ bias, typename DT::T* __restrict__ Y,
                                                 int B, int H, int W, int C, int OH, int OW) {
  using T = typename DT::T;
  // grid = output rows x ceil(OW * C/8 / 256) blocks per row: the row split is workgroup-uniform (scalar), the
  // per-thread (column, channel group) split one 32-bit division (64-bit div/mod per thread cost more than the
  // arithmetic on the fp32 path)
  const int CG = C >> 3, RW = OW * CG, nbx = (RW + 255) >> 8;
  const int row = (int)blockIdx.x / nbx, t = ((int)blockIdx.x - row * nbx) * 256 + (int)threadIdx.x;
  if (t >= RW) return;
  const int ox = t / CG, cg = t - ox * CG;
  const int oy = row % OH, b = row / OH;
  const int c = cg * 8;
  if constexpr (MODE == DW_PK16) {
    // packed fp16 (k_irb.hip, fp16 stride-2 blocks): 4 x v_pk_fma_f16 per tap, accumulator = the bias rounded to
    // fp16, kx outer / ky inner, taps outside the image multiply a zero -- the fused kernel's operations and order
    const float4 b0 = *reinterpret_cast<const float4*>(bias + c);
    const float4 b1 = *reinterpret_cast<const float4*>(bias + c + 4);
    f16x2 a[4] = {f16x2{(_Float16)b0.x, (_Float16)b0.y}, f16x2{(_Float16)b0.z, (_Float16)b0.w},
                  f16x2{(_Float16)b1.x, (_Float16)b1.y}, f16x2{(_Float16)b1.z, (_Float16)b1.w}};
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int ix = ox * S - 1 + kx;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int iy = oy * S - 1 + ky;
        const bool in = ix >= 0 && ix < W && iy >= 0 && iy < H;
        const uint4 xv = in ? *reinterpret_cast<const uint4*>(X + (((int64_t)b * H + iy) * W + ix) * C + c)
                            : make_uint4(0, 0, 0, 0);
        const uint4 wv = *reinterpret_cast<const uint4*>(W9 + (ky * 3 + kx) * C + c);
        pk_fma4(a, xv, wv);
      }
    }
    *reinterpret_cast<uint4*>(Y + (((int64_t)b * OH + oy) * OW + ox) * C + c) = relu_pk4(a);
    return;
  }
  float acc[8];
  {
    const float4 b0 = *reinterpret_cast<const float4*>(bias + c);
    const float4 b1 = *reinterpret_cast<const float4*>(bias + c + 4);
    acc[0] = b0.x; acc[1] = b0.y; acc[2] = b0.z; acc[3] = b0.w;
    acc[4] = b1.x; acc[5] = b1.y; acc[6] = b1.z; acc[7] = b1.w;
  }
  if constexpr (MODE == DW_PAIRS) {
    // vertical pairs (k_irb.hip, fp16 blocks 2-7): per kernel column, even output rows (and every stride-2 row)
    // dot2(ky 0, 1) then fma(ky 2); odd stride-1 rows fma(ky 0) then dot2(ky 1, 2). Rows outside the image are 0
    // (the fused kernels' zero padding), so the same instructions see the same operands.
    const bool odd = S == 1 && (oy & 1);
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int ix = ox * S - 1 + kx;
      if (ix < 0 || ix >= W) continue;
      f16x8 xv[3], wv[3];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int iy = oy * S - 1 + ky;
        xv[ky] = (iy >= 0 && iy < H) ? *reinterpret_cast<const f16x8*>(X + (((int64_t)b * H + iy) * W + ix) * C + c)
                                     : f16x8{};
        wv[ky] = *reinterpret_cast<const f16x8*>(W9 + (ky * 3 + kx) * C + c);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (!odd) {
          acc[e] = dot2h(pack_h2(xv[0][e], xv[1][e]), pack_h2(wv[0][e], wv[1][e]), acc[e]);
          acc[e] = fmaf((float)xv[2][e], (float)wv[2][e], acc[e]);
        } else {
          acc[e] = fmaf((float)xv[0][e], (float)wv[0][e], acc[e]);
          acc[e] = dot2h(pack_h2(xv[1][e], xv[2][e]), pack_h2(wv[1][e], wv[2][e]), acc[e]);
        }
      }
    }
  } else
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {        // kx outer, ky inner: the fused kernels' accumulation order
    const int ix = ox * S - 1 + kx;
    if (ix < 0 || ix >= W) continue;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = oy * S - 1 + ky;
      if (iy < 0 || iy >= H) continue;
      const typename DT::x8 v = load8<DT>(X + (((int64_t)b * H + iy) * W + ix) * C + c);
      float wv[8];
      load_dw8<DT>(W9 + (ky * 3 + kx) * C + c, wv);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf((float)v[e], wv[e], acc[e]);
    }
  }
  typename DT::x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (T)fmaxf(acc[e], 0.0f);
  *reinterpret_cast<typename DT::x8*>(Y + (((int64_t)b * OH + oy) * OW + ox) * C + c) = o;
}

// ------------------------------------------------------------------------------------------ last conv + mean
// grid (Np / (16*NT), B). The 4 waves split the image's pixel tiles; ReLU(conv + bias) is summed over
// pixels in fp32 registers (the 1280-channel map is never stored), reduced over the 16 pixel lanes by
// shuffles and over the 4 waves through LDS: deterministic, no atomics.
template <typename DT, int NT>
__global__ __launch_bounds__(256) void pw_pool_kernel(const typename DT::T* __restrict__ X, const typename DT::T* __restrict__ Wt,
                                                      const float* __restrict__ bias, float* __restrict__ pooled,
                                                      int HW, int K, int Kp, int N) {
  using T = typename DT::T;
  using x8 = typename DT::x8;
  __shared__ float red[4][NT * 16];
  const int b = blockIdx.y;
  const int n0 = blockIdx.x * 16 * NT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  const T* Xb = X + (size_t)b * HW * K;
  const T* wp = Wt + (size_t)(n0 + r16) * Kp + 8 * kg;
  f32x4 sum[NT];
  f32x4 bb[NT];
#pragma unroll
  for (int a = 0; a < NT; ++a) {
    sum[a] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float4 t = *reinterpret_cast<const float4*>(bias + n0 + 16 * a + 4 * kg);
    bb[a] = f32x4{t.x, t.y, t.z, t.w};
  }
  const int KS = Kp >> 5;
  for (int pt = wave; pt * 16 < HW; pt += 4) {
    const int j = pt * 16 + r16;
    const bool jv = j < HW;
    const T* xp = Xb + (size_t)(jv ? j : 0) * K + 8 * kg;
    f32x4 acc[NT];
#pragma unroll
    for (int a = 0; a < NT; ++a) acc[a] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int ks = 0; ks < KS; ++ks) {
      const bool kv = (ks * 32 + 8 * kg) < K;
      const x8 bv = (kv && jv) ? load8<DT>(xp + ks * 32) : zero8<DT>();
#pragma unroll
      for (int a = 0; a < NT; ++a) acc[a] = DT::mfma(load8<DT>(wp + (size_t)a * 16 * Kp + ks * 32), bv, acc[a]);
    }
    if (jv) {
#pragma unroll
      for (int a = 0; a < NT; ++a)
#pragma unroll
        for (int e = 0; e < 4; ++e) sum[a][e] += fmaxf(acc[a][e] + bb[a][e], 0.0f);
    }
  }
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float s = sum[a][e];
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      s += __shfl_xor(s, 4, 64);
      s += __shfl_xor(s, 8, 64);
      if (r16 == 0) red[wave][16 * a + 4 * kg + e] = s;
    }
  __syncthreads();
  if (threadIdx.x < NT * 16) {
    const int n = n0 + threadIdx.x;
    const float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    if (n < N) pooled[(size_t)b * N + n] = s / (float)HW;
  }
}

template <typename DT>
__global__ void to_f32_kernel(const typename DT::T* __restrict__ x, float* __restrict__ y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) y[i] = (float)x[i];
}

// ------------------------------------------------------------------------------------------ launchers
static inline unsigned blocks_for(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

hipError_t launch_stem(int dtype, int in_layout, const void* in, const float* w, const float* bias, void* y, int B,
                       int H, int W, int OH, int OW, hipStream_t s) {
  const int64_t g64 = (int64_t)B * OH * (((int64_t)OW * 4 + 255) / 256);
  if (g64 > 0x7fffffff) return hipErrorInvalidValue;
  const unsigned g = (unsigned)g64;
  if (dtype == DT_F32) {
    if (in_layout == IN_U8_NHWC)
      stem_kernel<F32, IN_U8_NHWC><<<g, 256, 0, s>>>(in, w, bias, (float*)y, B, H, W, OH, OW);
    else
      stem_kernel<F32, IN_F32_NCHW><<<g, 256, 0, s>>>(in, w, bias, (float*)y, B, H, W, OH, OW);
  } else if (dtype == DT_F16) {
    if (in_layout == IN_U8_NHWC)
      stem_kernel<F16, IN_U8_NHWC><<<g, 256, 0, s>>>(in, w, bias, (_Float16*)y, B, H, W, OH, OW);
    else
      stem_kernel<F16, IN_F32_NCHW><<<g, 256, 0, s>>>(in, w, bias, (_Float16*)y, B, H, W, OH, OW);
  } else {
    if (in_layout == IN_U8_NHWC)
      stem_kernel<BF16, IN_U8_NHWC><<<g, 256, 0, s>>>(in, w, bias, (__bf16*)y, B, H, W, OH, OW);
    else
      stem_kernel<BF16, IN_F32_NCHW><<<g, 256, 0, s>>>(in, w, bias, (__bf16*)y, B, H, W, OH, OW);
  }
  return hipGetLastError();
}

template <typename DT, int NT, int MT>
static hipError_t pw_go(int epi, const void* x, const void* wt, const float* bias, const void* r, void* y, int64_t M,
                        int K, int N, hipStream_t s) {
  using T = typename DT::T;
  const int Kp = (K + 31) & ~31, Np = (N + 15) & ~15;
  const int n_chunks = Np / (16 * NT);
  const int64_t ptiles = (M + 64 * MT - 1) / (64 * MT);
  const int64_t nwg64 = ptiles * n_chunks;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  const T* X = (const T*)x;
  const T* Wt = (const T*)wt;
  if (epi == EPI_RELU)
    pw_kernel<DT, NT, MT, EPI_RELU><<<nwg, 256, 0, s>>>(X, Wt, bias, nullptr, (T*)y, M, K, N, Kp, n_chunks, nwg);
  else if (epi == EPI_RES)
    pw_kernel<DT, NT, MT, EPI_RES><<<nwg, 256, 0, s>>>(X, Wt, bias, (const T*)r, (T*)y, M, K, N, Kp, n_chunks, nwg);
  else
    pw_kernel<DT, NT, MT, EPI_NONE><<<nwg, 256, 0, s>>>(X, Wt, bias, nullptr, (T*)y, M, K, N, Kp, n_chunks, nwg);
  return hipGetLastError();
}

template <typename DT>
static hipError_t pw_dispatch(int epi, const void* x, const void* wt, const float* bias, const void* r, void* y,
                              int64_t M, int K, int N, hipStream_t s) {
  const int n16 = ((N + 15) & ~15) / 16;
  // tile choice per output width (register budget: NT*MT accumulators <= 16)
  if (n16 == 1) return pw_go<DT, 1, 4>(epi, x, wt, bias, r, y, M, K, N, s);
  if (n16 == 2) return pw_go<DT, 2, 4>(epi, x, wt, bias, r, y, M, K, N, s);
  if (n16 == 4) return pw_go<DT, 4, 4>(epi, x, wt, bias, r, y, M, K, N, s);
  if (n16 % 6 == 0) return pw_go<DT, 6, 2>(epi, x, wt, bias, r, y, M, K, N, s);
  if (n16 % 5 == 0) return pw_go<DT, 5, 2>(epi, x, wt, bias, r, y, M, K, N, s);
  if (n16 % 4 == 0) return pw_go<DT, 4, 4>(epi, x, wt, bias, r, y, M, K, N, s);
  if (n16 % 3 == 0) return pw_go<DT, 3, 4>(epi, x, wt, bias, r, y, M, K, N, s);
  if (n16 % 2 == 0) return pw_go<DT, 2, 4>(epi, x, wt, bias, r, y, M, K, N, s);
  return pw_go<DT, 1, 4>(epi, x, wt, bias, r, y, M, K, N, s);
}

hipError_t launch_pw(int dtype, int epi, const void* x, const void* wt, const float* bias, const void* r, void* y,
                     int64_t M, int K, int N, hipStream_t s) {
  if (M <= 0) return hipSuccess;
  if ((K & 7) || (N & 3)) return hipErrorInvalidValue;
  return dtype == DT_F16 ? pw_dispatch<F16>(epi, x, wt, bias, r, y, M, K, N, s)
                         : pw_dispatch<BF16>(epi, x, wt, bias, r, y, M, K, N, s);
}

hipError_t launch_dw(int dtype, const void* x, const void* w9, const float* bias, void* y, int B, int H, int W, int C,
                     int stride, int OH, int OW, int mode, hipStream_t s) {
  if (C & 7) return hipErrorInvalidValue;
  if (mode != DW_FP32 && (dtype != DT_F16 || (mode != DW_PAIRS && mode != DW_PK16))) return hipErrorInvalidValue;
  const int64_t g64 = (int64_t)B * OH * (((int64_t)OW * (C / 8) + 255) / 256);
  if (g64 > 0x7fffffff || (int64_t)OW * (C / 8) > 0x7fffffff) return hipErrorInvalidValue;
  const unsigned g = (unsigned)g64;
#define SPEF_DW(DT_, TT, WT, M_)                                                                                     \
  (stride == 1 ? dw_kernel<DT_, 1, M_><<<g, 256, 0, s>>>((const TT*)x, (const WT*)w9, bias, (TT*)y, B, H, W, C, OH, OW) \
               : dw_kernel<DT_, 2, M_><<<g, 256, 0, s>>>((const TT*)x, (const WT*)w9, bias, (TT*)y, B, H, W, C, OH, OW))
  if (mode == DW_PAIRS) SPEF_DW(F16, _Float16, _Float16, DW_PAIRS);
  else if (mode == DW_PK16) SPEF_DW(F16, _Float16, _Float16, DW_PK16);
  else if (dtype == DT_F32) SPEF_DW(F32, float, float, DW_FP32);
  else if (dtype == DT_F16) SPEF_DW(F16, _Float16, _Float16, DW_FP32);
  else SPEF_DW(BF16, __bf16, float, DW_FP32);
#undef SPEF_DW
  return hipGetLastError();
}

hipError_t launch_pw_pool(int dtype, const void* x, const void* wt, const float* bias, float* pooled, int B, int HW,
                          int K, int N, hipStream_t s) {
  const int Kp = (K + 31) & ~31, Np = (N + 15) & ~15;
  if ((K & 7) || (Np % 64)) return hipErrorInvalidValue;
  dim3 g(Np / 64, B);
  if (dtype == DT_F16)
    pw_pool_kernel<F16, 4><<<g, 256, 0, s>>>((const _Float16*)x, (const _Float16*)wt, bias, pooled, HW, K, Kp, N);
  else
    pw_pool_kernel<BF16, 4><<<g, 256, 0, s>>>((const __bf16*)x, (const __bf16*)wt, bias, pooled, HW, K, Kp, N);
  return hipGetLastError();
}

hipError_t launch_to_f32(int dtype, const void* x, float* y, int64_t n, hipStream_t s) {
  if (dtype == DT_F32 || dtype == DT_X2) return hipMemcpyAsync(y, x, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, s);
  const unsigned g = blocks_for(n, 256);
  if (dtype == DT_F16)
    to_f32_kernel<F16><<<g, 256, 0, s>>>((const _Float16*)x, y, n);
  else
    to_f32_kernel<BF16><<<g, 256, 0, s>>>((const __bf16*)x, y, n);
  return hipGetLastError();
}

}  // namespace spef
