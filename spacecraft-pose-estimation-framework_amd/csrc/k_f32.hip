// Float32 schedule of the backbone (blob dtype 4): the reference's own arithmetic type end to end, for the
// parity-first variants -- the keypoint head, whose unpooled 122,880-wide Linear (head/keypoints.py:20-27) does
// not average fp16 storage rounding away, and the C2 feature comparison.
//
//   gemm_f32_kernel  1x1 ConvBnAct / projection (+ residual add) on the exact fp32 MFMA v_mfma_f32_16x16x4_f32:
//                    products are exact fp32, accumulation fp32, activations fp32 NHWC (pytorch_layers.py:78-96)
//   mean_hw_kernel   URSONetHead's x.mean([2,3]) (ursonet.py:30) over an fp32 NHWC map
// Stem and depthwise run the k_conv.hip kernels instantiated for fp32 storage.
#include "spef_common.hpp"
#include "spef_kernels.hpp"

namespace spef {

// C^T[n][m] = sum_k W[n][k] X[m][k] with channels on the MFMA row axis (A = weights) and pixels on the column
// axis (B = activations), as pw_kernel. 16x16x4 lane map: A[i = l&15][k = l>>4], B[k = l>>4][j = l&15],
// D[i = 4(l>>4)+r][j = l&15]. Each lane loads 4 consecutive k of its row (16 B) for a K step of 16 and feeds them to
// four MFMAs, MFMA s taking element s: lane group g then contributes k = 4g + s, a permutation of the 16 k applied
// identically to A and B. A wave owns NT channel tiles x MT pixel tiles; 4 waves per workgroup on 64*MT pixels.
template <int NT, int MT, int EPI>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ X, const float* __restrict__ Wt,
                                                       const float* __restrict__ bias, const float* __restrict__ R,
                                                       float* __restrict__ Y, int64_t M, int K, int N, int Kp,
                                                       int n_chunks, uint32_t nwg) {
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
  const float* wp = Wt + (size_t)(n0 + r16) * Kp + 4 * kg;
  const float* xp[MT];
  bool mv[MT];
#pragma unroll
  for (int b = 0; b < MT; ++b) {
    const int64_t m = m0 + 16 * b + r16;
    mv[b] = m < M;
    xp[b] = X + (size_t)(mv[b] ? m : 0) * K + 4 * kg;
  }
  const int KS = (K + 15) >> 4;   // weights are zero-padded to Kp >= 16 * KS; activations masked past K
  for (int ks = 0; ks < KS; ++ks) {
    const bool kv = (ks * 16 + 4 * kg) < K;   // K % 4 == 0: a lane's 4 k are all in range or all out
    float4 av[NT], bv[MT];
#pragma unroll
    for (int a = 0; a < NT; ++a) av[a] = *reinterpret_cast<const float4*>(wp + (size_t)a * 16 * Kp + ks * 16);
#pragma unroll
    for (int b = 0; b < MT; ++b)
      bv[b] = (kv && mv[b]) ? *reinterpret_cast<const float4*>(xp[b] + ks * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int b = 0; b < MT; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[a].x, bv[b].x, acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[a].y, bv[b].y, acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[a].z, bv[b].z, acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[a].w, bv[b].w, acc[a][b], 0, 0, 0);
      }
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
      if (EPI == EPI_RELU || EPI == EPI_RELU_F32) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.0f);
      }
      if (EPI == EPI_RES) {   // x + conv(x) (pytorch_layers.py:93-96): the residual added after the BN bias
        const float4 rr = *reinterpret_cast<const float4*>(R + (size_t)m * N + i);
        v[0] += rr.x; v[1] += rr.y; v[2] += rr.z; v[3] += rr.w;
      }
      *reinterpret_cast<float4*>(Y + (size_t)m * N + i) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

template <int NT, int MT>
static hipError_t gemm_f32_go(int epi, const float* x, const float* wt, const float* bias, const float* r, float* y,
                              int64_t M, int K, int N, hipStream_t s) {
  const int Kp = (K + 31) & ~31, Np = (N + 15) & ~15;
  const int n_chunks = Np / (16 * NT);
  const int64_t nwg64 = (M + 64 * MT - 1) / (64 * MT) * n_chunks;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  if (epi == EPI_RELU || epi == EPI_RELU_F32)
    gemm_f32_kernel<NT, MT, EPI_RELU><<<nwg, 256, 0, s>>>(x, wt, bias, nullptr, y, M, K, N, Kp, n_chunks, nwg);
  else if (epi == EPI_RES)
    gemm_f32_kernel<NT, MT, EPI_RES><<<nwg, 256, 0, s>>>(x, wt, bias, r, y, M, K, N, Kp, n_chunks, nwg);
  else
    gemm_f32_kernel<NT, MT, EPI_NONE><<<nwg, 256, 0, s>>>(x, wt, bias, nullptr, y, M, K, N, Kp, n_chunks, nwg);
  return hipGetLastError();
}

const char* gemm_f32_key(int N) {
  const int n16 = ((N + 15) & ~15) / 16;
  if (n16 == 1) return "gemm_f32_kernel<1,4>";
  if (n16 == 2) return "gemm_f32_kernel<2,4>";
  if (n16 % 4 == 0) return "gemm_f32_kernel<4,4>";
  if (n16 % 5 == 0) return "gemm_f32_kernel<5,2>";
  if (n16 % 6 == 0) return "gemm_f32_kernel<6,2>";
  if (n16 % 3 == 0) return "gemm_f32_kernel<3,4>";
  if (n16 % 2 == 0) return "gemm_f32_kernel<2,4>";
  return "gemm_f32_kernel<1,4>";
}

hipError_t launch_gemm_f32(int epi, const void* x, const void* wt, const float* bias, const void* r, void* y,
                           int64_t M, int K, int N, hipStream_t s) {
  if (M <= 0) return hipSuccess;
  if ((K & 3) || (N & 3)) return hipErrorInvalidValue;
  const float *X = (const float*)x, *W = (const float*)wt, *Rr = (const float*)r;
  float* Y = (float*)y;
  const int n16 = ((N + 15) & ~15) / 16;
  if (n16 == 1) return gemm_f32_go<1, 4>(epi, X, W, bias, Rr, Y, M, K, N, s);
  if (n16 == 2) return gemm_f32_go<2, 4>(epi, X, W, bias, Rr, Y, M, K, N, s);
  if (n16 % 4 == 0) return gemm_f32_go<4, 4>(epi, X, W, bias, Rr, Y, M, K, N, s);
  if (n16 % 5 == 0) return gemm_f32_go<5, 2>(epi, X, W, bias, Rr, Y, M, K, N, s);
  if (n16 % 6 == 0) return gemm_f32_go<6, 2>(epi, X, W, bias, Rr, Y, M, K, N, s);
  if (n16 % 3 == 0) return gemm_f32_go<3, 4>(epi, X, W, bias, Rr, Y, M, K, N, s);
  if (n16 % 2 == 0) return gemm_f32_go<2, 4>(epi, X, W, bias, Rr, Y, M, K, N, s);
  return gemm_f32_go<1, 4>(epi, X, W, bias, Rr, Y, M, K, N, s);
}

// pooled[b][c] = (sum over the HW pixels of x[b][p][c], in pixel order) / HW; one thread per (image, channel),
// consecutive threads on consecutive channels (coalesced NHWC rows).
__global__ __launch_bounds__(256) void mean_hw_kernel(const float* __restrict__ x, float* __restrict__ pooled, int B,
                                                      int HW, int C) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)B * C) return;
  const int b = (int)(i / C), c = (int)(i % C);
  const float* p = x + (size_t)b * HW * C + c;
  float s = 0.f;
  for (int j = 0; j < HW; ++j) s += p[(size_t)j * C];
  pooled[i] = s / (float)HW;
}

hipError_t launch_mean_hw(const float* x, float* pooled, int B, int HW, int C, hipStream_t s) {
  const int64_t n = (int64_t)B * C;
  mean_hw_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(x, pooled, B, HW, C);
  return hipGetLastError();
}

}  // namespace spef
