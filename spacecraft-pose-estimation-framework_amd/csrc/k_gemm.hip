// LDS-tiled MFMA GEMM for 1x1 convolutions (pytorch_layers.py:78-86 expand / project, :35-62 last conv):
//   Y[m][n] = epi( sum_k X[m][k] W[n][k] + b[n] ) (+ R[m][n])     X, Y, R: NHWC activations (rows = pixels)
// Output-transposed MFMA form (C^T = W X^T): channels on the MFMA row axis, pixels on the column axis, so
// each lane stores 4 consecutive channels of one pixel. Workgroup = 4 waves as WN (channel) x WM (pixel);
// wave tile = NT x MT 16x16 MFMA tiles; block tile BN = 16*WN*NT channels x BM = 16*WM*MT pixels.
// K advances 32 per step through a double-buffered LDS pair (register-staged global loads of step k+1 are
// issued before the MFMAs of step k; one barrier per step). Rows padded by 16 B (ds_read_b128 conflicts).
#include "spef_common.hpp"
#include "spef_kernels.hpp"

namespace spef {

template <typename DT, int WN, int NT, int MT, int EPI>
__global__ __launch_bounds__(256) void gemm_pw_kernel(const typename DT::T* __restrict__ X,
                                                      const typename DT::T* __restrict__ Wt,
                                                      const float* __restrict__ bias,
                                                      const typename DT::T* __restrict__ R,
                                                      typename DT::T* __restrict__ Y, int64_t M, int K, int N,
                                                      int Kp, int Np, int n_chunks, uint32_t nwg) {
  using T = typename DT::T;
  using x8 = typename DT::x8;
  using x4 = typename DT::x4;
  constexpr int WM = 4 / WN;
  constexpr int BN = 16 * WN * NT, BM = 16 * WM * MT;
  constexpr int RS = 48;                                   // LDS row stride: 96 B = 6 granules, conflict-free
  constexpr int XP = (BM * 4 + 255) / 256, WP = (BN * 4 + 255) / 256;   // 16-B pieces per thread
  __shared__ __attribute__((aligned(16))) T As[2][BN * RS];
  __shared__ __attribute__((aligned(16))) T Bs[2][BM * RS];

  const uint32_t L = xcd_remap(blockIdx.x, nwg);
  const int chunk = (int)(L % (uint32_t)n_chunks);
  const int64_t mt0 = (int64_t)(L / (uint32_t)n_chunks) * BM;
  const int n0 = chunk * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  const int wn = wave % WN, wm = wave / WN;

  x8 xr[XP], wr[WP];
  auto gload = [&](int ks) {
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int p = tid + 256 * i;
      const int row = p >> 2, g = p & 3;
      const int64_t m = mt0 + row;
      const int k = ks * 32 + 8 * g;
      xr[i] = (p < BM * 4 && m < M && k < K) ? load8<DT>(X + (size_t)m * K + k) : zero8<DT>();
    }
#pragma unroll
    for (int i = 0; i < WP; ++i) {
      const int p = tid + 256 * i;
      const int row = p >> 2, g = p & 3;
      const int n = n0 + row;
      wr[i] = (p < BN * 4 && n < Np) ? load8<DT>(Wt + (size_t)n * Kp + ks * 32 + 8 * g) : zero8<DT>();
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int p = tid + 256 * i;
      if (p < BM * 4) *reinterpret_cast<x8*>(&Bs[buf][(p >> 2) * RS + 8 * (p & 3)]) = xr[i];
    }
#pragma unroll
    for (int i = 0; i < WP; ++i) {
      const int p = tid + 256 * i;
      if (p < BN * 4) *reinterpret_cast<x8*>(&As[buf][(p >> 2) * RS + 8 * (p & 3)]) = wr[i];
    }
  };

  f32x4 acc[NT][MT];   // accumulators start at the folded-BN bias (same order as the fused block kernel)
#pragma unroll
  for (int a = 0; a < NT; ++a) {
    const int i = n0 + (wn * NT + a) * 16 + 4 * kg;
    float4 bb = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < Np) bb = *reinterpret_cast<const float4*>(bias + i);
#pragma unroll
    for (int b = 0; b < MT; ++b) acc[a][b] = f32x4{bb.x, bb.y, bb.z, bb.w};
  }

  const int KS = Kp >> 5;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int ks = 0; ks < KS; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < KS) gload(ks + 1);
    x8 af[NT], bf[MT];
#pragma unroll
    for (int a = 0; a < NT; ++a)
      af[a] = *reinterpret_cast<const x8*>(&As[buf][((wn * NT + a) * 16 + r16) * RS + 8 * kg]);
#pragma unroll
    for (int b = 0; b < MT; ++b)
      bf[b] = *reinterpret_cast<const x8*>(&Bs[buf][((wm * MT + b) * 16 + r16) * RS + 8 * kg]);
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int b = 0; b < MT; ++b) acc[a][b] = DT::mfma(af[a], bf[b], acc[a][b]);
    if (ks + 1 < KS) {
      lstore(buf ^ 1);
      __syncthreads();
    }
  }

#pragma unroll
  for (int a = 0; a < NT; ++a) {
    const int i = n0 + (wn * NT + a) * 16 + 4 * kg;
    if (i >= N) continue;
#pragma unroll
    for (int b = 0; b < MT; ++b) {
      const int64_t m = mt0 + (wm * MT + b) * 16 + r16;
      if (m >= M) continue;
      f32x4 v = acc[a][b];
      if (EPI == EPI_RELU || EPI == EPI_RELU_F32) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.0f);
      }
      if constexpr (EPI == EPI_RELU_F32) {   // fp32 feature map (keypoint head / backbone export)
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(Y) + (size_t)m * N + i) = make_float4(v[0], v[1], v[2], v[3]);
        continue;
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

template <typename DT, int WN, int NT, int MT>
static hipError_t gemm_go(int epi, const void* x, const void* wt, const float* bias, const void* r, void* y,
                          int64_t M, int K, int N, hipStream_t s) {
  using T = typename DT::T;
  constexpr int WM = 4 / WN;
  constexpr int BN = 16 * WN * NT, BM = 16 * WM * MT;
  const int Kp = (K + 31) & ~31, Np = (N + 15) & ~15;
  const int n_chunks = (Np + BN - 1) / BN;
  const int64_t nwg64 = (M + BM - 1) / BM * n_chunks;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  const T* X = (const T*)x;
  const T* W = (const T*)wt;
  if (epi == EPI_RELU)
    gemm_pw_kernel<DT, WN, NT, MT, EPI_RELU><<<nwg, 256, 0, s>>>(X, W, bias, nullptr, (T*)y, M, K, N, Kp, Np,
                                                                  n_chunks, nwg);
  else if (epi == EPI_RELU_F32)
    gemm_pw_kernel<DT, WN, NT, MT, EPI_RELU_F32><<<nwg, 256, 0, s>>>(X, W, bias, nullptr, (T*)y, M, K, N, Kp, Np,
                                                                      n_chunks, nwg);
  else if (epi == EPI_RES)
    gemm_pw_kernel<DT, WN, NT, MT, EPI_RES><<<nwg, 256, 0, s>>>(X, W, bias, (const T*)r, (T*)y, M, K, N, Kp, Np,
                                                                 n_chunks, nwg);
  else
    gemm_pw_kernel<DT, WN, NT, MT, EPI_NONE><<<nwg, 256, 0, s>>>(X, W, bias, nullptr, (T*)y, M, K, N, Kp, Np,
                                                                  n_chunks, nwg);
  return hipGetLastError();
}

// Block tile by output width: channel tile BN covers N (or an even split of it), pixel tile BM 64..128.
template <typename DT>
static hipError_t gemm_dispatch(int epi, const void* x, const void* wt, const float* bias, const void* r, void* y,
                                int64_t M, int K, int N, hipStream_t s) {
  const int n16 = ((N + 15) & ~15) / 16;
  switch (n16) {
    case 1: return gemm_go<DT, 1, 1, 2>(epi, x, wt, bias, r, y, M, K, N, s);     // BN 16,  BM 128
    case 2: return gemm_go<DT, 2, 1, 4>(epi, x, wt, bias, r, y, M, K, N, s);     // BN 32,  BM 128
    case 4: return gemm_go<DT, 2, 2, 4>(epi, x, wt, bias, r, y, M, K, N, s);     // BN 64,  BM 128
    case 6: return gemm_go<DT, 2, 3, 4>(epi, x, wt, bias, r, y, M, K, N, s);     // BN 96,  BM 128
    case 9: return gemm_go<DT, 1, 9, 1>(epi, x, wt, bias, r, y, M, K, N, s);     // BN 144, BM 64
    case 10: return gemm_go<DT, 2, 5, 2>(epi, x, wt, bias, r, y, M, K, N, s);    // BN 160, BM 64
    default: break;
  }
  if (n16 % 12 == 0) return gemm_go<DT, 2, 6, 2>(epi, x, wt, bias, r, y, M, K, N, s);   // BN 192, BM 64
  if (n16 % 10 == 0) return gemm_go<DT, 2, 5, 2>(epi, x, wt, bias, r, y, M, K, N, s);   // BN 160, BM 64
  if (n16 % 8 == 0) return gemm_go<DT, 2, 4, 4>(epi, x, wt, bias, r, y, M, K, N, s);    // BN 128, BM 128
  if (n16 % 4 == 0) return gemm_go<DT, 2, 2, 4>(epi, x, wt, bias, r, y, M, K, N, s);
  if (n16 % 2 == 0) return gemm_go<DT, 2, 1, 4>(epi, x, wt, bias, r, y, M, K, N, s);
  return gemm_go<DT, 1, 1, 2>(epi, x, wt, bias, r, y, M, K, N, s);
}

const char* gemm_key(int dtype, int epi, int N) {
  static thread_local char buf[64];
  const int n16 = ((N + 15) & ~15) / 16;
  int wn = 1, nt = 1, mt = 2;
  switch (n16) {
    case 1: wn = 1; nt = 1; mt = 2; break;
    case 2: wn = 2; nt = 1; mt = 4; break;
    case 4: wn = 2; nt = 2; mt = 4; break;
    case 6: wn = 2; nt = 3; mt = 4; break;
    case 9: wn = 1; nt = 9; mt = 1; break;
    case 10: wn = 2; nt = 5; mt = 2; break;
    default:
      if (n16 % 12 == 0) { wn = 2; nt = 6; mt = 2; }
      else if (n16 % 10 == 0) { wn = 2; nt = 5; mt = 2; }
      else if (n16 % 8 == 0) { wn = 2; nt = 4; mt = 4; }
      else if (n16 % 4 == 0) { wn = 2; nt = 2; mt = 4; }
      else if (n16 % 2 == 0) { wn = 2; nt = 1; mt = 4; }
  }
  snprintf(buf, sizeof(buf), "gemm_pw_kernel<%s,%d,%d,%d,%d>", dtype == DT_F16 ? "F16" : "BF16", wn, nt, mt, epi);
  return buf;
}

hipError_t launch_gemm_pw(int dtype, int epi, const void* x, const void* wt, const float* bias, const void* r,
                          void* y, int64_t M, int K, int N, hipStream_t s) {
  if (M <= 0) return hipSuccess;
  if ((K & 7) || (N & 3)) return hipErrorInvalidValue;
  return dtype == DT_F16 ? gemm_dispatch<F16>(epi, x, wt, bias, r, y, M, K, N, s)
                         : gemm_dispatch<BF16>(epi, x, wt, bias, r, y, M, K, N, s);
}

}  // namespace spef
