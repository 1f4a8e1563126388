// Last ConvBnAct 320->1280 1x1 + ReLU (mobilenet_v2.py:264) fused with URSONetHead's x.mean([2,3])
// (src/modeling/head/ursonet.py:30) as one LDS-tiled MFMA GEMM whose epilogue reduces over pixels.
//
// Workgroup = 8 waves (2 channel x 4 pixel) on one image x 128 output channels; pixel chunks of 256 are
// looped inside the workgroup (any H*W), K = 320 advances 32 per double-buffered LDS step. ReLU(conv + b) is
// summed in fp32 registers over the wave's pixel tiles, then over the 16 pixel lanes by shuffles and over the
// 4 pixel waves through LDS: the 1280-channel map never exists in memory and the mean is deterministic.
#include "spef_common.hpp"
#include <type_traits>
#include "spef_kernels.hpp"

// Pixel tile of the K = 320 instantiation: MT 16-pixel tiles per wave, NWM pixel waves (2 channel waves each).
// Measured at B = 64 (tools/ab.py): (MT, NWM) = (4, 4) 33.1 us, (2, 4) 30.9, (2, 2) 31.7-32.2 -- the kernel is bound
// by its per-K-step LDS round trip and barrier, not by occupancy (1, 2 or 3 workgroups per CU).
#ifndef SPEF_POOL_MT
#define SPEF_POOL_MT 2
#endif
#ifndef SPEF_POOL_NWM
#define SPEF_POOL_NWM 4
#endif

namespace spef {

// KSC > 0: the K step count is a compile-time constant (K = 32 * KSC, the URSONet last conv has K = 320) and the K loop
// is fully unrolled, which lets the compiler track the two register stages' outstanding loads exactly.
template <typename DT, int KSC, int MT = 4, int NWM = 4>
__global__ __launch_bounds__(2 * NWM * 64) void pool_gemm_kernel(const typename DT::T* __restrict__ X,
                                                        const typename DT::T* __restrict__ Wt,
                                                        const float* __restrict__ bias, float* __restrict__ pooled,
                                                        int HW, int K, int Kp, int N) {
  using T = typename DT::T;
  using x8 = typename DT::x8;
  constexpr int NT = 4;                         // wave tile: 64 channels x 16 MT pixels
  constexpr int NTHR = 2 * NWM * 64;            // 2 channel waves x NWM pixel waves
  constexpr int BN = 2 * 16 * NT, BM = NWM * 16 * MT;
  constexpr int RS = 48;                        // LDS row stride (96 B: conflict-free b128)
  constexpr int XP = (BM * 4 + NTHR - 1) / NTHR, WP = (BN * 4 + NTHR - 1) / NTHR; // 16-B pieces per thread per K step
  __shared__ __attribute__((aligned(16))) T As[2][BN * RS];
  __shared__ __attribute__((aligned(16))) T Bs[2][BM * RS];
  __shared__ float red[NWM][BN];

  // XCD-aware order: the channel blocks of one image run on one XCD, so its 320-channel map is fetched from
  // HBM once into that XCD's L2 instead of once per XCD (blocks are dealt round-robin over the 8 XCDs).
  const uint32_t nblk = gridDim.x * gridDim.y;
  const uint32_t L = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, nblk);
  const int b = (int)(L / gridDim.x), n0 = (int)(L % gridDim.x) * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  const int wn = wave & 1, wm = wave >> 1;
  const T* Xb = X + (size_t)b * HW * K;
  const int KS = KSC > 0 ? KSC : Kp >> 5;

  f32x4 sum[NT];
#pragma unroll
  for (int a = 0; a < NT; ++a) sum[a] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Two register stages of global fragments: step ks stores the fragments loaded during step ks-1 and loads
  // those of step ks+2, so each load has two K steps of MFMAs and barriers to land in (one step was not enough to
  // cover the L2/HBM latency). Loads are branch-free (out-of-range rows read row 0 and are zeroed at the LDS store):
  // a load inside a divergent branch is waited for at the branch join.
  x8 xr[2][XP], wr[2][WP];
  for (int m0 = 0; m0 < HW; m0 += BM) {
    auto xok = [&](int i, int ks) {
      const int p = tid + NTHR * i, row = p >> 2, g = p & 3;
      return row < BM && m0 + row < HW && ks * 32 + 8 * g < K;
    };
    auto gload = [&](int ks, auto stc) {
      constexpr int st = decltype(stc)::value;
#pragma unroll
      for (int i = 0; i < XP; ++i) {
        const int p = tid + NTHR * i, row = p >> 2, g = p & 3, k = ks * 32 + 8 * g;
        xr[st][i] = load8<DT>(Xb + (xok(i, ks) ? (size_t)(m0 + row) * K + k : 0));
      }
#pragma unroll
      for (int i = 0; i < WP; ++i) {
        const int p = tid + NTHR * i, row = (p >> 2) < BN ? p >> 2 : 0, g = p & 3;
        wr[st][i] = load8<DT>(Wt + (size_t)(n0 + row) * Kp + ks * 32 + 8 * g);
      }
    };
    auto lstore = [&](int buf, int ks, auto stc) {
      constexpr int st = decltype(stc)::value;
#pragma unroll
      for (int i = 0; i < XP; ++i) {
        const int p = tid + NTHR * i;
        if (BM * 4 % NTHR == 0 || (p >> 2) < BM)
          *reinterpret_cast<x8*>(&Bs[buf][(p >> 2) * RS + 8 * (p & 3)]) = xok(i, ks) ? xr[st][i] : zero8<DT>();
      }
#pragma unroll
      for (int i = 0; i < WP; ++i) {
        const int p = tid + NTHR * i;
        if (BN * 4 % NTHR == 0 || (p >> 2) < BN)
          *reinterpret_cast<x8*>(&As[buf][(p >> 2) * RS + 8 * (p & 3)]) = wr[st][i];
      }
    };
    f32x4 acc[NT][MT];   // bias as the MFMA C operand (re-read per pixel chunk: no registers held across chunks)
    {
      const float* bt = bias;
      asm volatile("" : "+s"(bt));
#pragma unroll
      for (int a = 0; a < NT; ++a) {
        const float4 t = *reinterpret_cast<const float4*>(bt + n0 + (wn * NT + a) * 16 + 4 * kg);
#pragma unroll
        for (int q = 0; q < MT; ++q) acc[a][q] = f32x4{t.x, t.y, t.z, t.w};
      }
    }
    __syncthreads();   // previous chunk's LDS reads done
    gload(0, std::integral_constant<int, 0>());
    if (KS > 1) gload(1, std::integral_constant<int, 1>());
    lstore(0, 0, std::integral_constant<int, 0>());
    __syncthreads();
    // K step ks uses LDS buffer and register stage ks & 1; the loop is unrolled by two so both are compile-time
    auto step = [&](int ks, auto par) {
      constexpr int P = decltype(par)::value;
      // stage P was stored to LDS at the end of step ks - 1. Issued unconditionally (the last two steps reload a
      // valid step that is never stored) so the count of outstanding loads is the same on every path and the
      // compiler's wait before the store below covers only the older stage.
      gload(ks + 2 < KS ? ks + 2 : KS - 1, std::integral_constant<int, P>());
      x8 af[NT], bf[MT];
#pragma unroll
      for (int a = 0; a < NT; ++a)
        af[a] = *reinterpret_cast<const x8*>(&As[P][((wn * NT + a) * 16 + r16) * RS + 8 * kg]);
#pragma unroll
      for (int q = 0; q < MT; ++q)
        bf[q] = *reinterpret_cast<const x8*>(&Bs[P][((wm * MT + q) * 16 + r16) * RS + 8 * kg]);
#pragma unroll
      for (int a = 0; a < NT; ++a)
#pragma unroll
        for (int q = 0; q < MT; ++q) acc[a][q] = DT::mfma(af[a], bf[q], acc[a][q]);
      if (ks + 1 < KS) {
        lstore(P ^ 1, ks + 1, std::integral_constant<int, P ^ 1>());
        __syncthreads();
      }
    };
#pragma unroll
    for (int ks = 0; ks < KS; ks += 2) {
      step(ks, std::integral_constant<int, 0>());
      if (ks + 1 < KS) step(ks + 1, std::integral_constant<int, 1>());
    }
#pragma unroll
    for (int q = 0; q < MT; ++q) {
      const bool pv = m0 + (wm * MT + q) * 16 + r16 < HW;
#pragma unroll
      for (int a = 0; a < NT; ++a)
#pragma unroll
        for (int e = 0; e < 4; ++e) sum[a][e] += pv ? fmaxf(acc[a][q][e], 0.f) : 0.f;
    }
  }
  // reduce over the 16 pixel lanes, then over the NWM pixel waves
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = sum[a][e];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      if (r16 == 0) red[wm][(wn * NT + a) * 16 + 4 * kg + e] = v;
    }
  __syncthreads();
  if (tid < BN && n0 + tid < N) {
    float v;
    if constexpr (NWM == 4) v = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
    else v = red[0][tid] + red[1][tid];
    pooled[(size_t)b * N + n0 + tid] = v / (float)HW;
  }
}

hipError_t launch_pool_gemm(int dtype, const void* x, const void* wt, const float* bias, float* pooled, int B, int HW,
                            int K, int N, hipStream_t s) {
  const int Kp = (K + 31) & ~31, Np = (N + 15) & ~15;
  if ((K & 7) || (Np % 128)) return hipErrorInvalidValue;
  dim3 g(Np / 128, B);
  if (dtype == DT_F16) {
    if (Kp == 320)
      pool_gemm_kernel<F16, 10, SPEF_POOL_MT, SPEF_POOL_NWM><<<g, 2 * SPEF_POOL_NWM * 64, 0, s>>>((const _Float16*)x, (const _Float16*)wt, bias, pooled, HW, K, Kp, N);
    else
      pool_gemm_kernel<F16, 0><<<g, 512, 0, s>>>((const _Float16*)x, (const _Float16*)wt, bias, pooled, HW, K, Kp, N);
  } else {
    pool_gemm_kernel<BF16, 0><<<g, 512, 0, s>>>((const __bf16*)x, (const __bf16*)wt, bias, pooled, HW, K, Kp, N);
  }
  return hipGetLastError();
}

}  // namespace spef
