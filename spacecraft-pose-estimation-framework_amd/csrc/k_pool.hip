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

// K = 32 * KSC fixed (URSONet: 320): each wave keeps its 32 output channels' weights for the whole K in registers
// (2 channel tiles x KSC fragments, loaded once), so the only LDS traffic is the pixel map, staged 64 pixels x K at a
// time with one barrier pair per chunk instead of one per 32-wide K step (the kernel above is bound by that per-step
// round trip). Every wave covers all pixels of its image for its channels: the mean needs no cross-wave reduction.
// Workgroup = 4 waves = 128 channels of one image; the next chunk's pixels are loaded into registers during the
// current chunk's MFMAs; full chunks skip the pixel masks; ReLU sums use packed adds. Measured (tools/ab.py, B=64,
// 512²): 31.3 -> 25.9 us per launch with 64-pixel chunks, whose 252 VGPRs (2 waves per SIMD) made the 640
// workgroups 1.25 rounds of the 512 slots; 32-pixel chunks (the same per-lane summation order) fit 168 VGPRs, 3 waves
// per SIMD, all 640 workgroups in one round of 768 slots: -1.7 us (A/B).
template <typename DT, int KSC, int PC = 32>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void pool_gemm_rk_kernel(const typename DT::T* __restrict__ X,
                                                           const typename DT::T* __restrict__ Wt,
                                                           const float* __restrict__ bias, float* __restrict__ pooled,
                                                           int HW, int N) {
  using T = typename DT::T;
  using x8 = typename DT::x8;
  constexpr int K = 32 * KSC;
  constexpr int NQ = PC / 16;                     // MFMA pixel tiles per chunk
  constexpr int RS = K + 16;                      // LDS row stride: K*2 + 32 B = 2 mod 4 granules, conflict-free b128
  static_assert(((RS * 2 / 16) & 3) == 2, "row stride");
  constexpr int GPR = K / 8;                      // 16-B pieces per pixel row
  constexpr int NP = PC * GPR / 256;              // pieces per thread per chunk
  static_assert(PC * GPR % 256 == 0, "chunk split");
  __shared__ __attribute__((aligned(16))) T Bs[PC * RS];

  const uint32_t nblk = gridDim.x * gridDim.y;
  const uint32_t L = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, nblk);   // an image's channel blocks on one XCD
  const int b = (int)(L / gridDim.x), n0 = (int)(L % gridDim.x) * 128;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  const int c0 = n0 + 32 * wave;                  // this wave's 32 output channels
  const T* Xb = X + (size_t)b * HW * K;

  // the wave's weight fragments for all of K (A operand: row = output channel c0 + 16 t + r16)
  x8 wa[2][KSC];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ks = 0; ks < KSC; ++ks) wa[t][ks] = load8<DT>(Wt + (size_t)(c0 + 16 * t + r16) * K + 32 * ks + 8 * kg);
  float4 bb[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) bb[t] = *reinterpret_cast<const float4*>(bias + c0 + 16 * t + 4 * kg);

  const int nch = (HW + PC - 1) / PC;
  // this thread's 16-B pieces of a chunk: pixel row and granule are chunk-invariant (computed once)
  int prow[NP], pofs[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int p = tid + 256 * i, row = p / GPR;
    prow[i] = row;
    pofs[i] = row * RS + 8 * (p - row * GPR);
  }
  x8 xr[NP];
  auto gload = [&](int ch) {   // branch-free: pixels past HW read pixel 0 and are zeroed at the store
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int px = ch * PC + prow[i];
      xr[i] = load8<DT>(Xb + (size_t)(px < HW ? px : 0) * K + (pofs[i] - prow[i] * RS));
    }
  };
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  f32x2 sum[2][2] = {};   // [channel tile][channel pair]: packed adds
  gload(0);
#pragma unroll 1
  for (int ch = 0; ch < nch; ++ch) {
    const bool full = (ch + 1) * PC <= HW;   // workgroup-uniform: masks only in a partial last chunk
    if (ch > 0) __syncthreads();   // every wave's reads of the previous chunk are done
    if (full) {
#pragma unroll
      for (int i = 0; i < NP; ++i) *reinterpret_cast<x8*>(&Bs[pofs[i]]) = xr[i];
    } else {
#pragma unroll
      for (int i = 0; i < NP; ++i)
        *reinterpret_cast<x8*>(&Bs[pofs[i]]) = ch * PC + prow[i] < HW ? xr[i] : zero8<DT>();
    }
    __syncthreads();
    if (ch + 1 < nch) gload(ch + 1);   // in flight across this chunk's MFMAs
    f32x4 acc[2][NQ];
#pragma unroll
    for (int ks = 0; ks < KSC; ++ks) {
      x8 bf[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) bf[q] = *reinterpret_cast<const x8*>(&Bs[(q * 16 + r16) * RS + 32 * ks + 8 * kg]);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int q = 0; q < NQ; ++q)   // bias as the first MFMA's C operand
          acc[t][q] = DT::mfma(wa[t][ks], bf[q], ks == 0 ? f32x4{bb[t].x, bb[t].y, bb[t].z, bb[t].w} : acc[t][q]);
    }
    if (full) {
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int e = 0; e < 2; ++e)
            sum[t][e] += f32x2{fmaxf(acc[t][q][2 * e], 0.f), fmaxf(acc[t][q][2 * e + 1], 0.f)};
    } else {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const float pv = ch * PC + q * 16 + r16 < HW ? 1.f : 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int e = 0; e < 2; ++e)
            sum[t][e] += f32x2{fmaxf(acc[t][q][2 * e], 0.f), fmaxf(acc[t][q][2 * e + 1], 0.f)} * pv;
      }
    }
  }
  // reduce over the 16 pixel lanes; lane r16 == 0 of each channel group writes its 4 channels' means
  float red[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = sum[t][e >> 1][e & 1];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      red[t][e] = v;
    }
  if (r16 == 0) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int c = c0 + 16 * t + 4 * kg;
      float4 o = make_float4(red[t][0] / (float)HW, red[t][1] / (float)HW, red[t][2] / (float)HW,
                             red[t][3] / (float)HW);
      if (c + 3 < N) *reinterpret_cast<float4*>(pooled + (size_t)b * N + c) = o;
      else
        for (int e = 0; e < 4; ++e)
          if (c + e < N) pooled[(size_t)b * N + c + e] = (&o.x)[e];
    }
  }
}

hipError_t launch_pool_gemm(int dtype, const void* x, const void* wt, const float* bias, float* pooled, int B, int HW,
                            int K, int N, hipStream_t s) {
  const int Kp = (K + 31) & ~31, Np = (N + 15) & ~15;
  if ((K & 7) || (Np % 128)) return hipErrorInvalidValue;
  dim3 g(Np / 128, B);
  if (K == 320) {   // the URSONet last conv: register-resident weights, one barrier pair per 64-pixel chunk
    if (dtype == DT_F16)
      pool_gemm_rk_kernel<F16, 10><<<g, 256, 0, s>>>((const _Float16*)x, (const _Float16*)wt, bias, pooled, HW, N);
    else
      pool_gemm_rk_kernel<BF16, 10><<<g, 256, 0, s>>>((const __bf16*)x, (const __bf16*)wt, bias, pooled, HW, N);
    return hipGetLastError();
  }
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
