// Three-stage pipelined fused InvertedResidual block (src/modeling/common/pytorch_layers.py:65-98) for the
// low-resolution MobileNet-V2 blocks 14-17 (16x16 output maps, 576-960 hidden channels).
//
// One workgroup per output tile. Its waves take two roles and pipeline the 32-channel hidden chunks in three stages
// with one barrier per chunk:
//
//   MFMA waves  [0, NM):      E(i+1)  expand chunk i+1: relu(x We^T + be) on MFMA        -> LDS slab Es[(i+1) & 1]
//                             P(i-1)  project chunk i-1 from Ds[(i-1) & 1] on MFMA      -> fp32 accumulators
//   VALU waves  [NM, NM+NV):  V(i)    3x3 depthwise (+BN, ReLU) of chunk i from Es[i & 1] -> LDS slab Ds[i & 1]
//
// so the matrix pipe of every SIMD is fed only by the MFMA waves and its vector pipe only by the depthwise waves.
// The MFMA waves are the critical role. They split the expand by hidden half and pixel tile (each wave streams half of
// a chunk's expand weights from L2, one step ahead) and keep their expand B fragments (input pixels, the same for
// every chunk) in registers; they split the project by output-channel tile (each wave streams only its own project
// weights). (The wave-specialised kernel, k_irw.hip, has the depthwise waves also issue the project MFMAs at the end
// of their dependent VALU chain and computes the depthwise twice when the project is split over output-channel
// groups.) Measured dead end: staging the weight chunks in LDS through the depthwise waves (their loop-carried
// staging registers went to scratch; 30 -> 61 us on blocks 15-16).
//
// Arithmetic and rounding are those of the slab kernel, the wave-specialised kernel and the unfused kernels: bias as
// the MFMA C input, fp16/bf16 after expand, fp32 depthwise in kx-outer/ky-inner tap order, fp16/bf16 after the
// depthwise, fp32 project accumulation over chunks in order -> bit-identical to the one-kernel-per-conv schedule.
#include "spef_common.hpp"
#include "spef_kernels.hpp"

namespace spef {

#ifndef SPEF_IRP_EARLY
#define SPEF_IRP_EARLY 1
#endif

template <int CIN, int HID, int COUT, int S, int TH, int TW, int NM, int NV, int DWB>
struct IrpGeom {
  static constexpr int NW = NM + NV;
  static constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3;
  static constexpr int PIN = IH * IW, PIN16 = (PIN + 15) / 16, PINP = PIN16 * 16;
  static constexpr int KS = CIN / 32;                  // expand K steps (CIN % 32 == 0 on every block here)
  static constexpr int ES = 48;                        // hidden slab row: 32 ch + pad, 6 granules (conflict-free b128)
  static constexpr int DS = 48;                        // depthwise-output slab row, same layout
  static constexpr int NCH = HID / 32;
  static constexpr int NCT = COUT / 16;
  static constexpr int POUT = TH * TW, POUT16 = POUT / 16;
  static constexpr int NG = NM / 2;                    // expand pixel-tile groups (MFMA waves pair up on hidden halves)
  static constexpr int EPT = (PIN16 + NG - 1) / NG;    // expand pixel tiles per MFMA wave
  static constexpr int NCTW = (NCT + NM - 1) / NM;     // project output-channel tiles per MFMA wave
  static constexpr int QPV = POUT16 / NV;              // depthwise pixel tiles per VALU wave
  static constexpr bool PAIR = S == 1 && TW == 16 && QPV % 2 == 0;   // vertically adjacent tiles share window rows
  static constexpr int bytes_for(int xs) {
    return PINP * xs * 2 + 2 * PINP * ES * 2 + 2 * POUT * DS * 2 + 9 * HID * DWB + 2 * HID * 4;
  }
  static constexpr int XS = bytes_for(CIN + 16) <= 163840 ? CIN + 16 : CIN + 8;   // input row stride (halves)
  static constexpr int LDS_BYTES = bytes_for(XS);
  // expand B fragments resident in registers across chunks when they and the project accumulators take at most half
  // of the per-wave VGPR budget (512 per SIMD lane shared by the waves of a SIMD); otherwise re-read per step
  static constexpr int VGPR_LIMIT = 512 / ((NW + 3) / 4) > 256 ? 256 : 512 / ((NW + 3) / 4);
  static constexpr bool BXR = 4 * (EPT * KS + POUT16 * NCTW) <= VGPR_LIMIT / 2;
  static_assert(CIN % 32 == 0 && HID % 32 == 0 && COUT % 16 == 0, "channel counts");
  static_assert(NM % 2 == 0 && POUT % 16 == 0 && POUT16 % NV == 0, "wave split");
  static_assert(EPT <= 32, "validity mask is 32 bits");
  static_assert(LDS_BYTES <= 163840, "LDS budget");
  static_assert(2 * NCH + 12 <= SPEF_TRACE_SLOTS, "trace slots");
};

template <typename DT, int CIN, int HID, int COUT, int S, int TH, int TW, bool RES, int NM, int NV>
__global__ __launch_bounds__((NM + NV) * 64) __attribute__((amdgpu_waves_per_eu(1, (NM + NV + 3) / 4))) void irp_kernel(
    const typename DT::T* __restrict__ X, const typename DT::T* __restrict__ We, const float* __restrict__ be,
    const typename DT::DW* __restrict__ Wd, const float* __restrict__ bd, const typename DT::T* __restrict__ Wp,
    const float* __restrict__ bp, typename DT::T* __restrict__ Y, int H, int W, int OH, int OW, int tiles_x,
    int tiles_y, uint32_t nwg) {
  using DW = typename DT::DW;
  using G = IrpGeom<CIN, HID, COUT, S, TH, TW, NM, NV, (int)sizeof(DW)>;
  using T = typename DT::T;
  using x8 = typename DT::x8;
  using x4 = typename DT::x4;
  constexpr int NW = G::NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Xs = reinterpret_cast<T*>(smem);                          // [PINP][XS] input tile (+halo)
  T* Es0 = Xs + G::PINP * G::XS;                               // [2][PINP][ES] hidden chunk slabs
  T* Ds0 = Es0 + 2 * G::PINP * G::ES;                          // [2][POUT][DS] depthwise output slabs
  DW* Wds = reinterpret_cast<DW*>(Ds0 + 2 * G::POUT * G::DS);  // [9][HID] depthwise weights
  float* Be = reinterpret_cast<float*>(Wds + 9 * HID);         // [HID] expand bias
  float* Bd = Be + HID;                                        // [HID] depthwise bias

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  SPEF_TRACE(0);
  uint32_t L = xcd_remap(blockIdx.x, nwg);       // the tiles of one image on one XCD (shared L2 for halos)
  const int tx = (int)(L % (uint32_t)tiles_x);
  L /= (uint32_t)tiles_x;
  const int ty = (int)(L % (uint32_t)tiles_y);
  const int b = (int)(L / (uint32_t)tiles_y);
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;

  // ---- 1. input tile, depthwise weights and biases -> LDS (16-B pieces, all loads before the stores)
  {
    constexpr int GPR = CIN / 8;
    constexpr int NXP = G::PINP * GPR;
    constexpr int EPP = 16 / (int)sizeof(DW);
    constexpr int DPR = HID / EPP;                     // depthwise pieces per tap
    constexpr int NDP = 9 * DPR;
    constexpr int NBP = HID / 4;
    constexpr int NTOT = NXP + NDP + 2 * NBP;
    constexpr int NIT = (NTOT + NW * 64 - 1) / (NW * 64);
    const T* Xb = X + (size_t)b * H * W * CIN;
    uint4 v[NIT];
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      int u = tid + NW * 64 * i;
      const void* src = nullptr;
      if (u < NXP) {
        const int p = u / GPR, g = u - p * GPR;
        if (p < G::PIN) {
          const int py = p / G::IW, px = p - py * G::IW;
          const int iy = iy0 + py, ix = ix0 + px;
          if (iy >= 0 && iy < H && ix >= 0 && ix < W) src = Xb + SPEF_KB_XOFF(((size_t)iy * W + ix) * CIN + g * 8);
        }
      } else if ((u -= NXP) < NDP) {
        const int tap = u / DPR, g = u - tap * DPR;
        src = Wd + (size_t)tap * HID + g * EPP;
      } else if ((u -= NDP) < 2 * NBP) {
        const int which = u / NBP, g = u - which * NBP;
        src = (which ? bd : be) + 4 * g;
      }
      v[i] = src ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      int u = tid + NW * 64 * i;
      char* dst = nullptr;
      if (u < NXP) {
        const int p = u / GPR, g = u - p * GPR;
        dst = reinterpret_cast<char*>(Xs + p * G::XS + g * 8);
      } else if ((u -= NXP) < NDP) {
        const int tap = u / DPR, g = u - tap * DPR;
        dst = reinterpret_cast<char*>(Wds + tap * HID + g * EPP);
      } else if ((u -= NDP) < 2 * NBP) {
        const int which = u / NBP, g = u - which * NBP;
        dst = reinterpret_cast<char*>((which ? Bd : Be) + 4 * g);
      }
      if (dst) *reinterpret_cast<uint4*>(dst) = v[i];
    }
  }
  SPEF_TRACE(1);

  if (wave < NM) {
    // =============================================================================== MFMA waves
    const int hh = wave & 1;                               // expand: hidden half of the chunk (16 channels)
    const int eg = wave >> 1;                              // expand: pixel-tile group
    const bool interior = iy0 >= 0 && ix0 >= 0 && iy0 + G::IH <= H && ix0 + G::IW <= W;
    uint32_t pvmask = 0;                                   // in-image pixels among this wave's expand tiles
    if (!interior)
#pragma unroll
      for (int jj = 0; jj < G::EPT; ++jj) {
        const int p = (eg + G::NG * jj) * 16 + r16;
        if (p < G::PIN) {
          const int py = p / G::IW, px = p - py * G::IW;
          const int iy = iy0 + py, ix = ix0 + px;
          if (iy >= 0 && iy < H && ix >= 0 && ix < W) pvmask |= 1u << jj;
        }
      }
    // expand A fragments of one hidden half: rows 32c + 16hh + r16, k = 32ks + 8kg
    x8 ea[G::KS];
    auto load_ea = [&](int c) {   // from L2, one step ahead
#if defined(SPEF_KBENCH_IRW_NO_WLOAD) || defined(SPEF_KBENCH_IRW_NO_ELOAD)   // tools/kbench timing ablations (wrong
      if (c > 1) return;                                                        // results): no weight loads after chunk 1
#endif
#ifdef SPEF_KBENCH_IRW_FIXED_WLOAD   // timing ablation: every chunk loads chunk 0's fragments (L1/L2-hot addresses)
      const T* w0 = We + (size_t)(16 * hh + r16) * CIN + 8 * kg;
#else
      const T* w0 = We + (size_t)(32 * c + 16 * hh + r16) * CIN + 8 * kg;
#endif
#pragma unroll
      for (int ks = 0; ks < G::KS; ++ks) ea[ks] = c < G::NCH ? load8<DT>(w0 + 32 * ks) : zero8<DT>();
    };
    // project A fragments: output-channel tiles wave + NM*t, hidden k = 32c + 8kg
    x8 pa[G::NCTW];
    auto load_pa = [&](int c) {
#if defined(SPEF_KBENCH_IRW_NO_WLOAD) || defined(SPEF_KBENCH_IRW_NO_PLOAD)
      if (c > 1) return;
#endif
#ifdef SPEF_KBENCH_IRW_FIXED_WLOAD
      const int cw = 0;
#else
      const int cw = c;
#endif
#pragma unroll
      for (int t = 0; t < G::NCTW; ++t) {
        const int ct = wave + NM * t;
        pa[t] = (c < G::NCH && ct < G::NCT) ? load8<DT>(Wp + (size_t)(16 * ct + r16) * HID + 32 * cw + 8 * kg)
                                            : zero8<DT>();
      }
    };
    f32x4 acc[G::POUT16][G::NCTW];
#pragma unroll
    for (int t = 0; t < G::NCTW; ++t) {
      const int ct = wave + NM * t;
      float4 bb = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ct < G::NCT) bb = *reinterpret_cast<const float4*>(bp + 16 * ct + 4 * kg);
#pragma unroll
      for (int q = 0; q < G::POUT16; ++q) acc[q][t] = f32x4{bb.x, bb.y, bb.z, bb.w};
    }

    // One pipeline step: E(ce) (this wave's pixel tiles x its hidden half of chunk ce -> Es[ce & 1]) and/or P(cp)
    // (all output pixel tiles x this wave's output-channel tiles, from Ds[cp & 1]). Every LDS read of the step is
    // issued first, the expand MFMAs run interleaved over the pixel tiles (independent accumulators; per tile the
    // K steps stay in order), the project MFMAs fill the expand MFMAs' result latency before the expand epilogue.
    // this wave's expand B fragments (its input pixel tiles), the same for every chunk: read once and kept in
    // registers (BXR), or re-read from the staged input tile at every step
    x8 bx[G::EPT][G::KS];
    auto read_bx = [&]() {
#pragma unroll
      for (int jj = 0; jj < G::EPT; ++jj) {
        const int pt = eg + G::NG * jj;
        if (pt < G::PIN16)
#pragma unroll
          for (int ks = 0; ks < G::KS; ++ks)
            bx[jj][ks] = *reinterpret_cast<const x8*>(Xs + (pt * 16 + r16) * G::XS + 32 * ks + 8 * kg);
      }
    };
    // ld_e / ld_p >= 0: the next expand / project fragments (chunks ld_e / ld_p) are issued inside the step, right after
    // the MFMAs that read the current ones, so their L2 latency overlaps the rest of the step and the barrier wait
    // (issued after the step, only the barrier wait covered it; the MFMA waves are the critical role).
    auto step = [&](int ce, int cp, bool do_e, bool do_p, int ld_e, int ld_p) {
      x8 bq[G::POUT16];
      if (!G::BXR && do_e) read_bx();
      if (do_p) {
        const T* Dr = Ds0 + (cp & 1) * G::POUT * G::DS;
#pragma unroll
        for (int q = 0; q < G::POUT16; ++q) bq[q] = *reinterpret_cast<const x8*>(Dr + (q * 16 + r16) * G::DS + 8 * kg);
      }
      f32x4 e[G::EPT];
      if (do_e) {
        const float4 eb = *reinterpret_cast<const float4*>(Be + 32 * ce + 16 * hh + 4 * kg);
#pragma unroll
        for (int jj = 0; jj < G::EPT; ++jj) e[jj] = f32x4{eb.x, eb.y, eb.z, eb.w};   // bias as MFMA C
#pragma unroll
        for (int ks = 0; ks < G::KS; ++ks)
#pragma unroll
          for (int jj = 0; jj < G::EPT; ++jj)
            if (eg + G::NG * jj < G::PIN16) e[jj] = DT::mfma(ea[ks], bx[jj][ks], e[jj]);
      }
      if (SPEF_IRP_EARLY && ld_e >= 0) load_ea(ld_e);
      if (do_p) {
#pragma unroll
        for (int q = 0; q < G::POUT16; ++q)
#pragma unroll
          for (int t = 0; t < G::NCTW; ++t)
            if (wave + NM * t < G::NCT) acc[q][t] = DT::mfma(pa[t], bq[q], acc[q][t]);   // wave-uniform
      }
      if (SPEF_IRP_EARLY && ld_p >= 0) load_pa(ld_p);
      if (do_e) {
        T* Ew = Es0 + (ce & 1) * G::PINP * G::ES;
#pragma unroll
        for (int jj = 0; jj < G::EPT; ++jj) {
          const int pt = eg + G::NG * jj;
          if (pt >= G::PIN16) break;
          x4 o = relu_cvt4<DT>(e[jj]);
          uint2 u = *reinterpret_cast<uint2*>(&o);
          if (!interior) {   // the depthwise zero padding: hidden values of pixels outside the image are 0
            const uint32_t m = ((pvmask >> jj) & 1u) ? 0xffffffffu : 0u;
            u.x &= m;
            u.y &= m;
          }
          *reinterpret_cast<uint2*>(Ew + (pt * 16 + r16) * G::ES + 16 * hh + 4 * kg) = u;
        }
      }
    };

    load_ea(0);
    load_pa(0);
    SPEF_TRACE(2);
    __syncthreads();                                   // B0: input tile, depthwise weights, biases visible
    SPEF_TRACE(3);
    __builtin_amdgcn_s_waitcnt(0x0F70);                // vmcnt(0): no load in flight across the role loop's header
    if (G::BXR) read_bx();
    step(0, 0, true, false, SPEF_IRP_EARLY ? 1 : -1, -1);
    if (!SPEF_IRP_EARLY) load_ea(1);
    SPEF_TRACE(4);
    __syncthreads();                                   // B1: Es[0] complete
    SPEF_TRACE(5);
    // iteration 0: E(1) while the depthwise waves run V(0)
    step(1, 0, true, false, SPEF_IRP_EARLY ? 2 : -1, -1);
    if (!SPEF_IRP_EARLY) load_ea(2);
    SPEF_TRACE(6);
    __syncthreads();
    SPEF_TRACE(7);
    // iterations 1 .. NCH-2: E(i+1) and P(i-1)
#pragma unroll 1
    for (int i = 1; i + 1 < G::NCH; ++i) {
      step(i + 1, i - 1, true, true, SPEF_IRP_EARLY ? i + 2 : -1, SPEF_IRP_EARLY ? i : -1);
      if (!SPEF_IRP_EARLY) {
        load_ea(i + 2);
        load_pa(i);
      }
      SPEF_TRACE(6 + 2 * i);
      __syncthreads();
      SPEF_TRACE(7 + 2 * i);
    }
    // iteration NCH-1: P(NCH-2); iteration NCH: P(NCH-1)
    step(0, G::NCH - 2, false, true, -1, SPEF_IRP_EARLY ? G::NCH - 1 : -1);
    if (!SPEF_IRP_EARLY) load_pa(G::NCH - 1);
    SPEF_TRACE(6 + 2 * (G::NCH - 1));
    __syncthreads();
    SPEF_TRACE(7 + 2 * (G::NCH - 1));
    step(0, G::NCH - 1, false, true, -1, -1);

    // ---- epilogue: + residual from the staged input tile -> y (NHWC)
#pragma unroll
    for (int q = 0; q < G::POUT16; ++q) {
      const int o = q * 16 + r16;
      const int oy = o / TW, ox = o - (o / TW) * TW;
      const int gy = oy0 + oy, gx = ox0 + ox;
      if (gy >= OH || gx >= OW) continue;
      T* yr = Y + (((size_t)b * OH + gy) * OW + gx) * COUT;
#pragma unroll
      for (int t = 0; t < G::NCTW; ++t) {
        const int ct = wave + NM * t;
        if (ct >= G::NCT) continue;
        const int co = 16 * ct + 4 * kg;
        f32x4 v = acc[q][t];
        if constexpr (RES) {
          const x4 r = *reinterpret_cast<const x4*>(Xs + ((oy + 1) * G::IW + (ox + 1)) * G::XS + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
        }
        x4 o4;
#pragma unroll
        for (int e = 0; e < 4; ++e) o4[e] = (T)v[e];
        SPEF_KB_YSTORE(*reinterpret_cast<x4*>(yr + co) = o4, o4);
      }
    }
  } else {
    // =============================================================================== depthwise waves
    const int vw = wave - NM;
    int oyq[G::QPV], oxq[G::QPV];
#pragma unroll
    for (int qi = 0; qi < G::QPV; ++qi) {
      const int o = (vw * G::QPV + qi) * 16 + r16;
      oyq[qi] = o / TW;
      oxq[qi] = o - oyq[qi] * TW;
    }
    // V(c): chunk c's depthwise for this wave's output pixel tiles, 8 channels per lane -> Ds[c & 1]
    auto depthwise = [&](int c) {
      const T* Es = Es0 + (c & 1) * G::PINP * G::ES;
      T* Dw = Ds0 + (c & 1) * G::POUT * G::DS;
      const DW* sl = Wds + 32 * c + 8 * kg;
      DW8<DT> wt[9];
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) wt[tap].load(sl + tap * HID);
      float db[8];
      {
        const float4 u0 = *reinterpret_cast<const float4*>(Bd + 32 * c + 8 * kg);
        const float4 u1 = *reinterpret_cast<const float4*>(Bd + 32 * c + 8 * kg + 4);
        db[0] = u0.x; db[1] = u0.y; db[2] = u0.z; db[3] = u0.w;
        db[4] = u1.x; db[5] = u1.y; db[6] = u1.z; db[7] = u1.w;
      }
      if constexpr (G::PAIR) {
#pragma unroll
        for (int qi = 0; qi < G::QPV; qi += 2) {
          float a0[8], a1[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) a0[e] = a1[e] = db[e];
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            x8 v[4];                                       // the column's 4 window rows, read together
#pragma unroll
            for (int r = 0; r < 4; ++r)
              v[r] = *reinterpret_cast<const x8*>(Es + ((oyq[qi] + r) * G::IW + oxq[qi] + kx) * G::ES + 8 * kg);
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                a0[e] = fmaf((float)v[ky][e], wt[ky * 3 + kx][e], a0[e]);
                a1[e] = fmaf((float)v[ky + 1][e], wt[ky * 3 + kx][e], a1[e]);
              }
          }
          *reinterpret_cast<x8*>(Dw + ((vw * G::QPV + qi) * 16 + r16) * G::DS + 8 * kg) = relu_cvt8<DT>(a0);
          *reinterpret_cast<x8*>(Dw + ((vw * G::QPV + qi + 1) * 16 + r16) * G::DS + 8 * kg) = relu_cvt8<DT>(a1);
        }
      } else {
#pragma unroll
        for (int qi = 0; qi < G::QPV; ++qi) {
          x8 v[9];                                         // the 3x3 window, all reads before the first FMA
#pragma unroll
          for (int kx = 0; kx < 3; ++kx)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
              v[kx * 3 + ky] = *reinterpret_cast<const x8*>(
                  Es + ((oyq[qi] * S + ky) * G::IW + (oxq[qi] * S + kx)) * G::ES + 8 * kg);
          float a8[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) a8[e] = db[e];
#pragma unroll
          for (int kx = 0; kx < 3; ++kx)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
              for (int e = 0; e < 8; ++e) a8[e] = fmaf((float)v[kx * 3 + ky][e], wt[ky * 3 + kx][e], a8[e]);
          *reinterpret_cast<x8*>(Dw + ((vw * G::QPV + qi) * 16 + r16) * G::DS + 8 * kg) = relu_cvt8<DT>(a8);
        }
      }
    };
    SPEF_TRACE(2);
    __syncthreads();                                   // B0
    SPEF_TRACE(3);
    SPEF_TRACE(4);
    __syncthreads();                                   // B1: Es[0] complete
    SPEF_TRACE(5);
#pragma unroll 1
    for (int i = 0; i < G::NCH; ++i) {
      depthwise(i);
      SPEF_TRACE(6 + 2 * i);
      __syncthreads();
      SPEF_TRACE(7 + 2 * i);
    }
  }
  SPEF_TRACE(SPEF_TRACE_SLOTS - 1);
}

// (variant, cin, hidden, cout, stride, TH x TW tile, residual, MFMA waves, depthwise waves).
// Variant 0 is the default; others are alternatives for tuning sweeps (SPEF_OPT_IRB_VARIANT).
#define SPEF_IRP_TABLE(X)                                                \
  X(0, 96, 576, 160, 2, 8, 8, false, 8, 4)      /* block 14     */       \
  X(1, 96, 576, 160, 2, 8, 8, false, 4, 4)                               \
  X(0, 160, 960, 160, 1, 8, 8, true, 4, 4)      /* blocks 15-16 */       \
  X(1, 160, 960, 160, 1, 8, 8, true, 8, 4)                               \
  X(0, 160, 960, 320, 1, 8, 8, false, 4, 4)     /* block 17     */       \
  X(1, 160, 960, 320, 1, 8, 8, false, 8, 4)
// Measured per launch at B = 64 (tools/kbench): block 14 25.5 us (k_irw.hip 35.6), blocks 15-16 30.4 us (45.6),
// block 17 41.3 us (slab kernel 60.5). The 32x32-map blocks 8-13 stay on k_irw.hip: their 16x16 tiles do not fit
// the two extra slabs in LDS, and 8x16 tiles (two workgroup rounds per CU) measured 25-35 % slower than k_irw.hip.

template <typename DT, int CIN, int HID, int COUT, int S, int TH, int TW, bool RES, int NM, int NV>
static hipError_t irp_go(const void* x, const void* we, const float* be, const void* wd, const float* bd,
                         const void* wp, const float* bp, void* y, int B, int H, int W, int OH, int OW, hipStream_t s) {
  using DW = typename DT::DW;
  using T = typename DT::T;
  using G = IrpGeom<CIN, HID, COUT, S, TH, TW, NM, NV, (int)sizeof(DW)>;
  const int tiles_x = (OW + TW - 1) / TW, tiles_y = (OH + TH - 1) / TH;
  const int64_t nwg64 = (int64_t)tiles_x * tiles_y * B;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  const size_t lds = (size_t)G::LDS_BYTES;
  auto k = irp_kernel<DT, CIN, HID, COUT, S, TH, TW, RES, NM, NV>;
  static DevOnce attr_set;   // > 64 KiB dynamic LDS needs the attribute (once per instantiation)
  if (!attr_set.done() && lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr_set.set();
  }
  k<<<nwg, G::NW * 64, lds, s>>>((const T*)x, (const T*)we, be, (const DW*)wd, bd, (const T*)wp, bp, (T*)y, H, W, OH,
                                 OW, tiles_x, tiles_y, nwg);
  return hipGetLastError();
}

static bool irp_has(int variant, int cin, int hid, int cout, int stride, bool expand, bool res) {
#define SPEF_IRP_HAS(V, CI, HI, CO, ST, TH_, TW_, RS, NM_, NV_) \
  if (variant == V && cin == CI && hid == HI && cout == CO && stride == ST && expand && res == RS) return true;
  SPEF_IRP_TABLE(SPEF_IRP_HAS)
#undef SPEF_IRP_HAS
  return false;
}

bool irp_supported(int cin, int hid, int cout, int stride, bool expand, bool res) {
  return irp_has(0, cin, hid, cout, stride, expand, res);
}

hipError_t launch_irp(int variant, int dtype, int cin, int hid, int cout, int stride, bool res, const void* x,
                      const void* we, const float* be, const void* wd, const float* bd, const void* wp, const float* bp,
                      void* y, int B, int H, int W, int OH, int OW, hipStream_t s) {
  if (dtype != DT_F16 || !irp_has(variant, cin, hid, cout, stride, true, res)) variant = 0;
#define SPEF_IRP_CASE(V, CI, HI, CO, ST, TH_, TW_, RS, NM_, NV_)                                                    \
  if (variant == V && cin == CI && hid == HI && cout == CO && stride == ST && res == RS)                           \
    return dtype == DT_F16                                                                                         \
               ? irp_go<F16, CI, HI, CO, ST, TH_, TW_, RS, NM_, NV_>(x, we, be, wd, bd, wp, bp, y, B, H, W, OH, OW, \
                                                                    s)                                             \
               : irp_go<BF16, CI, HI, CO, ST, TH_, TW_, RS, NM_, NV_>(x, we, be, wd, bd, wp, bp, y, B, H, W, OH,    \
                                                                     OW, s);
  SPEF_IRP_TABLE(SPEF_IRP_CASE)
#undef SPEF_IRP_CASE
  return hipErrorNotSupported;
}

}  // namespace spef
