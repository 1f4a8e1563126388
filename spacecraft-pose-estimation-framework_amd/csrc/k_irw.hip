// Wave-specialised fused InvertedResidual block (src/modeling/common/pytorch_layers.py:65-98) for the
// mid- and low-resolution MobileNet-V2 blocks (64x64 down to 16x16 maps, 192-960 hidden channels).
//
// The slab kernel (k_irb.hip) runs expand, barrier, depthwise+project on every wave in lock step: all waves of
// a SIMD are in the MFMA-heavy expand or in the VALU-heavy depthwise at the same time, and at one workgroup per
// CU (these blocks have 256 tiles for 256 CUs) nothing else fills the other pipe. Here the workgroup's waves
// take fixed roles and form a two-stage pipeline over 32-channel hidden chunks:
//
//   expand waves  [0, NE):   chunk c+1: hidden = relu(x We^T + be) on MFMA -> LDS slab Es[(c+1) & 1]
//   depthwise waves [NE, NW): chunk c:   3x3 depthwise (+BN, ReLU) from Es[c & 1] on VALU -> project MFMA
//
// with one barrier per chunk, so every SIMD holds one wave of each role and its matrix and vector pipes work
// concurrently. The input tile (+halo), all depthwise weights and all biases are staged in LDS once; the expand
// and project weight fragments stream from L2 into registers one chunk ahead (each role reads only its own).
//
// Arithmetic and rounding are those of the slab kernel (and of the unfused kernels): bias as the MFMA C input,
// fp16/bf16 after expand, fp32 depthwise in kx-outer/ky-inner tap order, fp16/bf16 after the depthwise, fp32
// project accumulation over chunks in order -> bit-identical to the one-kernel-per-conv schedule.
#include "spef_common.hpp"
#include <type_traits>
#include "spef_kernels.hpp"

namespace spef {

// Per-chunk barrier of the role loops. SPEF_KBENCH_NO_CHUNK_BARRIER (tools/kbench timing ablation only, wrong results)
// removes it to measure what the chunk hand-off costs.
#ifdef SPEF_KBENCH_NO_CHUNK_BARRIER
#define SPEF_IRW_CHUNK_SYNC() ((void)0)
#else
#define SPEF_IRW_CHUNK_SYNC() __syncthreads()
#endif
// Further tools/kbench timing ablations (wrong results, never in the library): SPEF_KBENCH_IRW_NO_WLOAD (no weight
// fragment loads after the first chunks), SPEF_KBENCH_IRW_NO_EXPAND (expand waves only keep the barrier count),
// SPEF_KBENCH_IRW_NO_DWMATH (depthwise reads kept, 2 instead of 4 VALU per channel and tap column),
// SPEF_KBENCH_IRW_NO_PROJ (no project MFMAs).

// Vertical-pair depthwise (fp16, stride 1, 16-wide tiles; blocks 8-13): the hidden slab holds, per (row pair, column)
// position, one dword per channel = (row 2m, row 2m+1), in four 8-channel regions (k_irb.hip's VP layout); a kernel
// column's taps ky 0,1 (or 1,2) are one v_dot2_f32_f16 and the third one v_fma_mix: 6 instead of 9 VALU per 3x3
// tap set. The depthwise weights are staged once as (w[0][kx], w[1][kx]) / (w[1][kx], w[2][kx]) pairs. The unfused
// dw_kernel (irb_dw_mode) evaluates the same instructions in the same order: bit-identical.
constexpr bool irw_vp(bool f16, int s, int th, int tw) { return f16 && s == 1 && tw == 16 && th % 2 == 0; }

template <int CIN, int HID, int COUT, int S, int TH, int TW, int NE, int ND, int WCO, int DWB, bool VP = false>
struct IrwGeom {
  static constexpr int NW = NE + ND;
  static constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3;
  static constexpr int PIN = IH * IW, PIN16 = (PIN + 15) / 16, PINP = PIN16 * 16;
  static constexpr bool K16 = CIN == 16;          // 16-channel input: K = 16 MFMA
  static constexpr int CINP = K16 ? 16 : (CIN + 31) / 32 * 32;
  static constexpr int KS = K16 ? 1 : CINP / 32;
  static constexpr int WKP = (CIN + 31) / 32 * 32;   // blob row length of the expand weights
  static constexpr int ES = 48;                   // 16-B granules per row = 2 mod 4: conflict-free b128 reads
  static constexpr int HIDP_ = (HID + 31) / 32 * 32;
  // VP slab: row pairs x columns, 16 positions per expand unit (two MFMA pixel tiles: even and odd row)
  static constexpr int PR = (IH + 1) / 2, NQ = PR * IW, NU = (NQ + 15) / 16, NQP = NU * 16;
  static constexpr int RS = NQP * 32 + 16;        // bytes per channel-group region (regions 16 B apart mod 256 B)
  static constexpr int EPU = (NU + NE - 1) / NE;  // expand units per expand wave
  static constexpr int ES_BYTES = VP ? 4 * RS : PINP * ES * 2;   // one hidden slab buffer
  static constexpr int WD_BYTES = VP ? 6 * HIDP_ * 4 : 9 * HIDP_ * DWB;
  static constexpr int bytes_for(int xs) { return PINP * xs * 2 + 2 * ES_BYTES + WD_BYTES + 2 * HIDP_ * 4; }
  static constexpr int XS = bytes_for(CINP + 16) <= 163840 ? CINP + 16 : CINP + 8;   // input row stride
  static constexpr int NCH = (HID + 31) / 32, HIDP = NCH * 32;
  static constexpr int NCT = (COUT + 15) / 16;
  static constexpr int EPT = (PIN16 + NE - 1) / NE;     // expand pixel tiles per expand wave
  static constexpr int POUT16 = TH * TW / 16;
  static constexpr int WP = ND / WCO;                   // pixel groups among the depthwise waves
  static constexpr int QPW = POUT16 / WP;               // output pixel tiles per depthwise wave
  static constexpr int NCTW = NCT / WCO;                // output-channel tiles per depthwise wave
  static constexpr bool PAIR = S == 1 && TW == 16 && QPW % 2 == 0;
  static constexpr int LDS_BYTES = bytes_for(XS);
  static_assert(CIN % 8 == 0 && HID % 16 == 0 && COUT % 8 == 0, "channel counts");
  static_assert(TH * TW % 16 == 0 && POUT16 % WP == 0 && ND % WCO == 0 && NCT % WCO == 0, "tile split");
  static_assert(EPT <= 32 && 2 * EPU <= 32, "validity mask is 32 bits");
  static_assert(!VP || PAIR, "VP depthwise runs two output rows per step");
  static_assert(2 * NCH + 8 <= SPEF_TRACE_SLOTS, "trace slots");
  static_assert(LDS_BYTES <= 163840, "LDS budget");
};

template <typename DT, int CIN, int HID, int COUT, int S, int TH, int TW, bool RES, int NE, int ND, int WCO>
__global__ __launch_bounds__((NE + ND) * 64) void irw_kernel(
    const typename DT::T* __restrict__ X, const typename DT::T* __restrict__ We, const float* __restrict__ be,
    const typename DT::DW* __restrict__ Wd, const float* __restrict__ bd, const typename DT::T* __restrict__ Wp,
    const float* __restrict__ bp, typename DT::T* __restrict__ Y, int H, int W, int OH, int OW, int tiles_x,
    int tiles_y, uint32_t nwg) {
  using DW = typename DT::DW;
  constexpr bool VP = irw_vp(std::is_same<DT, F16>::value, S, TH, TW);
  using G = IrwGeom<CIN, HID, COUT, S, TH, TW, NE, ND, WCO, (int)sizeof(DW), VP>;
  using T = typename DT::T;
  using x8 = typename DT::x8;
  using x4 = typename DT::x4;
  constexpr int NW = G::NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Xs = reinterpret_cast<T*>(smem);                          // [PINP][XS] input tile (+halo)
  T* Es0 = Xs + G::PINP * G::XS;                               // [2] hidden chunk slabs ([PINP][ES] or VP regions)
  char* Wdb = reinterpret_cast<char*>(Es0) + 2 * G::ES_BYTES;
  DW* Wds = reinterpret_cast<DW*>(Wdb);                        // [9][HIDP] depthwise weights (0 past HID)
  uint32_t* Wdp = reinterpret_cast<uint32_t*>(Wdb);            // VP: [kx][(w0,w1) | (w1,w2)][HIDP] weight pairs
  float* Be = reinterpret_cast<float*>(Wdb + G::WD_BYTES);     // [HIDP] expand bias
  float* Bd = Be + G::HIDP;                                    // [HIDP] depthwise bias

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  SPEF_TRACE(0);
  uint32_t L = xcd_remap(blockIdx.x, nwg);
  const int tx = (int)(L % (uint32_t)tiles_x);
  L /= (uint32_t)tiles_x;
  const int ty = (int)(L % (uint32_t)tiles_y);
  const int b = (int)(L / (uint32_t)tiles_y);
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;

  // ---- 1. input tile, depthwise weights and biases -> LDS (16-B pieces, all loads before the stores)
  {
    constexpr int GPR = G::CINP / 8, CG = CIN / 8;
    constexpr int NXP = G::PINP * GPR;
    constexpr int EPP = 16 / (int)sizeof(DW);
    constexpr int DPR = G::HIDP / EPP;                 // depthwise pieces per tap
    constexpr int NDP = VP ? 0 : 9 * DPR;
    constexpr int NBP = G::HIDP / 4;
    constexpr int NTOT = NXP + NDP + 2 * NBP;
    constexpr int NIT = (NTOT + NW * 64 - 1) / (NW * 64);
    const T* Xb = X + (size_t)b * H * W * CIN;
    // VP weight pairs: piece u = (kx, j, 4 channels) from two 8-B pieces of taps (j, kx) and (j + 1, kx)
    constexpr int NVP = VP ? 6 * G::HIDP / 4 : 0;
    constexpr int NIV = (NVP + NW * 64 - 1) / (NW * 64);
    uint2 wa[NIV > 0 ? NIV : 1], wb[NIV > 0 ? NIV : 1];
#pragma unroll
    for (int i = 0; i < NIV; ++i) {
      const int u = tid + NW * 64 * i;
      const int g = u % (G::HIDP / 4), kj = u / (G::HIDP / 4), kx = kj >> 1, j = kj & 1;
      const bool ok = u < NVP && 4 * g < HID;
      const int off = ok ? (j * 3 + kx) * HID + 4 * g : 0;
      wa[i] = *reinterpret_cast<const uint2*>(Wd + off);
      wb[i] = *reinterpret_cast<const uint2*>(Wd + (ok ? off + 3 * HID : 0));
      if (!ok) wa[i] = wb[i] = make_uint2(0, 0);
    }
    uint4 v[NIT];
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      int u = tid + NW * 64 * i;
      const void* src = nullptr;
      if (u < NXP) {
        const int p = u / GPR, g = u - p * GPR;
        if (p < G::PIN && g < CG) {
          const int py = p / G::IW, px = p - py * G::IW;
          const int iy = iy0 + py, ix = ix0 + px;
          if (iy >= 0 && iy < H && ix >= 0 && ix < W) src = Xb + SPEF_KB_XOFF(((size_t)iy * W + ix) * CIN + g * 8);
        }
      } else if ((u -= NXP) < NDP) {
        const int tap = u / DPR, g = u - tap * DPR;
        if (g * EPP < HID) src = Wd + (size_t)tap * HID + g * EPP;
      } else if ((u -= NDP) < 2 * NBP) {
        const int which = u / NBP, g = u - which * NBP;
        if (4 * g < HID) src = (which ? bd : be) + 4 * g;
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
        dst = reinterpret_cast<char*>(Wds + tap * G::HIDP + g * EPP);
      } else if ((u -= NDP) < 2 * NBP) {
        const int which = u / NBP, g = u - which * NBP;
        dst = reinterpret_cast<char*>((which ? Bd : Be) + 4 * g);
      }
      if (dst) *reinterpret_cast<uint4*>(dst) = v[i];
    }
#pragma unroll
    for (int i = 0; i < NIV; ++i) {   // (lo = tap j, hi = tap j + 1 of each channel)
      const int u = tid + NW * 64 * i;
      if (u < NVP) {
        const uint2 a = wa[i], c = wb[i];
        *reinterpret_cast<uint4*>(Wdp + 4 * u) =
            make_uint4((a.x & 0xffffu) | (c.x << 16), (a.x >> 16) | (c.x & 0xffff0000u), (a.y & 0xffffu) | (c.y << 16),
                       (a.y >> 16) | (c.y & 0xffff0000u));
      }
    }
  }
  SPEF_TRACE(1);

  const bool is_expand = wave < NE;   // wave-uniform role

  // ---- expand role state: weight fragments of the next chunk (prefetched from L2), pixel validity
  const int ew = wave;                                   // expand wave index (valid when is_expand)
  const bool interior = iy0 >= 0 && ix0 >= 0 && iy0 + G::IH <= H && ix0 + G::IW <= W;
  uint32_t pvmask = 0;
  x8 ea0[G::KS], ea1[G::KS];                             // expand A fragments of the chunk being produced
  x4 eq0, eq1;                                           // (16-channel input: K = 16 fragments)
  auto load_ea = [&](int c) {
#ifdef SPEF_KBENCH_IRW_NO_WLOAD
    if (c > 1) return;
#endif
    const bool ok0 = c < G::NCH, ok1 = ok0 && 32 * c + 16 < HID;
    if constexpr (G::K16) {
      const T* w0 = We + (size_t)(32 * c + r16) * G::WKP + 4 * kg;
      eq0 = ok0 ? *reinterpret_cast<const x4*>(w0) : x4{};
      eq1 = ok1 ? *reinterpret_cast<const x4*>(w0 + 16 * G::WKP) : x4{};
    } else {
#pragma unroll
      for (int ks = 0; ks < G::KS; ++ks) {
        const T* w0 = We + (size_t)(32 * c + r16) * G::WKP + 32 * ks + 8 * kg;
        ea0[ks] = ok0 ? load8<DT>(w0) : zero8<DT>();
        ea1[ks] = ok1 ? load8<DT>(w0 + 16 * G::WKP) : zero8<DT>();
      }
    }
  };
#ifdef SPEF_KBENCH_IRW_RESIDENT
  typename std::conditional<G::K16, x4, x8>::type vres[G::EPU][2][G::K16 ? 1 : G::KS];
#endif
  // expand of chunk c into slab Es[c & 1] by this expand wave
  auto expand_vp = [&](int c) {
    // unit u = 16 pair positions q; lane r16 computes the even- and odd-row pixel of its position (two MFMA pixel
    // tiles) and stores each channel's pair as one dword (channels 4kg.. -> region kg/2, 16+4kg.. -> region 2+kg/2)
    char* Ew = reinterpret_cast<char*>(Es0) + (c & 1) * G::ES_BYTES;
    const float4 eb0 = *reinterpret_cast<const float4*>(Be + 32 * c + 4 * kg);
    const float4 eb1 = *reinterpret_cast<const float4*>(Be + 32 * c + 16 + 4 * kg);
    constexpr int NBX = G::K16 ? 1 : G::KS;
    using BX = typename std::conditional<G::K16, x4, x8>::type;
    constexpr bool VBATCH = G::EPU * 2 * NBX * (G::K16 ? 2 : 4) <= 48;
#ifdef SPEF_KBENCH_IRW_RESIDENT
    auto& vbx = vres;
#else
    BX vbx[G::EPU][2][NBX];
#endif
    auto read_vbx = [&](int jj) {
      const int q = (ew + NE * jj) * 16 + r16;
      const int qc = q < G::NQ ? q : G::NQ - 1;
      const int pr = qc / G::IW, col = qc - pr * G::IW;
      const int p0 = 2 * pr * G::IW + col;
      const int p1 = (G::IH % 2 == 0 || 2 * pr + 1 < G::IH) ? p0 + G::IW : p0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const T* xr = Xs + (h ? p1 : p0) * G::XS;
        if constexpr (G::K16) {
          vbx[jj][h][0] = *reinterpret_cast<const x4*>(xr + 4 * kg);
        } else {
#pragma unroll
          for (int ks = 0; ks < G::KS; ++ks) vbx[jj][h][ks] = *reinterpret_cast<const x8*>(xr + 8 * kg + 32 * ks);
        }
      }
    };
#pragma unroll
    for (int jj = 0; jj < G::EPU; ++jj) {
#ifdef SPEF_KBENCH_IRW_RESIDENT
      if (c > 0) break;
#endif
      if (!VBATCH || ew + NE * jj >= G::NU) break;
      read_vbx(jj);
    }
#pragma unroll
    for (int jj = 0; jj < G::EPU; ++jj) {
      const int u = ew + NE * jj;
      if (u >= G::NU) break;
      if (!VBATCH) read_vbx(jj);
      f32x4 e[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        e[h][0] = f32x4{eb0.x, eb0.y, eb0.z, eb0.w};
        e[h][1] = f32x4{eb1.x, eb1.y, eb1.z, eb1.w};
        if constexpr (G::K16) {
          e[h][0] = DT::mfma16(eq0, vbx[jj][h][0], e[h][0]);
          e[h][1] = DT::mfma16(eq1, vbx[jj][h][0], e[h][1]);
        } else {
#pragma unroll
          for (int ks = 0; ks < G::KS; ++ks) {
            e[h][0] = DT::mfma(ea0[ks], vbx[jj][h][ks], e[h][0]);
            e[h][1] = DT::mfma(ea1[ks], vbx[jj][h][ks], e[h][1]);
          }
        }
      }
      uint4 d[2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
        d[t] = make_uint4(relu_pk2(e[0][t][0], e[1][t][0]), relu_pk2(e[0][t][1], e[1][t][1]),
                          relu_pk2(e[0][t][2], e[1][t][2]), relu_pk2(e[0][t][3], e[1][t][3]));
      if (!interior) {   // zero the halves of pixels outside the image (the depthwise padding)
        const uint32_t m = (((pvmask >> (2 * jj)) & 1u) ? 0x0000ffffu : 0u) |
                           (((pvmask >> (2 * jj)) & 2u) ? 0xffff0000u : 0u);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          d[t].x &= m; d[t].y &= m; d[t].z &= m; d[t].w &= m;
        }
      }
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      char* er = Ew + (u * 16 + r16) * 32 + (kg & 1) * 16;
      *reinterpret_cast<u32x4*>(er + (kg >> 1) * G::RS) = u32x4{d[0].x, d[0].y, d[0].z, d[0].w};
      *reinterpret_cast<u32x4*>(er + (2 + (kg >> 1)) * G::RS) = u32x4{d[1].x, d[1].y, d[1].z, d[1].w};
    }
  };
  auto expand = [&](int c) {
#ifdef SPEF_KBENCH_IRW_NO_EXPAND
    if (c > 0) return;
#endif
    if constexpr (VP) {
      expand_vp(c);
    } else {
      T* Ew = Es0 + (c & 1) * G::PINP * G::ES;
      const float4 eb0 = *reinterpret_cast<const float4*>(Be + 32 * c + 4 * kg);
      const float4 eb1 = *reinterpret_cast<const float4*>(Be + 32 * c + 16 + 4 * kg);
      // all of this wave's B fragments first, then MFMAs + epilogues (the compiler cannot hoist an Xs read above the
      // previous tile's slab store: same LDS array), within a register budget for the expand role
      constexpr int NBX = G::K16 ? 1 : G::KS;
      constexpr bool BATCH = G::EPT * NBX * (G::K16 ? 2 : 4) <= 48;
      typename std::conditional<G::K16, x4, x8>::type bxs[G::EPT][NBX];
      auto read_bx = [&](int jj) {
        const int pt = ew + NE * jj;
        if constexpr (G::K16) {
          bxs[jj][0] = *reinterpret_cast<const x4*>(Xs + (pt * 16 + r16) * G::XS + 4 * kg);
        } else {
#pragma unroll
          for (int ks = 0; ks < G::KS; ++ks)
            bxs[jj][ks] = *reinterpret_cast<const x8*>(Xs + (pt * 16 + r16) * G::XS + 8 * kg + 32 * ks);
        }
      };
#pragma unroll
      for (int jj = 0; jj < G::EPT; ++jj) {
        if (!BATCH || ew + NE * jj >= G::PIN16) break;
        read_bx(jj);
      }
#pragma unroll
      for (int jj = 0; jj < G::EPT; ++jj) {
        const int pt = ew + NE * jj;
        if (pt >= G::PIN16) break;
        if (!BATCH) read_bx(jj);
        f32x4 e0 = {eb0.x, eb0.y, eb0.z, eb0.w}, e1 = {eb1.x, eb1.y, eb1.z, eb1.w};   // bias as MFMA C
        if constexpr (G::K16) {
          e0 = DT::mfma16(eq0, bxs[jj][0], e0);
          e1 = DT::mfma16(eq1, bxs[jj][0], e1);
        } else {
#pragma unroll
          for (int ks = 0; ks < G::KS; ++ks) {
            e0 = DT::mfma(ea0[ks], bxs[jj][ks], e0);
            e1 = DT::mfma(ea1[ks], bxs[jj][ks], e1);
          }
        }
        x4 o0 = relu_cvt4<DT>(e0), o1 = relu_cvt4<DT>(e1);
        uint2 u0 = *reinterpret_cast<uint2*>(&o0), u1 = *reinterpret_cast<uint2*>(&o1);
        if (!interior) {   // the depthwise zero padding: hidden values of pixels outside the image are 0
          const uint32_t m0 = ((pvmask >> jj) & 1u) ? 0xffffffffu : 0u;
          u0.x &= m0; u0.y &= m0; u1.x &= m0; u1.y &= m0;
        }
        T* er = Ew + (pt * 16 + r16) * G::ES + 4 * kg;
        *reinterpret_cast<uint2*>(er) = u0;
        *reinterpret_cast<uint2*>(er + 16) = u1;
      }
    }
  };

  // ---- depthwise role state
  const int dwv = wave - NE;                             // depthwise wave index (valid when !is_expand)
  const int wp = dwv % G::WP, wc = dwv / G::WP;
  int oyq[G::QPW], oxq[G::QPW];
#pragma unroll
  for (int qi = 0; qi < G::QPW; ++qi) {
    const int o = (wp * G::QPW + qi) * 16 + r16;
    oyq[qi] = o / TW;
    oxq[qi] = o - oyq[qi] * TW;
  }
  f32x4 acc[G::QPW][G::NCTW];
  x8 pa[G::NCTW];                                        // project A fragments of the chunk being consumed
  auto load_pa = [&](int c) {
    const T* wpp = Wp + (size_t)(wc * G::NCTW * 16 + r16) * G::HIDP + 32 * c + 8 * kg;
#pragma unroll
    for (int t = 0; t < G::NCTW; ++t) pa[t] = c < G::NCH ? load8<DT>(wpp + (size_t)t * 16 * G::HIDP) : zero8<DT>();
  };

  // The two roles run separate loops with the same barrier count (2 + NCH), so each role's registers (the
  // project accumulators, the expand fragments) are allocated independently.
  if (is_expand) {
    if (VP && !interior) {   // VP: bits 2j / 2j+1 = even / odd row pixel of unit j
#pragma unroll
      for (int jj = 0; jj < G::EPU; ++jj) {
        const int q = (ew + NE * jj) * 16 + r16;
        if (q < G::NQ) {
          const int pr = q / G::IW, col = q - pr * G::IW;
          const int iy = iy0 + 2 * pr, ix = ix0 + col;
          const bool cx = ix >= 0 && ix < W;
          if (cx && iy >= 0 && iy < H) pvmask |= 1u << (2 * jj);
          if (cx && 2 * pr + 1 < G::IH && iy + 1 >= 0 && iy + 1 < H) pvmask |= 2u << (2 * jj);
        }
      }
    } else if (!interior)   // only edge tiles mask (workgroup-uniform branch)
#pragma unroll
    for (int jj = 0; jj < G::EPT; ++jj) {
      const int p = (ew + NE * jj) * 16 + r16;
      if (p < G::PIN) {
        const int py = p / G::IW, px = p - py * G::IW;
        const int iy = iy0 + py, ix = ix0 + px;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) pvmask |= 1u << jj;
      }
    }
    load_ea(0);
    SPEF_TRACE(2);
    __syncthreads();                                      // input tile, depthwise weights, biases visible
    SPEF_TRACE(3);
    expand(0);
    load_ea(1);
    SPEF_TRACE(4);
    __syncthreads();                                      // Es[0] visible
    SPEF_TRACE(5);
#pragma unroll 1
    for (int c = 0; c < G::NCH; ++c) {
      if (c + 1 < G::NCH) {
        expand(c + 1);          // into Es[(c+1) & 1]: last read by the depthwise of chunk c-1, before the barrier
        load_ea(c + 2);
      }
      SPEF_TRACE(6 + 2 * c);
      SPEF_IRW_CHUNK_SYNC();    // Es[(c+1) & 1] complete; Es[c & 1] free for chunk c+2
      SPEF_TRACE(7 + 2 * c);
    }
  } else {
#pragma unroll
    for (int t = 0; t < G::NCTW; ++t) {
      const float4 bb = *reinterpret_cast<const float4*>(bp + (wc * G::NCTW + t) * 16 + 4 * kg);
#pragma unroll
      for (int qi = 0; qi < G::QPW; ++qi) acc[qi][t] = f32x4{bb.x, bb.y, bb.z, bb.w};
    }
    load_pa(0);
    SPEF_TRACE(2);
    __syncthreads();
    SPEF_TRACE(3);
    SPEF_TRACE(4);
    __syncthreads();
    SPEF_TRACE(5);
    // Retire load_pa(0) before the loop: otherwise the loop header merges "pa pending" from this edge, and the
    // waitcnt pass makes every chunk's project MFMAs wait for the next chunk's fragment loads issued just before.
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    // One chunk: depthwise from Es[c & 1] with the project fragments pcur; the next chunk's fragments are issued
    // into pnext (the last chunk re-reads its own: valid addresses, no branch). The chunk loop below alternates two
    // fragment buffers instead of copying them.
    x8 pb[G::NCTW];
    auto dw_chunk = [&](const int c, x8 (&pcur)[G::NCTW], x8 (&pnext)[G::NCTW]) {
      const T* Es = Es0 + (c & 1) * G::PINP * G::ES;
      const DW* sl = Wds + 32 * c;                        // tap t of chunk c: sl[t * HIDP + ch]
      const bool hv = 32 * c + 8 * kg < HID;
      // next chunk's project fragments: issued now, consumed after this chunk's MFMAs
      {
        const int cn = c + 1 < G::NCH ? c + 1 : c;
        const T* wpp = Wp + (size_t)(wc * G::NCTW * 16 + r16) * G::HIDP + 32 * cn + 8 * kg;
#pragma unroll
        for (int t = 0; t < G::NCTW; ++t)
#ifdef SPEF_KBENCH_IRW_NO_WLOAD
          pnext[t] = pcur[t];
#else
          pnext[t] = load8<DT>(wpp + (size_t)t * 16 * G::HIDP);
#endif
      }
      float db[8];
      {
        const float4 u0 = *reinterpret_cast<const float4*>(Bd + 32 * c + 8 * kg);
        const float4 u1 = *reinterpret_cast<const float4*>(Bd + 32 * c + 8 * kg + 4);
        db[0] = u0.x; db[1] = u0.y; db[2] = u0.z; db[3] = u0.w;
        db[4] = u1.x; db[5] = u1.y; db[6] = u1.z; db[7] = u1.w;
      }
      if constexpr (VP) {
        // per kernel column kx: row oy (even) dot2(ky 0,1) then fma(ky 2); row oy + 1 fma(ky 0) then dot2(ky 1,2)
        // -- dw_kernel<.., VP>'s order. This lane's channels 8kg.. live in region kg (32 B per position).
        auto rd8 = [&](const void* p, uint32_t v[8]) {
          const uint4 a = *reinterpret_cast<const uint4*>(p), b = *(reinterpret_cast<const uint4*>(p) + 1);
          v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        };
        const char* er = reinterpret_cast<const char*>(Es0) + (c & 1) * G::ES_BYTES + kg * G::RS;
        uint32_t w01[3][8], w12[3][8];   // the chunk's weight pairs, read once for all of this wave's pixel tiles
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          rd8(Wdp + (2 * kx) * G::HIDP + 32 * c + 8 * kg, w01[kx]);
          rd8(Wdp + (2 * kx + 1) * G::HIDP + 32 * c + 8 * kg, w12[kx]);
        }
#pragma unroll
        for (int qi = 0; qi < G::QPW; qi += 2) {   // output rows oy (even) and oy + 1: pairs m = oy / 2 and m + 1
          x8 bf0, bf1;
          {
            float a0[8], a1[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) a0[e] = a1[e] = db[e];
            const char* pb = er + ((oyq[qi] >> 1) * G::IW + oxq[qi]) * 32;
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
              uint32_t pc[8], pn[8];
              rd8(pb + kx * 32, pc);
              rd8(pb + (G::IW + kx) * 32, pn);
#pragma unroll
              for (int e = 0; e < 8; ++e) {
#ifdef SPEF_KBENCH_IRW_NO_DWMATH
                a0[e] = dot2h(pc[e], w01[kx][e], a0[e]);
                a1[e] = dot2h(pn[e], w12[kx][e], a1[e]);
#else
                a1[e] = fmaf(h_hi(pc[e]), h_lo(w01[kx][e]), a1[e]);
                a0[e] = dot2h(pc[e], w01[kx][e], a0[e]);
                a0[e] = fmaf(h_lo(pn[e]), h_hi(w12[kx][e]), a0[e]);
                a1[e] = dot2h(pn[e], w12[kx][e], a1[e]);
#endif
              }
            }
            bf0 = relu_cvt8<DT>(a0);
            bf1 = relu_cvt8<DT>(a1);
          }
#ifdef SPEF_KBENCH_IRW_NO_PROJ
          asm volatile("" ::"v"(bf0), "v"(bf1));
#else
#pragma unroll
          for (int t = 0; t < G::NCTW; ++t) {
            acc[qi][t] = DT::mfma(pcur[t], bf0, acc[qi][t]);
            acc[qi + 1][t] = DT::mfma(pcur[t], bf1, acc[qi + 1][t]);
          }
#endif
        }
      } else {
      // the chunk's 9 depthwise weight vectors, read once for all of this wave's pixel tiles
      DW8<DT> wt[9];
      if (hv) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) wt[tap].load(sl + tap * G::HIDP + 8 * kg);
      }
      if constexpr (G::PAIR) {
#pragma unroll
        for (int qi = 0; qi < G::QPW; qi += 2) {
          x8 bf0 = zero8<DT>(), bf1 = zero8<DT>();
          if (hv) {
            float a0[8], a1[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) a0[e] = a1[e] = db[e];
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
              x8 v[4];                                     // the column's 4 window rows, read together
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
            bf0 = relu_cvt8<DT>(a0);
            bf1 = relu_cvt8<DT>(a1);
          }
#pragma unroll
          for (int t = 0; t < G::NCTW; ++t) {
            acc[qi][t] = DT::mfma(pcur[t], bf0, acc[qi][t]);
            acc[qi + 1][t] = DT::mfma(pcur[t], bf1, acc[qi + 1][t]);
          }
        }
      } else {
#pragma unroll
        for (int qi = 0; qi < G::QPW; ++qi) {
          x8 bf = zero8<DT>();
          if (hv) {
            x8 v[9];                                       // the 3x3 window, all reads before the first FMA
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
            bf = relu_cvt8<DT>(a8);
          }
#pragma unroll
          for (int t = 0; t < G::NCTW; ++t) acc[qi][t] = DT::mfma(pcur[t], bf, acc[qi][t]);
        }
      }
      }
      SPEF_TRACE(6 + 2 * c);
      SPEF_IRW_CHUNK_SYNC();
      SPEF_TRACE(7 + 2 * c);
    };
    if constexpr (VP) {
#pragma unroll 1
      for (int c = 0; c + 1 < G::NCH; c += 2) {
        dw_chunk(c, pa, pb);
        dw_chunk(c + 1, pb, pa);
      }
      if constexpr (G::NCH % 2 == 1) dw_chunk(G::NCH - 1, pa, pb);
    } else {   // (the unpaired depthwise has no registers for two inlined chunk bodies)
#pragma unroll 1
      for (int c = 0; c < G::NCH; ++c) {
        dw_chunk(c, pa, pb);
#pragma unroll
        for (int t = 0; t < G::NCTW; ++t) pa[t] = pb[t];
      }
    }
  }

  // ---- epilogue (depthwise waves): + residual from the staged input tile -> y (NHWC)
  if (!is_expand) {
#pragma unroll
    for (int qi = 0; qi < G::QPW; ++qi) {
      const int oy = oyq[qi], ox = oxq[qi];
      const int gy = oy0 + oy, gx = ox0 + ox;
      if (gy >= OH || gx >= OW) continue;
      T* yr = Y + (((size_t)b * OH + gy) * OW + gx) * COUT;
#pragma unroll
      for (int t = 0; t < G::NCTW; ++t) {
        const int co = (wc * G::NCTW + t) * 16 + 4 * kg;
        if (co >= COUT) continue;
        f32x4 v = acc[qi][t];
        if constexpr (RES) {
          const x4 r = *reinterpret_cast<const x4*>(Xs + ((oy + 1) * G::IW + (ox + 1)) * G::XS + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
        }
        x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (T)v[e];
        SPEF_KB_YSTORE(*reinterpret_cast<x4*>(yr + co) = o, o);
      }
    }
  }
  SPEF_TRACE(SPEF_TRACE_SLOTS - 1);
}

// (variant, cin, hidden, cout, stride, TH x TW tile, residual, expand waves, depthwise waves, cout groups).
// Variant 0 is the default; others are alternatives for tuning sweeps (SPEF_OPT_IRB_VARIANT). With the pair depthwise,
// 4 depthwise waves of two pair steps each (weight pairs read once for both) beat 8 waves of one step on blocks 12-13
// (interleaved A/B: 88.8 -> 82.2 us per step) and tie on blocks 8-10; block 11 keeps 4. (4 expand + 2 depthwise waves
// spill.)
#define SPEF_IRW_TABLE(X)                                                   \
  X(0, 64, 384, 64, 1, 16, 16, true, 4, 4, 1)      /* blocks 8-10  */       \
  X(1, 64, 384, 64, 1, 16, 16, true, 4, 8, 1)                               \
  X(0, 64, 384, 96, 1, 16, 16, false, 4, 4, 1)     /* block 11     */       \
  X(1, 64, 384, 96, 1, 16, 16, false, 4, 8, 1)                              \
  X(0, 96, 576, 96, 1, 16, 16, true, 4, 4, 1)      /* blocks 12-13 */       \
  X(1, 96, 576, 96, 1, 16, 16, true, 4, 8, 1)                               \
  X(0, 96, 576, 160, 2, 8, 8, false, 4, 4, 2)      /* block 14     */       \
  X(1, 96, 576, 160, 2, 8, 8, false, 4, 8, 2)                               \
  X(0, 160, 960, 160, 1, 8, 8, true, 4, 4, 2)      /* blocks 15-16 */       \
  X(1, 160, 960, 160, 1, 8, 8, true, 4, 8, 2)
// Blocks 2-4 stay on the slab kernel (measured: the wave-specialised form is 0-70 % slower there -- the stride-2
// input tiles make the double-buffered slab too large for more than one or two workgroups per CU).
// Blocks 5-6 (32 -> 192 -> 32, 64x64 maps) moved back to the slab kernel (8x16 tiles, 4 waves) once its prologue
// loads were branch-free and its expand weights prefetched: 76 us vs 85 us here.
// Block 17 (160 -> 960 -> 320) stays on the slab kernel: with 20 output-channel tiles the depthwise waves carry
// too many accumulators (measured 72-80 us here vs 61 us slab).

template <typename DT, int CIN, int HID, int COUT, int S, int TH, int TW, bool RES, int NE, int ND, int WCO>
static hipError_t irw_go(const void* x, const void* we, const float* be, const void* wd, const float* bd,
                         const void* wp, const float* bp, void* y, int B, int H, int W, int OH, int OW, hipStream_t s) {
  using DW = typename DT::DW;
  using T = typename DT::T;
  using G = IrwGeom<CIN, HID, COUT, S, TH, TW, NE, ND, WCO, (int)sizeof(DW),
                    irw_vp(std::is_same<DT, F16>::value, S, TH, TW)>;
  const int tiles_x = (OW + TW - 1) / TW, tiles_y = (OH + TH - 1) / TH;
  const int64_t nwg64 = (int64_t)tiles_x * tiles_y * B;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  const size_t lds = (size_t)G::LDS_BYTES;
  auto k = irw_kernel<DT, CIN, HID, COUT, S, TH, TW, RES, NE, ND, WCO>;
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

static bool irw_has(int variant, int cin, int hid, int cout, int stride, bool expand, bool res) {
#define SPEF_IRW_HAS(V, CI, HI, CO, ST, TH_, TW_, RS, NE_, ND_, WC_) \
  if (variant == V && cin == CI && hid == HI && cout == CO && stride == ST && expand && res == RS) return true;
  SPEF_IRW_TABLE(SPEF_IRW_HAS)
#undef SPEF_IRW_HAS
  return false;
}

bool irw_supported(int cin, int hid, int cout, int stride, bool expand, bool res) {
  return irw_has(0, cin, hid, cout, stride, expand, res);
}

hipError_t launch_irw(int variant, int dtype, int cin, int hid, int cout, int stride, bool res, const void* x,
                      const void* we, const float* be, const void* wd, const float* bd, const void* wp, const float* bp,
                      void* y, int B, int H, int W, int OH, int OW, hipStream_t s) {
  if (dtype != DT_F16 || !irw_has(variant, cin, hid, cout, stride, true, res)) variant = 0;
#define SPEF_IRW_CASE(V, CI, HI, CO, ST, TH_, TW_, RS, NE_, ND_, WC_)                                               \
  if (variant == V && cin == CI && hid == HI && cout == CO && stride == ST && res == RS)                            \
    return dtype == DT_F16                                                                                          \
               ? irw_go<F16, CI, HI, CO, ST, TH_, TW_, RS, NE_, ND_, WC_>(x, we, be, wd, bd, wp, bp, y, B, H, W, OH, \
                                                                        OW, s)                                     \
               : irw_go<BF16, CI, HI, CO, ST, TH_, TW_, RS, NE_, ND_, WC_>(x, we, be, wd, bd, wp, bp, y, B, H, W,   \
                                                                         OH, OW, s);
  SPEF_IRW_TABLE(SPEF_IRW_CASE)
#undef SPEF_IRW_CASE
  return hipErrorNotSupported;
}

}  // namespace spef
