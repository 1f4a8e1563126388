// Fused InvertedResidual block (src/modeling/common/pytorch_layers.py:65-98) on gfx950:
//   expand 1x1 + BN + ReLU  ->  depthwise 3x3 (stride S) + BN + ReLU  ->  project 1x1 + BN  (+ x)
// in ONE kernel. The 6x-wide hidden tensor never leaves the CU: per output tile, the input tile (+halo) is
// staged in LDS once, the hidden channels are produced 32 at a time into a double-buffered LDS slab by MFMA,
// the depthwise stencil reads that slab and produces the project GEMM's B fragment directly in registers,
// and the project accumulates over hidden chunks in MFMA accumulators. HBM traffic per block = read x
// (+ halo re-reads, mostly L2 hits) + write y; weights stream from L2.
//
// Rounding points are identical to the unfused kernels (fp16/bf16 after expand, after depthwise, after
// project), and so is the accumulation order: the fused block is bit-identical to the unfused schedule.
//
// MFMA 16x16x32 C^T formulation (see k_conv.hip): A = weights [out ch][k], B = activations [k][pixel],
// lane l holds B[k = 8(l>>4)+e][pixel l&15] = 16 contiguous bytes of an LDS pixel row.
#include "spef_common.hpp"
#include "spef_kernels.hpp"

namespace spef {

template <int CIN, int HID, int COUT, int S, int TH, int TW, bool EXPAND, bool RES, int NW>
struct IrbGeom {
  static constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3;
  static constexpr int PIN = IH * IW;
  static constexpr int PIN16 = (PIN + 15) / 16;
  static constexpr int PINP = PIN16 * 16;
  static constexpr int CINP = (CIN + 31) / 32 * 32;
  static constexpr int XS = CINP + 8;        // Xs row stride (elements): +16 B against bank conflicts
  static constexpr int ES = EXPAND ? 40 : XS;  // hidden-chunk row stride (32 ch + 16 B)
  static constexpr int NCH = (HID + 31) / 32;
  static constexpr int HIDP = NCH * 32;      // project K (blob pads to 32)
  static constexpr int POUT = TH * TW;
  static constexpr int POUT16 = POUT / 16;
  static constexpr int QPW = POUT16 / NW;    // output pixel tiles per wave
  static constexpr int NCT = (COUT + 15) / 16;
  static constexpr int LDS_ELEMS = PINP * XS + (EXPAND ? 2 * PINP * ES : 0);
  static_assert(POUT % 16 == 0 && POUT16 % NW == 0, "output tile must split into 16-pixel MFMA tiles per wave");
  static_assert(CIN % 8 == 0 && HID % 8 == 0 && COUT % 4 == 0, "channel counts must be multiples of 8");
  static_assert(EXPAND || HID == 32, "t == 1 blocks are supported for 32 channels (MobileNet-V2 block 1)");
  static_assert(!RES || (S == 1 && CIN == COUT), "residual needs stride 1 and cin == cout");
};

template <typename DT, int CIN, int HID, int COUT, int S, int TH, int TW, bool EXPAND, bool RES, int NW>
__global__ __launch_bounds__(NW * 64) void irb_kernel(
    const typename DT::T* __restrict__ X, const typename DT::T* __restrict__ We, const float* __restrict__ be,
    const float* __restrict__ Wd, const float* __restrict__ bd, const typename DT::T* __restrict__ Wp,
    const float* __restrict__ bp, typename DT::T* __restrict__ Y, int H, int W, int OH, int OW, int tiles_x,
    int tiles_y, uint32_t nwg) {
  using G = IrbGeom<CIN, HID, COUT, S, TH, TW, EXPAND, RES, NW>;
  using T = typename DT::T;
  using x8 = typename DT::x8;
  using x4 = typename DT::x4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Xs = reinterpret_cast<T*>(smem);
  T* Es0 = Xs + G::PINP * G::XS;
  T* Es1 = Es0 + G::PINP * G::ES;

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  uint32_t L = xcd_remap(blockIdx.x, nwg);       // neighbouring tiles (shared halo rows) on one XCD
  const int tx = (int)(L % (uint32_t)tiles_x);
  L /= (uint32_t)tiles_x;
  const int ty = (int)(L % (uint32_t)tiles_y);
  const int b = (int)(L / (uint32_t)tiles_y);
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;

  // ---- 1. stage the input tile (+halo) in LDS; outside the image (and K padding) -> 0
  {
    constexpr int GPR = G::CINP / 8;        // 16-B groups per LDS row
    constexpr int CG = CIN / 8;             // valid groups
    const T* Xb = X + (size_t)b * H * W * CIN;
    for (int u = tid; u < G::PINP * GPR; u += NW * 64) {
      const int p = u / GPR, g = u - p * GPR;
      x8 v = zero8<DT>();
      if (p < G::PIN && g < CG) {
        const int py = p / G::IW, px = p - py * G::IW;
        const int iy = iy0 + py, ix = ix0 + px;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) v = load8<DT>(Xb + ((size_t)iy * W + ix) * CIN + g * 8);
      }
      *reinterpret_cast<x8*>(Xs + p * G::XS + g * 8) = v;
    }
  }
  __syncthreads();

  // per-lane output pixel of each owned 16-pixel tile
  int opix[G::QPW];
#pragma unroll
  for (int qi = 0; qi < G::QPW; ++qi) opix[qi] = (wave * G::QPW + qi) * 16 + r16;

  f32x4 acc[G::QPW][G::NCT];
#pragma unroll
  for (int qi = 0; qi < G::QPW; ++qi)
#pragma unroll
    for (int t = 0; t < G::NCT; ++t) acc[qi][t] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
  for (int c = 0; c < G::NCH; ++c) {
    const T* Es;
    if constexpr (EXPAND) {
      T* Ew = (c & 1) ? Es1 : Es0;
      const int vh = HID - 32 * c < 32 ? HID - 32 * c : 32;   // valid hidden channels in this chunk
      // ---- 2. expand: E[p][h] = relu(sum_k X[p][k] We[32c+h][k] + be) for all tile pixels
      for (int pt = wave; pt < G::PIN16; pt += NW) {
        f32x4 e0 = {0.f, 0.f, 0.f, 0.f}, e1 = {0.f, 0.f, 0.f, 0.f};
        const T* xr = Xs + (pt * 16 + r16) * G::XS + 8 * kg;
        const T* w0 = We + (size_t)(32 * c + r16) * G::CINP + 8 * kg;
#pragma unroll
        for (int ks = 0; ks < G::CINP / 32; ++ks) {
          const x8 bx = *reinterpret_cast<const x8*>(xr + 32 * ks);
          e0 = DT::mfma(load8<DT>(w0 + 32 * ks), bx, e0);
          if (vh > 16) e1 = DT::mfma(load8<DT>(w0 + 16 * G::CINP + 32 * ks), bx, e1);
        }
        const int p = pt * 16 + r16;
        bool pv = p < G::PIN;
        if (pv) {
          const int py = p / G::IW, px = p - py * G::IW;
          const int iy = iy0 + py, ix = ix0 + px;
          pv = iy >= 0 && iy < H && ix >= 0 && ix < W;     // zero padding of the depthwise input
        }
        T* er = Ew + p * G::ES + 4 * kg;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const f32x4 e = t ? e1 : e0;
          x4 o;
          if (16 * t < vh && pv) {
            const float4 bb = *reinterpret_cast<const float4*>(be + 32 * c + 16 * t + 4 * kg);
            o[0] = (T)fmaxf(e[0] + bb.x, 0.f);
            o[1] = (T)fmaxf(e[1] + bb.y, 0.f);
            o[2] = (T)fmaxf(e[2] + bb.z, 0.f);
            o[3] = (T)fmaxf(e[3] + bb.w, 0.f);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = (T)0.f;
          }
          *reinterpret_cast<x4*>(er + 16 * t) = o;
        }
      }
      __syncthreads();
      Es = Ew;
    } else {
      Es = Xs;
    }

    // ---- 3. depthwise 3x3 on this hidden chunk -> project B fragment in registers; 4. project MFMA
    const int hch = 32 * c + 8 * kg;           // this lane's 8 hidden channels
    const bool hv = hch < HID;
    float wdv[9][8];
    float bdv[8];
    if (hv) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const float4 a = *reinterpret_cast<const float4*>(Wd + tap * HID + hch);
        const float4 bq = *reinterpret_cast<const float4*>(Wd + tap * HID + hch + 4);
        wdv[tap][0] = a.x; wdv[tap][1] = a.y; wdv[tap][2] = a.z; wdv[tap][3] = a.w;
        wdv[tap][4] = bq.x; wdv[tap][5] = bq.y; wdv[tap][6] = bq.z; wdv[tap][7] = bq.w;
      }
      const float4 a = *reinterpret_cast<const float4*>(bd + hch);
      const float4 bq = *reinterpret_cast<const float4*>(bd + hch + 4);
      bdv[0] = a.x; bdv[1] = a.y; bdv[2] = a.z; bdv[3] = a.w;
      bdv[4] = bq.x; bdv[5] = bq.y; bdv[6] = bq.z; bdv[7] = bq.w;
    }
#pragma unroll
    for (int qi = 0; qi < G::QPW; ++qi) {
      x8 bf = zero8<DT>();
      if (hv) {
        const int oy = opix[qi] / TW, ox = opix[qi] - (opix[qi] / TW) * TW;
        float a8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) a8[e] = bdv[e];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int p = (oy * S + ky) * G::IW + (ox * S + kx);
            const x8 v = *reinterpret_cast<const x8*>(Es + p * G::ES + (EXPAND ? 8 * kg : hch));
#pragma unroll
            for (int e = 0; e < 8; ++e) a8[e] = fmaf((float)v[e], wdv[ky * 3 + kx][e], a8[e]);
          }
#pragma unroll
        for (int e = 0; e < 8; ++e) bf[e] = (T)fmaxf(a8[e], 0.f);
      }
      const T* wp = Wp + (size_t)r16 * G::HIDP + 32 * c + 8 * kg;
#pragma unroll
      for (int t = 0; t < G::NCT; ++t) acc[qi][t] = DT::mfma(load8<DT>(wp + (size_t)t * 16 * G::HIDP), bf, acc[qi][t]);
    }
  }

  // ---- 5. epilogue: + bias (+ residual from the staged input tile) -> y (NHWC)
#pragma unroll
  for (int qi = 0; qi < G::QPW; ++qi) {
    const int oy = opix[qi] / TW, ox = opix[qi] - (opix[qi] / TW) * TW;
    const int gy = oy0 + oy, gx = ox0 + ox;
    if (gy >= OH || gx >= OW) continue;
    T* yr = Y + (((size_t)b * OH + gy) * OW + gx) * COUT;
#pragma unroll
    for (int t = 0; t < G::NCT; ++t) {
      const int co = 16 * t + 4 * kg;
      if (co >= COUT) continue;
      const float4 bb = *reinterpret_cast<const float4*>(bp + co);
      f32x4 v = acc[qi][t];
      v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
      if constexpr (RES) {
        const x4 r = *reinterpret_cast<const x4*>(Xs + ((oy + 1) * G::IW + (ox + 1)) * G::XS + co);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
      }
      x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (T)v[e];
      *reinterpret_cast<x4*>(yr + co) = o;
    }
  }
}

// ------------------------------------------------------------------------------------------ dispatch
// One instantiation per MobileNet-V2 block geometry, tile sized so the LDS working set leaves room for
// 2-3 workgroups per CU. Unknown geometries return hipErrorNotSupported -> the executor falls back to the
// unfused kernels.
#define SPEF_IRB_TABLE(X)                                      \
  X(32, 32, 16, 1, 16, 16, false, false, 4)   /* block 1      */ \
  X(16, 96, 24, 2, 8, 8, true, false, 4)      /* block 2      */ \
  X(24, 144, 24, 1, 8, 16, true, true, 4)     /* block 3      */ \
  X(24, 144, 32, 2, 8, 8, true, false, 4)     /* block 4      */ \
  X(32, 192, 32, 1, 8, 16, true, true, 4)     /* blocks 5-6   */ \
  X(32, 192, 64, 2, 8, 8, true, false, 4)     /* block 7      */ \
  X(64, 384, 64, 1, 8, 16, true, true, 4)     /* blocks 8-10  */ \
  X(64, 384, 96, 1, 8, 16, true, false, 4)    /* block 11     */ \
  X(96, 576, 96, 1, 8, 16, true, true, 4)     /* blocks 12-13 */ \
  X(96, 576, 160, 2, 4, 8, true, false, 2)    /* block 14     */ \
  X(160, 960, 160, 1, 8, 8, true, true, 4)    /* blocks 15-16 */ \
  X(160, 960, 320, 1, 8, 8, true, false, 4)   /* block 17     */

template <typename DT, int CIN, int HID, int COUT, int S, int TH, int TW, bool EXPAND, bool RES, int NW>
static hipError_t irb_go(const void* x, const void* we, const float* be, const float* wd, const float* bd,
                         const void* wp, const float* bp, void* y, int B, int H, int W, int OH, int OW,
                         hipStream_t s) {
  using G = IrbGeom<CIN, HID, COUT, S, TH, TW, EXPAND, RES, NW>;
  using T = typename DT::T;
  const int tiles_x = (OW + TW - 1) / TW, tiles_y = (OH + TH - 1) / TH;
  const int64_t nwg64 = (int64_t)tiles_x * tiles_y * B;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  const size_t lds = (size_t)G::LDS_ELEMS * sizeof(T);
  auto k = irb_kernel<DT, CIN, HID, COUT, S, TH, TW, EXPAND, RES, NW>;
  static bool attr_set = false;   // > 64 KiB dynamic LDS needs the attribute (once per instantiation)
  if (!attr_set && lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  k<<<nwg, NW * 64, lds, s>>>((const T*)x, (const T*)we, be, wd, bd, (const T*)wp, bp, (T*)y, H, W, OH, OW, tiles_x,
                              tiles_y, nwg);
  return hipGetLastError();
}

template <typename DT>
static hipError_t irb_dispatch(int cin, int hid, int cout, int stride, bool expand, bool res, const void* x,
                               const void* we, const float* be, const float* wd, const float* bd, const void* wp,
                               const float* bp, void* y, int B, int H, int W, int OH, int OW, hipStream_t s) {
#define SPEF_IRB_CASE(CI, HI, CO, ST, TH_, TW_, EX, RS, NW_)                                                  \
  if (cin == CI && hid == HI && cout == CO && stride == ST && expand == EX && res == RS)                      \
    return irb_go<DT, CI, HI, CO, ST, TH_, TW_, EX, RS, NW_>(x, we, be, wd, bd, wp, bp, y, B, H, W, OH, OW, s);
  SPEF_IRB_TABLE(SPEF_IRB_CASE)
#undef SPEF_IRB_CASE
  return hipErrorNotSupported;
}

bool irb_supported(int cin, int hid, int cout, int stride, bool expand, bool res) {
#define SPEF_IRB_HAS(CI, HI, CO, ST, TH_, TW_, EX, RS, NW_) \
  if (cin == CI && hid == HI && cout == CO && stride == ST && expand == EX && res == RS) return true;
  SPEF_IRB_TABLE(SPEF_IRB_HAS)
#undef SPEF_IRB_HAS
  return false;
}

hipError_t launch_irb(int dtype, int cin, int hid, int cout, int stride, bool expand, bool res, const void* x,
                      const void* we, const float* be, const float* wd, const float* bd, const void* wp,
                      const float* bp, void* y, int B, int H, int W, int OH, int OW, hipStream_t s) {
  return dtype == DT_F16
             ? irb_dispatch<F16>(cin, hid, cout, stride, expand, res, x, we, be, wd, bd, wp, bp, y, B, H, W, OH, OW, s)
             : irb_dispatch<BF16>(cin, hid, cout, stride, expand, res, x, we, be, wd, bd, wp, bp, y, B, H, W, OH, OW,
                                  s);
}

}  // namespace spef
