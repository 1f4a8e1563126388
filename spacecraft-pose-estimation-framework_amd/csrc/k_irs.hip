// Strip-streaming fused InvertedResidual block (src/modeling/common/pytorch_layers.py:65-98) for the
// high-resolution MobileNet-V2 blocks: expand 1x1 + BN + ReLU -> depthwise 3x3 (stride S) + BN + ReLU ->
// project 1x1 + BN (+ x), with the hidden tensor kept in REGISTERS instead of an LDS slab.
//
// Why: in the slab kernel (k_irb.hip) every hidden value is written to LDS once and read back by nine
// depthwise taps, and all waves of a workgroup meet at a barrier per 32-channel chunk; for the wide-map blocks
// that LDS traffic and the lock-stepped phases, not HBM or the MFMA pipe, set the time.
//
// Here each wave owns a strip of 16 output columns x R output rows and streams the hidden channels through
// registers: for a 32-channel chunk and a depthwise column kx it runs the expand MFMA directly on the input
// pixels that column of taps reads (lane j <- input column j*S + kx), so the depthwise becomes lane-local fp32
// FMAs -- no hidden values cross lanes or touch LDS, and there are no per-chunk barriers. The price is the expand
// recomputed per kx (MFMA, which these blocks leave mostly idle). LDS holds only the input tile (+halo) and the
// block's weights (a few tens of KB for these geometries), staged once per workgroup behind the single barrier.
//
// Layouts (gfx950 16x16 MFMA lane map, see spef_common.hpp): expand D[i = hidden ch][j = pixel] gives lane
// (j, kg) the 4 hidden channels 16g + 4kg + r of pixel j; the depthwise keeps that layout; the project's B
// fragment for a 32-channel chunk is {channels 4kg..4kg+3, 16+4kg..16+4kg+3} of the pixel, so the project
// weights are read with the same K permutation (two 8-B pieces per fragment; no blob change).
//
// Rounding: the expand output stays fp32 (the slab kernels round it to the storage type), the depthwise
// accumulates in fp32 in the same tap order (kx outer, ky inner) from the same bias, its output is rounded to
// fp16/bf16 (+ReLU) as the project's B operand, and the project accumulates in fp32 from the bias. Results are
// therefore closer to the FP32 reference than the slab kernels', not bit-identical to them.
#include "spef_common.hpp"
#include "spef_kernels.hpp"

#include <type_traits>

namespace spef {

template <int CIN, int HID, int COUT, int S, int R, int NW>
struct IrsGeom {
  static constexpr int TW = 16;                   // output columns per tile (the MFMA pixel dimension)
  static constexpr int TH = R * NW;               // output rows per tile (R per wave)
  static constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3;
  static constexpr bool K16 = CIN == 16;          // 16-channel input: K = 16 MFMA
  static constexpr int CINP = K16 ? 16 : (CIN + 31) / 32 * 32;
  static constexpr int XS = CINP + 8;             // LDS pixel stride (elements)
  static constexpr int KS = K16 ? 1 : CINP / 32;
  static constexpr int WKP = (CIN + 31) / 32 * 32;   // blob row length of the expand weights
  static constexpr int NCH = (HID + 31) / 32;
  static constexpr int HIDP = NCH * 32;           // project K (blob pads to 32)
  static constexpr int NCT = (COUT + 15) / 16;
  static constexpr int RIN = (R - 1) * S + 3;     // input rows one wave reads
  static constexpr int PIX = IH * IW;
  static constexpr int WES = WKP + 8;             // LDS row strides of the staged weights (elements)
  static constexpr int WPS = HIDP + 8;
  static constexpr int NCTP = NCT * 16;
  template <int DWB>
  static constexpr int lds_bytes() {
    return (PIX * XS + HIDP * WES + NCTP * WPS) * 2 + 9 * HIDP * DWB + 2 * HIDP * 4;
  }
  static_assert(CIN % 8 == 0 && HID % 16 == 0 && COUT % 4 == 0, "channel counts");
};

template <typename DT, int CIN, int HID, int COUT, int S, int R, int NW, bool RES>
__global__ __launch_bounds__(NW * 64) void irs_kernel(
    const typename DT::T* __restrict__ X, const typename DT::T* __restrict__ We, const float* __restrict__ be,
    const typename DT::DW* __restrict__ Wd, const float* __restrict__ bd, const typename DT::T* __restrict__ Wp,
    const float* __restrict__ bp, typename DT::T* __restrict__ Y, int H, int W, int OH, int OW, int tiles_x,
    int tiles_y, uint32_t nwg) {
  using G = IrsGeom<CIN, HID, COUT, S, R, NW>;
  using T = typename DT::T;
  using DW = typename DT::DW;
  using x8 = typename DT::x8;
  using x4 = typename DT::x4;
  using W4 = typename std::conditional<sizeof(DW) == 2, f16x4, f32x4>::type;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Xs = reinterpret_cast<T*>(smem);                 // [PIX][XS] input tile (+halo)
  T* WEs = Xs + G::PIX * G::XS;                        // [HIDP][WES] expand weights (rows >= HID zero)
  T* WPs = WEs + G::HIDP * G::WES;                     // [NCTP][WPS] project weights
  DW* WDs = reinterpret_cast<DW*>(WPs + G::NCTP * G::WPS);   // [9][HIDP] depthwise weights (zero >= HID)
  float* BE = reinterpret_cast<float*>(WDs + 9 * G::HIDP);   // [HIDP] expand bias
  float* BD = BE + G::HIDP;                                  // [HIDP] depthwise bias

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int j = lane & 15, kg = lane >> 4;
  uint32_t L = xcd_remap(blockIdx.x, nwg);
  const int tx = (int)(L % (uint32_t)tiles_x);
  L /= (uint32_t)tiles_x;
  const int ty = (int)(L % (uint32_t)tiles_y);
  const int b = (int)(L / (uint32_t)tiles_y);
  const int oy0 = ty * G::TH, ox0 = tx * G::TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;

  // ---- 1. input tile (+halo) and ALL of the block's weights -> LDS in one pass of 16-B pieces (all loads in
  // flight before the first store): zero outside the image, in the K padding and past HID.
  {
    constexpr int GPR = G::CINP / 8, CG = CIN / 8;
    constexpr int NXP = G::PIX * GPR;                         // input pieces
    constexpr int NEP = G::HIDP * (G::WKP / 8);               // expand weight pieces
    constexpr int NPP = G::NCTP * (G::HIDP / 8);              // project weight pieces
    constexpr int DPR = G::HIDP * (int)sizeof(DW) / 16;       // depthwise pieces per tap
    constexpr int NDP = 9 * DPR;
    constexpr int NBP = G::HIDP / 4;                          // bias pieces per vector
    constexpr int NTOT = NXP + NEP + NPP + NDP + 2 * NBP;
    constexpr int NIT = (NTOT + NW * 64 - 1) / (NW * 64);
    const T* Xb = X + (size_t)b * H * W * CIN;
    uint4 v[NIT];
    char* dst[NIT];
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      int u = tid + NW * 64 * i;
      const void* src = nullptr;
      dst[i] = nullptr;
      if (u < NXP) {
        const int p = u / GPR, g = u - p * GPR;
        dst[i] = reinterpret_cast<char*>(Xs + p * G::XS + g * 8);
        const int py = p / G::IW, px = p - py * G::IW;
        const int iy = iy0 + py, ix = ix0 + px;
        if (g < CG && iy >= 0 && iy < H && ix >= 0 && ix < W) src = Xb + ((size_t)iy * W + ix) * CIN + g * 8;
      } else if ((u -= NXP) < NEP) {
        const int row = u / (G::WKP / 8), g = u - row * (G::WKP / 8);
        dst[i] = reinterpret_cast<char*>(WEs + row * G::WES + g * 8);
        if (row < HID) src = We + (size_t)row * G::WKP + g * 8;
      } else if ((u -= NEP) < NPP) {
        const int row = u / (G::HIDP / 8), g = u - row * (G::HIDP / 8);
        dst[i] = reinterpret_cast<char*>(WPs + row * G::WPS + g * 8);
        src = Wp + (size_t)row * G::HIDP + g * 8;
      } else if ((u -= NPP) < NDP) {
        const int tap = u / DPR, g = u - tap * DPR;
        constexpr int EPP = 16 / (int)sizeof(DW);
        dst[i] = reinterpret_cast<char*>(WDs + tap * G::HIDP + g * EPP);
        if (g * EPP < HID) src = Wd + (size_t)tap * HID + g * EPP;
      } else if ((u -= NDP) < 2 * NBP) {
        const int which = u / NBP, g = u - which * NBP;
        dst[i] = reinterpret_cast<char*>((which ? BD : BE) + 4 * g);
        if (4 * g < HID) src = (which ? bd : be) + 4 * g;
      }
      v[i] = src ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NIT; ++i)
      if (dst[i]) *reinterpret_cast<uint4*>(dst[i]) = v[i];
  }
  __syncthreads();

  // ---- 2. this wave's strip: output rows wy0 .. wy0+R-1 of the tile, columns 0..15 (lane j)
  const int wy0 = wave * R;
  const int ry0 = iy0 + wy0 * S;                       // image row of the strip's first input row
  // the depthwise zero padding applies to the HIDDEN tensor: expand outputs at pixels outside the image are 0
  const bool interior = ry0 >= 0 && ry0 + G::RIN <= H && ix0 >= 0 && ix0 + G::IW <= W;
  uint32_t colok = 0;                                  // bit kx: lane's input column for tap column kx in image
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    const int ix = ix0 + j * S + kx;
    if (ix >= 0 && ix < W) colok |= 1u << kx;
  }

  f32x4 acc[R][G::NCT];   // project accumulators start at the folded-BN bias
#pragma unroll
  for (int t = 0; t < G::NCT; ++t) {
    const float4 bb = *reinterpret_cast<const float4*>(bp + t * 16 + 4 * kg);
#pragma unroll
    for (int y = 0; y < R; ++y) acc[y][t] = f32x4{bb.x, bb.y, bb.z, bb.w};
  }

#pragma unroll 1
  for (int c = 0; c < G::NCH; ++c) {
    const bool g1 = 32 * c + 16 < HID;                // the chunk's second 16-channel group exists
    // expand A fragments (rows = hidden channels 32c + 16g + j), expand and depthwise biases -- from LDS
    x8 a[2][G::KS];
    x4 q[2];
    float4 eb[2], db[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const T* wr = WEs + (32 * c + 16 * g + j) * G::WES;
      if constexpr (G::K16) {
        q[g] = *reinterpret_cast<const x4*>(wr + 4 * kg);
      } else {
#pragma unroll
        for (int ks = 0; ks < G::KS; ++ks) a[g][ks] = *reinterpret_cast<const x8*>(wr + 32 * ks + 8 * kg);
      }
      eb[g] = *reinterpret_cast<const float4*>(BE + 32 * c + 16 * g + 4 * kg);
      db[g] = *reinterpret_cast<const float4*>(BD + 32 * c + 16 * g + 4 * kg);
    }
    // project A fragments with the chunk's K permutation: k = 8kg'+e <-> hidden 32c + 16(e>>2) + 4kg' + (e&3)
    x8 pa[G::NCT];
#pragma unroll
    for (int t = 0; t < G::NCT; ++t) {
      const T* wr = WPs + (t * 16 + j) * G::WPS + 32 * c + 4 * kg;
      const x4 lo = *reinterpret_cast<const x4*>(wr), hi = *reinterpret_cast<const x4*>(wr + 16);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pa[t][e] = lo[e];
        pa[t][4 + e] = hi[e];
      }
    }

    // depthwise accumulators of the strip: [row][group*4 + r], starting at the folded-BN bias
    float d[R][8];
#pragma unroll
    for (int y = 0; y < R; ++y) {
      d[y][0] = db[0].x; d[y][1] = db[0].y; d[y][2] = db[0].z; d[y][3] = db[0].w;
      d[y][4] = db[1].x; d[y][5] = db[1].y; d[y][6] = db[1].z; d[y][7] = db[1].w;
    }

#pragma unroll 1
    for (int kx = 0; kx < 3; ++kx) {
      // depthwise weights of this tap column, [ky][group] x 4 channels, in the blob's type (fp16: read by
      // v_fma_mix directly, exact)
      W4 wf[3][2];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int g = 0; g < 2; ++g)
          wf[ky][g] = *reinterpret_cast<const W4*>(WDs + (ky * 3 + kx) * G::HIDP + 32 * c + 16 * g + 4 * kg);

#pragma unroll
      for (int r = 0; r < G::RIN; ++r) {
        // expand of input row r (of the strip) at the pixels tap column kx reads: lane j <- column j*S + kx
        const T* xr = Xs + ((wy0 * S + r) * G::IW + j * S + kx) * G::XS;
        f32x4 e[2];
#pragma unroll
        for (int g = 0; g < 2; ++g) e[g] = f32x4{eb[g].x, eb[g].y, eb[g].z, eb[g].w};   // bias as MFMA C
        if constexpr (G::K16) {
          const x4 bx = *reinterpret_cast<const x4*>(xr + 4 * kg);
          e[0] = DT::mfma16(q[0], bx, e[0]);
          if (g1) e[1] = DT::mfma16(q[1], bx, e[1]);
        } else {
#pragma unroll
          for (int ks = 0; ks < G::KS; ++ks) {
            const x8 bx = *reinterpret_cast<const x8*>(xr + 32 * ks + 8 * kg);
            e[0] = DT::mfma(a[0][ks], bx, e[0]);
            if (g1) e[1] = DT::mfma(a[1][ks], bx, e[1]);
          }
        }
        // expand ReLU, kept in fp32 (no storage rounding: the hidden tensor never leaves the registers)
        float hv[8];
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {
          hv[e4] = fmaxf(e[0][e4], 0.f);
          hv[4 + e4] = fmaxf(e[1][e4], 0.f);
        }
        if (!interior) {
          const int iy = ry0 + r;
          const bool ok = iy >= 0 && iy < H && ((colok >> kx) & 1u);
#pragma unroll
          for (int e8 = 0; e8 < 8; ++e8) hv[e8] = ok ? hv[e8] : 0.f;
        }
        // this input row feeds output rows y with ky = r - y*S in [0, 2]; per output: kx outer, ky inner
#pragma unroll
        for (int y = 0; y < R; ++y) {
          const int ky = r - y * S;
          if (ky < 0 || ky > 2) continue;
#pragma unroll
          for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4)
              d[y][4 * g + e4] = fmaf(hv[4 * g + e4], (float)wf[ky][g][e4], d[y][4 * g + e4]);
        }
      }
    }

    // depthwise ReLU -> project B fragment (permuted K) -> project MFMA
#pragma unroll
    for (int y = 0; y < R; ++y) {
      x8 bf;
#pragma unroll
      for (int e = 0; e < 8; ++e) bf[e] = (T)fmaxf(d[y][e], 0.f);
#pragma unroll
      for (int t = 0; t < G::NCT; ++t) acc[y][t] = DT::mfma(pa[t], bf, acc[y][t]);
    }
  }

  // ---- 3. epilogue: (+ residual from the staged input) -> y (NHWC); lane holds channels 16t + 4kg + r of pixel j
  const int gx = ox0 + j;
#pragma unroll
  for (int y = 0; y < R; ++y) {
    const int gy = oy0 + wy0 + y;
    if (gy >= OH || gx >= OW) continue;
    T* yr = Y + (((size_t)b * OH + gy) * OW + gx) * COUT;
#pragma unroll
    for (int t = 0; t < G::NCT; ++t) {
      const int co = t * 16 + 4 * kg;
      if (co >= COUT) continue;
      f32x4 v = acc[y][t];
      if constexpr (RES) {
        const x4 rr = *reinterpret_cast<const x4*>(Xs + ((wy0 + y + 1) * G::IW + (j + 1)) * G::XS + co);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (float)rr[e];
      }
      x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (T)v[e];
      *reinterpret_cast<x4*>(yr + co) = o;
    }
  }
}

// (cin, hidden, cout, stride, R rows per wave, NW waves, residual)
#define SPEF_IRS_TABLE(X)                                   \
  X(16, 96, 24, 2, 4, 4, false)     /* block 2      */    \
  X(24, 144, 24, 1, 4, 4, true)     /* block 3      */    \
  X(24, 144, 32, 2, 4, 2, false)    /* block 4      */    \
  X(32, 192, 32, 1, 4, 4, true)     /* blocks 5-6   */    \
  X(32, 192, 64, 2, 2, 4, false)    /* block 7      */

template <typename DT, int CIN, int HID, int COUT, int S, int R, int NW, bool RES>
static hipError_t irs_go(const void* x, const void* we, const float* be, const void* wd, const float* bd,
                         const void* wp, const float* bp, void* y, int B, int H, int W, int OH, int OW, hipStream_t s) {
  using G = IrsGeom<CIN, HID, COUT, S, R, NW>;
  using T = typename DT::T;
  using DW = typename DT::DW;
  const int tiles_x = (OW + G::TW - 1) / G::TW, tiles_y = (OH + G::TH - 1) / G::TH;
  const int64_t nwg64 = (int64_t)tiles_x * tiles_y * B;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  constexpr size_t lds = (size_t)G::template lds_bytes<(int)sizeof(DW)>();
  static_assert(lds <= 163840, "LDS budget");
  auto k = irs_kernel<DT, CIN, HID, COUT, S, R, NW, RES>;
  static bool attr_set = false;   // > 64 KiB dynamic LDS needs the attribute (once per instantiation)
  if (!attr_set && lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  k<<<nwg, NW * 64, lds, s>>>((const T*)x, (const T*)we, be, (const DW*)wd, bd, (const T*)wp, bp, (T*)y, H, W, OH, OW,
                              tiles_x, tiles_y, nwg);
  return hipGetLastError();
}

bool irs_supported(int cin, int hid, int cout, int stride, bool expand, bool res) {
#define SPEF_IRS_HAS(CI, HI, CO, ST, R_, NW_, RS) \
  if (cin == CI && hid == HI && cout == CO && stride == ST && expand && res == RS) return true;
  SPEF_IRS_TABLE(SPEF_IRS_HAS)
#undef SPEF_IRS_HAS
  return false;
}

hipError_t launch_irs(int dtype, int cin, int hid, int cout, int stride, bool res, const void* x, const void* we,
                      const float* be, const void* wd, const float* bd, const void* wp, const float* bp, void* y,
                      int B, int H, int W, int OH, int OW, hipStream_t s) {
#define SPEF_IRS_CASE(CI, HI, CO, ST, R_, NW_, RS)                                                              \
  if (cin == CI && hid == HI && cout == CO && stride == ST && res == RS)                                        \
    return dtype == DT_F16                                                                                      \
               ? irs_go<F16, CI, HI, CO, ST, R_, NW_, RS>(x, we, be, wd, bd, wp, bp, y, B, H, W, OH, OW, s)     \
               : irs_go<BF16, CI, HI, CO, ST, R_, NW_, RS>(x, we, be, wd, bd, wp, bp, y, B, H, W, OH, OW, s);
  SPEF_IRS_TABLE(SPEF_IRS_CASE)
#undef SPEF_IRS_CASE
  return hipErrorNotSupported;
}

}  // namespace spef
