// fp32-accurate fused schedule on the fp16 matrix cores (blob dtype 5, "fp16x2"): the parity variant for heads
// whose output error the fp16 schedule cannot bound -- sharp URSONet heads (tools/sharp_head_budget.py: fp16 storage
// gives 1.6e-2 max |d logit| at head_std 0.3, hi + lo everything 1.8e-5) and the unpooled keypoint head
// (head/keypoints.py:20-27).
//
// Every value that feeds a matrix product is carried as an unevaluated pair of fp16 numbers, v = hi + lo with
// hi = fp16(v), lo = fp16(v - hi) (22 significant bits; |v - hi - lo| <= 2^-22 |v|, or 3e-8 absolute where lo is
// subnormal). A product a * b is the three MFMAs a_hi b_hi + a_lo b_hi + a_hi b_lo on the fp16 MFMA
// (v_mfma_f32_16x16x32_f16: fp32 accumulation, 16 cycles), which is 5.3x the rate of the exact fp32 MFMA
// (v_mfma_f32_16x16x4_f32, 8 instructions of 32 cycles for the same 16x16x32 tile; cdna_hip_programming.md section 3).
// The dropped a_lo b_lo term is below 2^-22 relative.
//
//   x2_irb_kernel  one InvertedResidual (pytorch_layers.py:65-98) per kernel: input tile (+halo) fp32 from HBM, split
//                  once into hi / lo LDS tiles; per 32-channel hidden chunk the expand (3 MFMAs per K step) writes
//                  ReLU(x We^T + be) as fp32 into an LDS slab; the depthwise 3x3 runs in fp32 (v_fma_f32 chains,
//                  kx-outer / ky-inner) on the slab, its ReLU'd output is split into hi / lo project B fragments in
//                  registers; the project accumulates over chunks in fp32 MFMA accumulators; + residual (fp32, read
//                  back from HBM) -> fp32 block output. Block 1 (t = 1) stages its input straight into the slab.
//   x2_pw_kernel   1x1 conv on fp32 activations (the last ConvBnAct 320 -> 1280, mobilenet_v2.py:264): B fragments
//                  split on load, ReLU, fp32 output (the keypoint head's flatten input or the URSONet mean's).
//
// Block I/O is fp32 NHWC; weights come from the blob split by the packer (spef_amd/blob.py, dtype fp16x2).
#include "spef_common.hpp"
#include "spef_kernels.hpp"

namespace spef {

// hi / lo split of 8 fp32 values (the residual v - hi is exact in fp32; fmaf((float)h, -1, v) is one v_fma_mix)
__device__ __forceinline__ void split8(const float v[8], f16x8& hi, f16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const _Float16 h = (_Float16)v[e];
    hi[e] = h;
    lo[e] = (_Float16)fmaf((float)h, -1.0f, v[e]);
  }
}
__device__ __forceinline__ void split4(float4 v, uint2& hi, uint2& lo) {
  const float a[4] = {v.x, v.y, v.z, v.w};
  _Float16 h[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = (_Float16)a[e];
    l[e] = (_Float16)fmaf((float)h[e], -1.0f, a[e]);
  }
  hi = make_uint2(pack_h2(h[0], h[1]), pack_h2(h[2], h[3]));
  lo = make_uint2(pack_h2(l[0], l[1]), pack_h2(l[2], l[3]));
}
// acc += (a_hi + a_lo)(b_hi + b_lo) without the lo*lo term
__device__ __forceinline__ f32x4 mfma_x2(f16x8 ah, f16x8 al, f16x8 bh, f16x8 bl, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc, 0, 0, 0);
}

// Geometry. Output tile TH x TW, NW waves; the depthwise/project phase gives wave w the output pixel tiles of group
// w % WP and the output-channel tiles of group w / WP (WCO groups; WCO > 1 repeats the depthwise to cut accumulators).
template <int CIN, int HID, int COUT, int S, int TH, int TW, bool EXPAND, int NW, int WCO>
struct X2Geom {
  static constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3;
  static constexpr int PIN = IH * IW, PIN16 = (PIN + 15) / 16, PINP = PIN16 * 16;
  static constexpr int CINP = (CIN + 31) / 32 * 32;   // K of the expand (blob rows padded to 32, zeros)
  static constexpr int KS = CINP / 32;
  static constexpr int XS = CINP + 16;                // hi / lo tile row (halves): 2 mod 4 granules
  static constexpr int SS = S == 1 ? 40 : 36;         // slab row (floats)
  static constexpr int NCH = (HID + 31) / 32, HIDP = NCH * 32;
  static constexpr int NCT = (COUT + 15) / 16;
  static constexpr int POUT16 = TH * TW / 16;
  static constexpr int WP = NW / WCO, QPW = POUT16 / WP, NCTW = NCT / WCO;
  static constexpr int EPT = (PIN16 + NW - 1) / NW;   // expand pixel tiles per wave
  static constexpr int X_BYTES = EXPAND ? 2 * PINP * XS * 2 : 0;
  static constexpr int LDS_BYTES = X_BYTES + PINP * SS * 4;
  static_assert(CIN % 4 == 0 && COUT % 4 == 0 && HID % 8 == 0, "channel counts");
  static_assert(EXPAND || (CIN == HID && CIN % 32 == 0), "t == 1 blocks stage their input as the hidden slab");
  static_assert(TH * TW % 16 == 0 && POUT16 % WP == 0 && NW % WCO == 0 && NCT % WCO == 0, "tile split");
  static_assert(EPT <= 32, "validity mask is 32 bits");
  static_assert(LDS_BYTES <= 163840, "LDS budget");
};

template <int CIN, int HID, int COUT, int S, int TH, int TW, bool EXPAND, bool RES, int NW, int WCO>
__global__ __launch_bounds__(NW * 64) void x2_irb_kernel(
    const float* __restrict__ X, const _Float16* __restrict__ We, const float* __restrict__ be,
    const float* __restrict__ Wd, const float* __restrict__ bd, const _Float16* __restrict__ Wp,
    const float* __restrict__ bp, float* __restrict__ Y, int H, int W, int OH, int OW, int tiles_x, int tiles_y,
    uint32_t nwg) {
  using G = X2Geom<CIN, HID, COUT, S, TH, TW, EXPAND, NW, WCO>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  _Float16* Xh = reinterpret_cast<_Float16*>(smem);   // [PINP][XS] input tile, hi
  _Float16* Xl = Xh + G::PINP * G::XS;                 // [PINP][XS] lo
  float* Sl = reinterpret_cast<float*>(smem + G::X_BYTES);   // [PINP][SS] hidden chunk (fp32)

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  uint32_t L = xcd_remap(blockIdx.x, nwg);
  const int tx = (int)(L % (uint32_t)tiles_x);
  L /= (uint32_t)tiles_x;
  const int ty = (int)(L % (uint32_t)tiles_y);
  const int b = (int)(L / (uint32_t)tiles_y);
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
  const float* Xb = X + (size_t)b * H * W * CIN;

  // ---- 1. input tile (+halo, zero outside the image): fp32 -> hi / lo LDS tiles (t = 1: fp32 slab). All global
  // loads of a thread are issued before its LDS stores.
  {
    constexpr int GPR = G::CINP / 4, CG = CIN / 4;     // float4 pieces per pixel row (padded / real)
    constexpr int NP = G::PINP * GPR;
    constexpr int NIT = (NP + NW * 64 - 1) / (NW * 64);
    float4 v[NIT];
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int u = tid + NW * 64 * i;
      const int p = u / GPR, g = u - p * GPR;
      v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (u < NP && p < G::PIN && g < CG) {
        const int py = p / G::IW, px = p - py * G::IW;
        const int iy = iy0 + py, ix = ix0 + px;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) v[i] = *reinterpret_cast<const float4*>(Xb + ((size_t)iy * W + ix) * CIN + 4 * g);
      }
    }
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int u = tid + NW * 64 * i;
      if (u >= NP) break;
      const int p = u / GPR, g = u - p * GPR;
      if constexpr (EXPAND) {
        uint2 h, l;
        split4(v[i], h, l);
        *reinterpret_cast<uint2*>(Xh + p * G::XS + 4 * g) = h;
        *reinterpret_cast<uint2*>(Xl + p * G::XS + 4 * g) = l;
      } else {
        *reinterpret_cast<float4*>(Sl + p * G::SS + 4 * g) = v[i];
      }
    }
  }
  // expand validity: bit jj = pixel (wave + NW jj) * 16 + r16 of the input tile lies in the image (the depthwise's
  // zero padding applies to the hidden tensor, whose out-of-image values must be 0, not ReLU(bias))
  uint32_t pvmask = 0;
#pragma unroll
  for (int jj = 0; jj < G::EPT; ++jj) {
    const int p = (wave + NW * jj) * 16 + r16;
    if (p < G::PIN) {
      const int py = p / G::IW, px = p - py * G::IW;
      const int iy = iy0 + py, ix = ix0 + px;
      if (iy >= 0 && iy < H && ix >= 0 && ix < W) pvmask |= 1u << jj;
    }
  }

  const int wp = wave % G::WP, wc = wave / G::WP;
  f32x4 acc[G::QPW][G::NCTW];
#pragma unroll
  for (int t = 0; t < G::NCTW; ++t) {
    const float4 bb = *reinterpret_cast<const float4*>(bp + (wc * G::NCTW + t) * 16 + 4 * kg);
#pragma unroll
    for (int q = 0; q < G::QPW; ++q) acc[q][t] = f32x4{bb.x, bb.y, bb.z, bb.w};
  }
  constexpr int NPC = (G::NCT * 16);                   // project weight rows per plane
  const _Float16* WpLo = Wp + (size_t)NPC * G::HIDP;
  const _Float16* WeLo = We + (size_t)G::HIDP * G::CINP;

#pragma unroll 1
  for (int c = 0; c < G::NCH; ++c) {
    __syncthreads();   // c == 0: the staged tile; c > 0: every wave is done reading the slab of chunk c - 1
    if constexpr (EXPAND) {
      // ---- expand chunk c: hidden channels 32c + 16h + 4kg + r of input-tile pixel 16 pt + r16 -> slab
      f32x4 e[G::EPT][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 eb = *reinterpret_cast<const float4*>(be + 32 * c + 16 * h + 4 * kg);
#pragma unroll
        for (int jj = 0; jj < G::EPT; ++jj) e[jj][h] = f32x4{eb.x, eb.y, eb.z, eb.w};
      }
#pragma unroll
      for (int ks = 0; ks < G::KS; ++ks) {
        f16x8 ah[2], al[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const size_t off = (size_t)(32 * c + 16 * h + r16) * G::CINP + 32 * ks + 8 * kg;
          ah[h] = *reinterpret_cast<const f16x8*>(We + off);
          al[h] = *reinterpret_cast<const f16x8*>(WeLo + off);
        }
#pragma unroll
        for (int jj = 0; jj < G::EPT; ++jj) {
          const int pt = wave + NW * jj;
          if (pt >= G::PIN16) break;
          const int ro = (pt * 16 + r16) * G::XS + 32 * ks + 8 * kg;
          const f16x8 bh = *reinterpret_cast<const f16x8*>(Xh + ro);
          const f16x8 bl = *reinterpret_cast<const f16x8*>(Xl + ro);
#pragma unroll
          for (int h = 0; h < 2; ++h) e[jj][h] = mfma_x2(ah[h], al[h], bh, bl, e[jj][h]);
        }
      }
#pragma unroll
      for (int jj = 0; jj < G::EPT; ++jj) {
        const int pt = wave + NW * jj;
        if (pt >= G::PIN16) break;
        const bool ok = (pvmask >> jj) & 1u;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float4 o;
          o.x = ok ? fmaxf(e[jj][h][0], 0.f) : 0.f;
          o.y = ok ? fmaxf(e[jj][h][1], 0.f) : 0.f;
          o.z = ok ? fmaxf(e[jj][h][2], 0.f) : 0.f;
          o.w = ok ? fmaxf(e[jj][h][3], 0.f) : 0.f;
          *reinterpret_cast<float4*>(Sl + (pt * 16 + r16) * G::SS + 16 * h + 4 * kg) = o;
        }
      }
      __syncthreads();   // slab of chunk c complete
    }

    // ---- depthwise 3x3 (stride S, fp32, kx outer / ky inner) + BN + ReLU of this wave's output pixel tiles,
    // channels 32c + 8kg .. +7 -> hi / lo B fragments -> project accumulation
    float a[G::QPW][8];
    {
      const float4 d0 = *reinterpret_cast<const float4*>(bd + 32 * c + 8 * kg);
      const float4 d1 = *reinterpret_cast<const float4*>(bd + 32 * c + 8 * kg + 4);
#pragma unroll
      for (int q = 0; q < G::QPW; ++q) {
        a[q][0] = d0.x; a[q][1] = d0.y; a[q][2] = d0.z; a[q][3] = d0.w;
        a[q][4] = d1.x; a[q][5] = d1.y; a[q][6] = d1.z; a[q][7] = d1.w;
      }
    }
    int pbase[G::QPW];
#pragma unroll
    for (int q = 0; q < G::QPW; ++q) {
      const int o = (wp * G::QPW + q) * 16 + r16;
      const int oy = o / TW, ox = o - (o / TW) * TW;
      pbase[q] = (oy * S * G::IW + ox * S) * G::SS + 8 * kg;
    }
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const float* wt = Wd + (size_t)(ky * 3 + kx) * G::HIDP + 32 * c + 8 * kg;
        const float4 w0 = *reinterpret_cast<const float4*>(wt), w1 = *reinterpret_cast<const float4*>(wt + 4);
        const float w8[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
        for (int q = 0; q < G::QPW; ++q) {
          const float* sp = Sl + pbase[q] + (ky * G::IW + kx) * G::SS;
          const float4 x0 = *reinterpret_cast<const float4*>(sp), x1 = *reinterpret_cast<const float4*>(sp + 4);
          const float x8[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) a[q][e] = fmaf(x8[e], w8[e], a[q][e]);
        }
      }
    f16x8 bh[G::QPW], bl[G::QPW];
#pragma unroll
    for (int q = 0; q < G::QPW; ++q) {
#pragma unroll
      for (int e = 0; e < 8; ++e) a[q][e] = fmaxf(a[q][e], 0.f);
      split8(a[q], bh[q], bl[q]);
    }
#pragma unroll
    for (int t = 0; t < G::NCTW; ++t) {
      const size_t off = (size_t)((wc * G::NCTW + t) * 16 + r16) * G::HIDP + 32 * c + 8 * kg;
      const f16x8 ph = *reinterpret_cast<const f16x8*>(Wp + off);
      const f16x8 pl = *reinterpret_cast<const f16x8*>(WpLo + off);
#pragma unroll
      for (int q = 0; q < G::QPW; ++q) acc[q][t] = mfma_x2(ph, pl, bh[q], bl[q], acc[q][t]);
    }
  }

  // ---- epilogue: + residual (fp32 block input, pytorch_layers.py:93-96, added after the BN bias) -> fp32 NHWC
#pragma unroll
  for (int q = 0; q < G::QPW; ++q) {
    const int o = (wp * G::QPW + q) * 16 + r16;
    const int oy = o / TW, ox = o - (o / TW) * TW;
    const int gy = oy0 + oy, gx = ox0 + ox;
    if (gy >= OH || gx >= OW) continue;
    const size_t pix = ((size_t)b * OH + gy) * OW + gx;
#pragma unroll
    for (int t = 0; t < G::NCTW; ++t) {
      const int co = (wc * G::NCTW + t) * 16 + 4 * kg;
      if (co >= COUT) continue;
      f32x4 v = acc[q][t];
      if constexpr (RES) {
        const float4 r = *reinterpret_cast<const float4*>(X + pix * CIN + co);
        v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
      }
      *reinterpret_cast<float4*>(Y + pix * COUT + co) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

// (cin, hidden, cout, stride, expand, residual, TH, TW, waves, cout groups): MobileNet-V2's 17 blocks
// (mobilenet_v2.py:240-249). Tiles keep the LDS (hi / lo input tile + fp32 slab) at 2+ workgroups per CU where the
// geometry allows.
#define SPEF_X2_TABLE(X)                                   \
  X(32, 32, 16, 1, false, false, 16, 16, 4, 1)   /* 1 */   \
  X(16, 96, 24, 2, true, false, 8, 8, 4, 1)      /* 2 */   \
  X(24, 144, 24, 1, true, true, 8, 16, 4, 1)     /* 3 */   \
  X(24, 144, 32, 2, true, false, 8, 8, 4, 1)     /* 4 */   \
  X(32, 192, 32, 1, true, true, 8, 16, 4, 1)     /* 5-6 */ \
  X(32, 192, 64, 2, true, false, 8, 8, 4, 1)     /* 7 */   \
  X(64, 384, 64, 1, true, true, 8, 8, 4, 1)      /* 8-10 */ \
  X(64, 384, 96, 1, true, false, 8, 8, 4, 2)     /* 11 */  \
  X(96, 576, 96, 1, true, true, 8, 8, 4, 2)      /* 12-13 */ \
  X(96, 576, 160, 2, true, false, 4, 8, 2, 2)    /* 14 */  \
  X(160, 960, 160, 1, true, true, 8, 8, 4, 2)    /* 15-16 */ \
  X(160, 960, 320, 1, true, false, 8, 8, 4, 4)   /* 17 */

template <int CIN, int HID, int COUT, int S, bool EXPAND, bool RES, int TH, int TW, int NW, int WCO>
static hipError_t x2_irb_go(const void* x, const void* we, const float* be, const float* wd, const float* bd,
                            const void* wp, const float* bp, void* y, int B, int H, int W, int OH, int OW,
                            hipStream_t s) {
  using G = X2Geom<CIN, HID, COUT, S, TH, TW, EXPAND, NW, WCO>;
  const int tiles_x = (OW + TW - 1) / TW, tiles_y = (OH + TH - 1) / TH;
  const int64_t nwg64 = (int64_t)tiles_x * tiles_y * B;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  auto k = x2_irb_kernel<CIN, HID, COUT, S, TH, TW, EXPAND, RES, NW, WCO>;
  static bool attr_set = false;   // > 64 KiB dynamic LDS needs the attribute (once per instantiation)
  if (!attr_set && G::LDS_BYTES > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  k<<<nwg, NW * 64, G::LDS_BYTES, s>>>((const float*)x, (const _Float16*)we, be, wd, bd, (const _Float16*)wp, bp,
                                      (float*)y, H, W, OH, OW, tiles_x, tiles_y, nwg);
  return hipGetLastError();
}

bool x2_irb_supported(int cin, int hid, int cout, int stride, bool expand, bool res) {
#define SPEF_X2_HAS(CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_) \
  if (cin == CI && hid == HI && cout == CO && stride == ST && expand == EX && res == RS) return true;
  SPEF_X2_TABLE(SPEF_X2_HAS)
#undef SPEF_X2_HAS
  return false;
}

hipError_t launch_x2_irb(int cin, int hid, int cout, int stride, bool expand, bool res, const void* x, const void* we,
                         const float* be, const float* wd, const float* bd, const void* wp, const float* bp, void* y,
                         int B, int H, int W, int OH, int OW, hipStream_t s) {
#define SPEF_X2_CASE(CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_)                                          \
  if (cin == CI && hid == HI && cout == CO && stride == ST && expand == EX && res == RS)                  \
    return x2_irb_go<CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_>(x, we, be, wd, bd, wp, bp, y, B, H, W, OH, OW, s);
  SPEF_X2_TABLE(SPEF_X2_CASE)
#undef SPEF_X2_CASE
  return hipErrorNotSupported;
}

// ------------------------------------------------------------------------------------------ 1x1 conv, fp32 I/O
// C^T = W X^T as pw_kernel: a wave owns NT output-channel tiles x MT pixel tiles; 4 waves on 64 MT consecutive
// pixels; channel chunks fastest-varying so one pixel block's chunks share an XCD L2. B fragments: 8 fp32 values
// per lane from HBM / L2, split once and used by all NT channel tiles.
template <int NT, int MT>
__global__ __launch_bounds__(256) void x2_pw_kernel(const float* __restrict__ X, const _Float16* __restrict__ Wt,
                                                    const float* __restrict__ bias, float* __restrict__ Y, int64_t M,
                                                    int K, int N, int Np, int Kp, int n_chunks, uint32_t nwg) {
  const uint32_t L = xcd_remap(blockIdx.x, nwg);
  const int chunk = (int)(L % (uint32_t)n_chunks);
  const int64_t ptile = L / (uint32_t)n_chunks;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  const int n0 = chunk * 16 * NT;
  const int64_t m0 = ptile * (64 * MT) + (int64_t)wave * 16 * MT;
  const _Float16* Wlo = Wt + (size_t)Np * Kp;
  f32x4 acc[NT][MT];
#pragma unroll
  for (int a = 0; a < NT; ++a) {
    const float4 bb = *reinterpret_cast<const float4*>(bias + n0 + 16 * a + 4 * kg);
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[a][m] = f32x4{bb.x, bb.y, bb.z, bb.w};
  }
  const float* xp[MT];
  bool mv[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int64_t p = m0 + 16 * m + r16;
    mv[m] = p < M;
    xp[m] = X + (size_t)(mv[m] ? p : 0) * K + 8 * kg;
  }
#pragma unroll 1
  for (int k0 = 0; k0 < Kp; k0 += 32) {
    const bool kv = k0 + 8 * kg < K;   // K % 8 == 0: a lane's 8 k are all in range or all out
    f16x8 bh[MT], bl[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (kv && mv[m]) {
        const float4 u0 = *reinterpret_cast<const float4*>(xp[m] + k0);
        const float4 u1 = *reinterpret_cast<const float4*>(xp[m] + k0 + 4);
        v[0] = u0.x; v[1] = u0.y; v[2] = u0.z; v[3] = u0.w; v[4] = u1.x; v[5] = u1.y; v[6] = u1.z; v[7] = u1.w;
      }
      split8(v, bh[m], bl[m]);
    }
#pragma unroll
    for (int a = 0; a < NT; ++a) {
      const size_t off = (size_t)(n0 + 16 * a + r16) * Kp + k0 + 8 * kg;
      const f16x8 ah = *reinterpret_cast<const f16x8*>(Wt + off);
      const f16x8 al = *reinterpret_cast<const f16x8*>(Wlo + off);
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[a][m] = mfma_x2(ah, al, bh[m], bl[m], acc[a][m]);
    }
  }
#pragma unroll
  for (int a = 0; a < NT; ++a) {
    const int i = n0 + 16 * a + 4 * kg;
    if (i >= N) continue;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int64_t p = m0 + 16 * m + r16;
      if (p >= M) continue;
      const f32x4 v = acc[a][m];
      *reinterpret_cast<float4*>(Y + (size_t)p * N + i) =
          make_float4(fmaxf(v[0], 0.f), fmaxf(v[1], 0.f), fmaxf(v[2], 0.f), fmaxf(v[3], 0.f));
    }
  }
}

hipError_t launch_x2_pw_relu(const void* x, const void* wt, const float* bias, float* y, int64_t M, int K, int N,
                             hipStream_t s) {
  if (M <= 0) return hipSuccess;
  const int Kp = (K + 31) & ~31, Np = (N + 15) & ~15;
  if ((K & 7) || (N & 3) || Np % 64) return hipErrorInvalidValue;
  constexpr int NT = 4, MT = 4;
  const int n_chunks = Np / (16 * NT);
  const int64_t nwg64 = (M + 64 * MT - 1) / (64 * MT) * n_chunks;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  x2_pw_kernel<NT, MT><<<nwg, 256, 0, s>>>((const float*)x, (const _Float16*)wt, bias, y, M, K, N, Np, Kp, n_chunks,
                                           nwg);
  return hipGetLastError();
}

}  // namespace spef
