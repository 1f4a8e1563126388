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
//   x2_irb_kernel  one InvertedResidual (pytorch_layers.py:65-98) per kernel (high-resolution blocks 1-7): each wave
//                  loads the fp32 input pixels of its expand tiles once and keeps them split (hi / lo B fragments) in
//                  registers; per 32-channel hidden chunk the expand (3 MFMAs per K step) writes ReLU(x We^T + be) as
//                  fp32 into an LDS slab; the depthwise 3x3 runs in fp32 (v_fma_f32 chains, kx-outer / ky-inner, weights
//                  staged in LDS once) on the slab, its ReLU'd output is split into hi / lo project B fragments in
//                  registers; the project accumulates over chunks in fp32 MFMA accumulators; + residual (fp32, read
//                  back from L2) -> fp32 block output. Block 1 (t = 1) stages its input straight into the slab.
//   x2_irw_kernel  the same block, role-split into expand and depthwise/project waves with LDS-staged weights (blocks
//                  8-17, below).
//   x2_pw_kernel   1x1 conv on fp32 activations (the last ConvBnAct 320 -> 1280, mobilenet_v2.py:264): B fragments
//                  split on load, ReLU, fp32 output (the keypoint head's flatten input or the URSONet mean's).
//
// Block I/O is fp32 NHWC; weights come from the blob split by the packer (spef_amd/blob.py, dtype fp16x2).
#include <type_traits>

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
// lo halves of a pair: fp16(a - hi.x), fp16(b - hi.y), each ONE v_fma_mix{lo,hi}_f16 (the difference is formed
// exactly and rounded once, the same value as split8's fp32 residual + convert, which takes 1.5 ops per value)
__device__ __forceinline__ uint32_t lo_pair(uint32_t hi2, float a, float b) {
  uint32_t r;
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(r) : "v"(hi2), "v"(a), "v"(b));
  return r;
}
// ReLU + hi / lo split of 8 fp32 values: 8 v_max + 4 v_cvt_pk + 8 v_fma_mix (bit-identical to max + split8)
__device__ __forceinline__ void relu_split8(const f32x2 v[4], f16x8& hi, f16x8& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = fmaxf(v[i].x, 0.f), b = fmaxf(v[i].y, 0.f);
    h[i] = pack_h2((_Float16)a, (_Float16)b);
    l[i] = lo_pair(h[i], a, b);
  }
  hi = __builtin_bit_cast(f16x8, make_uint4(h[0], h[1], h[2], h[3]));
  lo = __builtin_bit_cast(f16x8, make_uint4(l[0], l[1], l[2], l[3]));
}
// acc += (a_hi + a_lo)(b_hi + b_lo) without the lo*lo term
__device__ __forceinline__ f32x4 mfma_x2(f16x8 ah, f16x8 al, f16x8 bh, f16x8 bl, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc, 0, 0, 0);
}
// acc += (a_hi + a_lo) b for an operand b that is exact in fp16 (fp16-stored activations: the fp16mx schedule)
__device__ __forceinline__ f32x4 mfma_x2w(f16x8 ah, f16x8 al, f16x8 b, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, b, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(al, b, acc, 0, 0, 0);
}
// depthwise tap on 8 channels as 4 v_pk_fma_f32 (each channel's fma in the same order as scalar fmaf chains)
__device__ __forceinline__ void dw_tap8(f32x2 a[4], float4 x0, float4 x1, const f32x2 w[4]) {
  a[0] = __builtin_elementwise_fma(f32x2{x0.x, x0.y}, w[0], a[0]);
  a[1] = __builtin_elementwise_fma(f32x2{x0.z, x0.w}, w[1], a[1]);
  a[2] = __builtin_elementwise_fma(f32x2{x1.x, x1.y}, w[2], a[2]);
  a[3] = __builtin_elementwise_fma(f32x2{x1.z, x1.w}, w[3], a[3]);
}
// block I/O element types (IO template bits): fp32, or fp16 where the fp16mx schedule stores a block output in fp16
constexpr int IO_IN16 = 1, IO_OUT16 = 2;
__device__ __forceinline__ float4 ld_act4(const void* p, size_t i, bool f16) {   // 4 channels at element i
  if (f16) {
    const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const _Float16*>(p) + i);
    return make_float4(h_lo(u.x), h_hi(u.x), h_lo(u.y), h_hi(u.y));
  }
  return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + i);
}
__device__ __forceinline__ void st_act4(void* p, size_t i, f32x4 v, bool f16) {
  if (f16)
    *reinterpret_cast<uint2*>(reinterpret_cast<_Float16*>(p) + i) =
        make_uint2(pack_h2((_Float16)v[0], (_Float16)v[1]), pack_h2((_Float16)v[2], (_Float16)v[3]));
  else
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(p) + i) = make_float4(v[0], v[1], v[2], v[3]);
}

// Hidden-chunk slab in LDS (fp32): two planes per 32-channel chunk, plane h holding channels 8k + 4h .. 8k + 4h + 3
// (k = 0..3) of every tile pixel as one 16-B granule each. A depthwise lane (pixel r16, channels 8kg .. 8kg + 7)
// reads granule kg of its pixel row in plane 0 and in plane 1; an expand lane writes the float4 of channels
// 16h + 4kg .. +3 (plane kg & 1, granule 2h + kg / 2). Row strides from the ds_read_b128 lane groups of
// MI355X_MICROARCH.md (LDS): 24 floats make the 16 consecutive rows of a 16-wide stride-1 pixel tile conflict-free
// (2-way on 8-wide tiles), 20 floats the stride-2 rows; the plane-1 base is offset to keep the expand's mixed-plane
// stores conflict-free.
template <int S, int PINP>
struct X2Slab {
  static constexpr int SSP = S == 2 ? 20 : 24;                   // floats per pixel row of a plane
  static constexpr int TGT = S == 2 ? 0 : 1;                     // plane-1 base, granules mod 16
  static constexpr int PLANE = PINP * SSP + ((TGT - PINP * SSP / 4) % 16 + 16) % 16 * 4;
  static constexpr int FLOATS = 2 * PLANE;
  static __device__ __forceinline__ int at(int p, int c4) {      // float offset of channels 4 c4 .. 4 c4 + 3 of pixel p
    return (c4 & 1) * PLANE + p * SSP + 4 * (c4 >> 1);
  }
};

// Geometry. Output tile TH x TW, NW waves; the depthwise/project phase gives wave w the output pixel tiles of group
// w % WP and the output-channel tiles of group w / WP (WCO groups; WCO > 1 repeats the depthwise to cut accumulators).
#ifndef SPEF_X2_RES_AHEAD   // persistent tiles: chunks before a tile's end at which its residual is fetched (4: no gain)
#define SPEF_X2_RES_AHEAD 2
#endif
#ifndef SPEF_X2_ROWS0   // slab kernels: input rows shared between a wave's vertically adjacent pixel tiles
#define SPEF_X2_ROWS0 1   // interleaved A/B, bit-identical: blocks 5-6 117.8 -> 111.0 us per step
#endif
template <int CIN, int HID, int COUT, int S, int TH, int TW, bool EXPAND, int NW, int WCO>
struct X2Geom {
  static constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3;
  static constexpr int PIN = IH * IW, PIN16 = (PIN + 15) / 16, PINP = PIN16 * 16;
  static constexpr int CINP = (CIN + 31) / 32 * 32;   // K of the expand (blob rows padded to 32, zeros)
  static constexpr int KS = CINP / 32;
  using SL = X2Slab<S, PINP>;
  static constexpr int NCH = (HID + 31) / 32, HIDP = NCH * 32;
  static constexpr int NCT = (COUT + 15) / 16;
  static constexpr int POUT16 = TH * TW / 16;
  static constexpr int WP = NW / WCO, QPW = POUT16 / WP, NCTW = NCT / WCO;
  static constexpr int EPT = (PIN16 + NW - 1) / NW;   // expand pixel tiles per wave
  static constexpr int DWS = 11 * HIDP;               // staged floats: depthwise [9][HIDP], bias, expand bias
  static constexpr int TRASH = EXPAND ? 16 * 24 : 0;   // dummy rows: expand stores of invalid input-tile pixels
  static constexpr int LDS_BYTES = (SL::FLOATS + DWS + TRASH) * 4;
  // waves per SIMD the LDS allows (workgroups per CU x NW / 4 SIMDs): the VGPR budget is held to it, so registers never
  // cost occupancy (the 8-wave 16 x 16 tiles: 2 workgroups per CU = 4 waves per SIMD = 128 VGPRs)
  static constexpr int WAVES_PER_EU = (163840 / LDS_BYTES) * NW / 4 > 8 ? 8 : (163840 / LDS_BYTES) * NW / 4;
  static_assert(CIN % 8 == 0 && COUT % 4 == 0 && HID % 8 == 0, "channel counts");
  static_assert(EXPAND || (CIN == HID && CIN == 32), "t == 1 blocks stage their 32-channel input as the hidden slab");
  static_assert(TH * TW % 16 == 0 && POUT16 % WP == 0 && NW % WCO == 0 && NCT % WCO == 0, "tile split");
  static_assert(EPT <= 32, "validity mask is 32 bits");
  static_assert(LDS_BYTES <= 163840, "LDS budget");
};

// IO: IO_IN16 = fp16 block input (the fp16mx schedule's early block outputs; the expand's B operand is then exact
// in fp16, two MFMAs per product), IO_OUT16 = fp16 block output. VALU per hidden value (the slab kernels are
// VALU-issue bound): the expand epilogue is one v_max (invalid input-tile pixels -- the
// depthwise's zero padding -- keep the zeros stored once at the start: their lanes store into a dummy LDS row), the
// depthwise 4.5 v_pk_fma_f32 per 9 taps, ReLU + split 1.5 (v_cvt_pk + v_fma_mix{lo,hi}). Each channel's fma chain is
// the same as with scalar fmaf, so the IO = 0 results equal the previous form bit for bit.
template <int CIN, int HID, int COUT, int S, int TH, int TW, bool EXPAND, bool RES, int NW, int WCO, int IO = 0>
__global__ __launch_bounds__(NW * 64) __attribute__((
    amdgpu_waves_per_eu(X2Geom<CIN, HID, COUT, S, TH, TW, EXPAND, NW, WCO>::WAVES_PER_EU))) void x2_irb_kernel(
    const void* __restrict__ X, const _Float16* __restrict__ We, const float* __restrict__ be,
    const float* __restrict__ Wd, const float* __restrict__ bd, const _Float16* __restrict__ Wp,
    const float* __restrict__ bp, void* __restrict__ Y, int H, int W, int OH, int OW, int tiles_x, int tiles_y,
    uint32_t nwg) {
  using G = X2Geom<CIN, HID, COUT, S, TH, TW, EXPAND, NW, WCO>;
  using SL = typename G::SL;
  constexpr bool IN16 = (IO & IO_IN16) != 0, OUT16 = (IO & IO_OUT16) != 0;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Sl = reinterpret_cast<float*>(smem);          // hidden chunk slab (plane layout)
  float* Ds = Sl + SL::FLOATS;                          // [9][HIDP] depthwise weights, [HIDP] bias, [HIDP] expand bias

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  uint32_t L = xcd_remap(blockIdx.x, nwg);
  const int tx = (int)(L % (uint32_t)tiles_x);
  L /= (uint32_t)tiles_x;
  const int ty = (int)(L % (uint32_t)tiles_y);
  const int b = (int)(L / (uint32_t)tiles_y);
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
  const size_t xb = (size_t)b * H * W * CIN;            // element offset of this image's input

  // ---- 1. staging: depthwise weights + biases of every chunk (LDS, once per workgroup); the input tile: B fragments
  // of this wave's expand pixel tiles pt = wave + NW j (fp32 input: hi / lo, split once; fp16 input: as loaded), in
  // registers for every chunk, or for t = 1 the tile itself as the slab. All global loads are issued before the first
  // LDS store.
  constexpr int NBX = EXPAND ? G::EPT : 1;
  f16x8 bxh[NBX][G::KS], bxl[IN16 ? 1 : NBX][G::KS];
  uint32_t pvmask = 0;
  int soff[NBX];                                        // slab store offset of this lane's pixel (h = 0), or Tr
  {
    constexpr int NDP = G::DWS / 4;                       // float4 pieces of the depthwise stage
    constexpr int NTP = EXPAND ? 0 : G::PINP * 8;         // t = 1: float4 pieces of the 32-channel input tile
    constexpr int NIT = (NDP + NTP + NW * 64 - 1) / (NW * 64);
    float4 v[NIT];
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      int u = tid + NW * 64 * i;
      v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (u < NDP) {
        const int part = u / (G::HIDP / 4), g = u - part * (G::HIDP / 4);
        if (part < 10 || EXPAND)                          // t = 1: no be
          v[i] = *reinterpret_cast<const float4*>((part < 9 ? Wd + (size_t)part * G::HIDP : part == 9 ? bd : be) + 4 * g);
      } else if ((u -= NDP) < NTP) {
        const int p = u >> 3, g = u & 7;
        if (p < G::PIN) {
          const int py = p / G::IW, px = p - py * G::IW;
          const int iy = iy0 + py, ix = ix0 + px;
          if (iy >= 0 && iy < H && ix >= 0 && ix < W) v[i] = ld_act4(X, xb + ((size_t)iy * W + ix) * CIN + 4 * g, IN16);
        }
      }
    }
    if constexpr (EXPAND) {
      uint4 raw[G::EPT][G::KS][IN16 ? 1 : 2];
#pragma unroll
      for (int j = 0; j < G::EPT; ++j) {
        const int p = (wave + NW * j) * 16 + r16;
        bool ok = false;
        int iy = 0, ix = 0;
        if (p < G::PIN) {
          const int py = p / G::IW, px = p - py * G::IW;
          iy = iy0 + py;
          ix = ix0 + px;
          ok = iy >= 0 && iy < H && ix >= 0 && ix < W;
        }
        if (ok) pvmask |= 1u << j;
        soff[j] = ok ? SL::at(p, kg) : SL::FLOATS + G::DWS + r16 * 24 + 4 * kg;
#pragma unroll
        for (int ks = 0; ks < G::KS; ++ks) {
          const int ch = 32 * ks + 8 * kg;
#pragma unroll
          for (int u = 0; u < (IN16 ? 1 : 2); ++u) raw[j][ks][u] = make_uint4(0u, 0u, 0u, 0u);
          if (ok && ch < CIN) {
            const size_t e0 = xb + ((size_t)iy * W + ix) * CIN + ch;
            if constexpr (IN16) {
              raw[j][ks][0] = *reinterpret_cast<const uint4*>(reinterpret_cast<const _Float16*>(X) + e0);
            } else {
              raw[j][ks][0] = *reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(X) + e0);
              raw[j][ks][1] = *reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(X) + e0 + 4);
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < G::EPT; ++j)
#pragma unroll
        for (int ks = 0; ks < G::KS; ++ks) {
          if constexpr (IN16) {
            bxh[j][ks] = __builtin_bit_cast(f16x8, raw[j][ks][0]);
          } else {
            const float4 a = __builtin_bit_cast(float4, raw[j][ks][0]), c = __builtin_bit_cast(float4, raw[j][ks][1]);
            const float v8[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
            split8(v8, bxh[j][ks], bxl[j][ks]);
          }
        }
      // invalid pixels (outside the image: the depthwise's zero padding) hold zeros for every chunk: stored once here,
      // never overwritten (their lanes' expand stores go to the dummy row)
#pragma unroll
      for (int j = 0; j < G::EPT; ++j) {
        const int pt = wave + NW * j;
        // (tiles past PIN16: the dummy tiles below, nothing to zero)
        if (pt < G::PIN16 && !((pvmask >> j) & 1u)) {
          const int p = pt * 16 + r16;
#pragma unroll
          for (int h = 0; h < 2; ++h)
            *reinterpret_cast<float4*>(Sl + SL::at(p, kg) + 8 * h) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      int u = tid + NW * 64 * i;
      if (u < NDP) {
        *reinterpret_cast<float4*>(Ds + 4 * u) = v[i];
      } else if ((u -= NDP) < NTP) {
        *reinterpret_cast<float4*>(Sl + SL::at(u >> 3, u & 7)) = v[i];
      }
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
  constexpr int NPC = G::NCT * 16;                      // project weight rows per plane
  const _Float16* WpLo = Wp + (size_t)NPC * G::HIDP;
  const _Float16* WeLo = We + (size_t)G::HIDP * G::CINP;
  // weight fragments of the chunk being computed, from L2; the next chunk's are issued right after their last use
  f16x8 eah[EXPAND ? 2 : 1][G::KS], eal[EXPAND ? 2 : 1][G::KS], pah[G::NCTW], pal[G::NCTW];
  auto load_ea = [&](int k) {
    if constexpr (EXPAND) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int ks = 0; ks < G::KS; ++ks) {
          const size_t off = (size_t)(32 * k + 16 * h + r16) * G::CINP + 32 * ks + 8 * kg;
          eah[h][ks] = *reinterpret_cast<const f16x8*>(We + off);
          eal[h][ks] = *reinterpret_cast<const f16x8*>(WeLo + off);
        }
    }
  };
  auto load_pa = [&](int k) {
#pragma unroll
    for (int t = 0; t < G::NCTW; ++t) {
      const size_t off = (size_t)((wc * G::NCTW + t) * 16 + r16) * G::HIDP + 32 * k + 8 * kg;
      pah[t] = *reinterpret_cast<const f16x8*>(Wp + off);
      pal[t] = *reinterpret_cast<const f16x8*>(WpLo + off);
    }
  };
  load_ea(0);
  load_pa(0);
  int pbase[G::QPW];
#pragma unroll
  for (int q = 0; q < G::QPW; ++q) {
    const int o = (wp * G::QPW + q) * 16 + r16;
    const int oy = o / TW, ox = o - (o / TW) * TW;
    pbase[q] = oy * S * G::IW + ox * S;
  }

#pragma unroll 1
  for (int c = 0; c < G::NCH; ++c) {
    __syncthreads();   // c == 0: the staged depthwise weights / t = 1 tile; c > 0: the slab of chunk c - 1 is consumed
    if constexpr (EXPAND) {
      // ---- expand chunk c: hidden channels 32c + 16h + 4kg + r of input-tile pixel 16 pt + r16 -> slab
      f32x4 e[G::EPT][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 eb = *reinterpret_cast<const float4*>(Ds + 10 * G::HIDP + 32 * c + 16 * h + 4 * kg);
#pragma unroll
        for (int j = 0; j < G::EPT; ++j) e[j][h] = f32x4{eb.x, eb.y, eb.z, eb.w};
      }
#pragma unroll
      for (int ks = 0; ks < G::KS; ++ks)
#pragma unroll
        for (int j = 0; j < G::EPT; ++j) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            if constexpr (IN16)
              e[j][h] = mfma_x2w(eah[h][ks], eal[h][ks], bxh[j][ks], e[j][h]);
            else
              e[j][h] = mfma_x2(eah[h][ks], eal[h][ks], bxh[j][ks], bxl[IN16 ? 0 : j][ks], e[j][h]);
          }
        }
      if (c + 1 < G::NCH) load_ea(c + 1);
#pragma unroll
      for (int j = 0; j < G::EPT; ++j) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 o = make_float4(fmaxf(e[j][h][0], 0.f), fmaxf(e[j][h][1], 0.f), fmaxf(e[j][h][2], 0.f),
                                       fmaxf(e[j][h][3], 0.f));
          *reinterpret_cast<float4*>(Sl + soff[j] + 8 * h) = o;
        }
      }
      __syncthreads();   // slab of chunk c complete
    }

    // ---- depthwise 3x3 (stride S, fp32, kx outer / ky inner) + BN + ReLU of this wave's output pixel tiles,
    // channels 32c + 8kg .. +7 -> hi / lo B fragments -> project accumulation
    f32x2 a[G::QPW][4];
    {
      const float4 d0 = *reinterpret_cast<const float4*>(Ds + 9 * G::HIDP + 32 * c + 8 * kg);
      const float4 d1 = *reinterpret_cast<const float4*>(Ds + 9 * G::HIDP + 32 * c + 8 * kg + 4);
#pragma unroll
      for (int q = 0; q < G::QPW; ++q) {
        a[q][0] = f32x2{d0.x, d0.y}; a[q][1] = f32x2{d0.z, d0.w};
        a[q][2] = f32x2{d1.x, d1.y}; a[q][3] = f32x2{d1.z, d1.w};
      }
    }
    // (blocks 5-6 only: block 3's 16 x 16 form, capped at 128 VGPRs for four waves per SIMD, spilled 30-44 VGPRs
    // with it and ran 184 -> 374 us per step in the fp16x2 schedule)
    if constexpr (SPEF_X2_ROWS0 && S == 1 && TW == 16 && G::QPW > 1 && NW == 4 && EXPAND && CIN >= 32) {
      // a wave's pixel tiles are consecutive output rows: per column, QPW + 2 input rows read once (tap (ky, q) is
      // row q + ky); same FMA order as below
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        float4 wv3[3][2], sr[G::QPW + 2][2];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const float* wt = Ds + (ky * 3 + kx) * G::HIDP + 32 * c + 8 * kg;
          wv3[ky][0] = *reinterpret_cast<const float4*>(wt);
          wv3[ky][1] = *reinterpret_cast<const float4*>(wt + 4);
        }
#pragma unroll
        for (int r = 0; r < G::QPW + 2; ++r) {
          const int p = pbase[0] + r * G::IW + kx;
          sr[r][0] = *reinterpret_cast<const float4*>(Sl + SL::at(p, 2 * kg));
          sr[r][1] = *reinterpret_cast<const float4*>(Sl + SL::at(p, 2 * kg + 1));
        }
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const float4 w0 = wv3[ky][0], w1 = wv3[ky][1];
          const f32x2 w4[4] = {f32x2{w0.x, w0.y}, f32x2{w0.z, w0.w}, f32x2{w1.x, w1.y}, f32x2{w1.z, w1.w}};
#pragma unroll
          for (int q = 0; q < G::QPW; ++q) dw_tap8(a[q], sr[q + ky][0], sr[q + ky][1], w4);
        }
      }
    } else {
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const float* wt = Ds + (ky * 3 + kx) * G::HIDP + 32 * c + 8 * kg;
        const float4 w0 = *reinterpret_cast<const float4*>(wt), w1 = *reinterpret_cast<const float4*>(wt + 4);
        const f32x2 w4[4] = {f32x2{w0.x, w0.y}, f32x2{w0.z, w0.w}, f32x2{w1.x, w1.y}, f32x2{w1.z, w1.w}};
#pragma unroll
        for (int q = 0; q < G::QPW; ++q) {
          const int p = pbase[q] + ky * G::IW + kx;
          dw_tap8(a[q], *reinterpret_cast<const float4*>(Sl + SL::at(p, 2 * kg)),
                  *reinterpret_cast<const float4*>(Sl + SL::at(p, 2 * kg + 1)), w4);
        }
      }
    }
    f16x8 bh[G::QPW], bl[G::QPW];
#pragma unroll
    for (int q = 0; q < G::QPW; ++q) relu_split8(a[q], bh[q], bl[q]);
#pragma unroll
    for (int t = 0; t < G::NCTW; ++t)
#pragma unroll
      for (int q = 0; q < G::QPW; ++q) acc[q][t] = mfma_x2(pah[t], pal[t], bh[q], bl[q], acc[q][t]);
    if (c + 1 < G::NCH) load_pa(c + 1);
  }

  // ---- epilogue: + residual (the block input, pytorch_layers.py:93-96, added after the BN bias) -> NHWC
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
        const float4 r = ld_act4(X, pix * CIN + co, IN16);
        v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
      }
      st_act4(Y, pix * COUT + co, v, OUT16);
    }
  }
}

// ------------------------------------------------------------------------------------------ role-split form
// The low-resolution blocks (8-17: 32x32 and 16x16 maps at 512^2, 256-1024 tiles for 256 CUs, 12-30 hidden chunks)
// are bound by how fast a workgroup streams the chunk weights, not by arithmetic: every chunk needs its expand and
// project weights (hi + lo, 20 KB each for 160 -> 960 -> 160) from L2 at ~29 B/clk per CU, and a lone workgroup per
// CU exposes every round trip. Here 8 waves take fixed roles in a two-stage pipeline with ONE barrier per chunk:
//
//   expand waves [0, 4): stage the weights of chunks c+1 / c+2 (global -> registers -> LDS, once per workgroup) and
//                        expand chunk c+1 into slab (c+1) & 1; their input-tile B fragments (hi + lo) are loaded and
//                        split once and stay in registers for every chunk (no input tile in LDS)
//   depthwise waves [4, 8): depthwise of chunk c from slab c & 1 + project accumulation (weights from the LDS stage)
//
// Stage buffers (double-buffered, written one iteration before use): expand weights + expand bias of chunk k in
// iteration k - 2, depthwise weights + bias and project weights of chunk k in iteration k - 1. Same arithmetic and
// rounding as x2_irb_kernel (bit-identical results).
#ifndef SPEF_X2_STAMP   // timing builds only (outputs overwritten): s_memtime stamps per chunk of one workgroup
#define SPEF_X2_STAMP 0
#endif
#ifndef SPEF_X2_GLDS   // stage the role-split kernels' chunk weights by LDS-DMA (global_load_lds) instead of registers
#define SPEF_X2_GLDS 1
#endif
#ifndef SPEF_X2_GLDS_S2   // ... on block 14 (stride 2) too
#define SPEF_X2_GLDS_S2 1
#endif
template <int CIN, int HID, int COUT, int S, int TH, int TW, int WCO, bool PST, int P = 1>
struct X2wGeom {
  static constexpr int NE = 4, ND = 4, NW = NE + ND;
  static constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3;
  static constexpr int PIN = IH * IW, PIN16 = (PIN + 15) / 16, PINP = PIN16 * 16;
  static constexpr int CINP = (CIN + 31) / 32 * 32, KS = CINP / 32;
  static constexpr int WES = CINP + 16;                 // staged expand row (halves): 2 mod 4 granules
  static constexpr int WPS = 48;                        // staged project row (halves, 32 used)
  using SL = X2Slab<S, PINP>;
  static constexpr int NCH = (HID + 31) / 32, HIDP = NCH * 32;
  static constexpr int NCL = NCH / P;                   // chunks of this workgroup's hidden part
  static constexpr int NCT = (COUT + 15) / 16, NPC = NCT * 16;
  static constexpr int POUT16 = TH * TW / 16;
  static constexpr int WP = ND / WCO, QPW = POUT16 / WP, NCTW = NCT / WCO;
  static constexpr int EPT = (PIN16 + NE - 1) / NE;     // expand pixel tiles per expand wave
  // LDS: slabs | expand stage [2] | depthwise stage [2] | project stage [2]
  static constexpr int SLAB_B = SL::FLOATS * 4;
  static constexpr int SE_B = 2 * 32 * WES * 2 + 32 * 4;   // hi / lo weight planes + expand bias
  static constexpr int SD_B = (9 * 32 + 32) * 4;        // depthwise weights [9][32] + depthwise bias
  static constexpr int SP_B = PST ? 2 * NPC * WPS * 2 : 0;
  // LDS-DMA staging (GL): every stage region a whole number of 1-KiB wave-instruction pieces (a piece writes 64 x 16 B
  // lane-linearly); per buffer the depthwise and project stages are one contiguous region. Interleaved A/B at B = 64:
  // blocks 14 and 15-16 -2 / -5 us per step, block 17 +3, blocks 8-13 no gain (same box, interleaved), so the
  // cout = 160 blocks only.
  static constexpr bool GL = SPEF_X2_GLDS && COUT == 160 && (S == 1 || SPEF_X2_GLDS_S2);
  static constexpr int SE_BQ = (SE_B + 1023) / 1024 * 1024, SD_BQ = (SD_B + 1023) / 1024 * 1024;
  static constexpr int SP_BQ = (SP_B + 1023) / 1024 * 1024, DP_BQ = SD_BQ + SP_BQ;
  static constexpr int NIE = SE_BQ / 1024, NID = DP_BQ / 1024;                  // pieces per chunk stage
  static constexpr int IEW = (NIE + NE - 1) / NE, IDW = (NID + ND - 1) / ND;    // pieces per wave
  static constexpr int SE_STR = GL ? SE_BQ : SE_B, SD_STR = GL ? DP_BQ : SD_B, SP_STR = GL ? DP_BQ : SP_B;
  static constexpr int OFF_SE = 2 * SLAB_B;
  static constexpr int OFF_SD = GL ? OFF_SE + 2 * SE_BQ : OFF_SE + 2 * SE_B;
  static constexpr int OFF_SP = GL ? OFF_SD + SD_BQ : OFF_SD + 2 * SD_B;
  static constexpr int OFF_TR = GL ? OFF_SD + 2 * DP_BQ : OFF_SP + 2 * SP_B;   // dummy rows: invalid pixels' stores
  static constexpr int OFF_ST = OFF_TR + 16 * 24 * 4;     // SPEF_X2_STAMP: per-chunk clock stamps
  static constexpr int LDS_BYTES = OFF_ST + (SPEF_X2_STAMP ? 8 * 4 * 64 : 0);
  // 16-B stage pieces per chunk
  static constexpr int NPE = 2 * 32 * (CINP / 8) + 8, NPD = 9 * 8 + 8, NPP = PST ? 2 * NPC * 4 : 0;
  static constexpr int NPIECE = (NPE + NPD + NPP + NE * 64 - 1) / (NE * 64);
  static_assert(CIN % 8 == 0 && COUT % 4 == 0 && HID % 8 == 0, "channel counts");
  static_assert(TH * TW % 16 == 0 && POUT16 % WP == 0 && ND % WCO == 0 && NCT % WCO == 0, "tile split");
  static_assert(EPT <= 32 && NCH % P == 0 && NCL >= 2, "validity mask / hidden parts / pipeline depth");
  static_assert(SE_B % 16 == 0 && SD_B % 16 == 0 && SP_B % 16 == 0 && SLAB_B % 16 == 0, "16-B aligned stages");
  static_assert(LDS_BYTES <= 163840, "LDS budget");
};

// P > 1 (hidden split): the P workgroups of a tile each run NCH / P consecutive hidden chunks and store their
// project partial sums (no bias, no residual) to Y + part * pstride; x2_split_reduce_kernel adds the P parts in order,
// the bias and the residual. Small maps get P times the workgroups while every workgroup streams only 1 / P of the
// block's weights.
// PT (persistent tiles): a workgroup runs tiles L, L + nwg, ... < ntile as ONE chunk stream (global chunk g = tile
// t * NCL + chunk c): the expand waves fetch the next tile's input two chunks ahead and expand its chunk 0 while the
// depthwise waves finish the current tile (residual fetched two chunks ahead, epilogue stores issued, accumulators
// reset), so a second tile per CU costs no prologue, epilogue or dispatch gap. Invalid input pixels are stored as
// zeros by every expand (a pixel valid in one tile may be padding in the next). NCL even: the stage / slab parity of
// global chunk g is that of its chunk c.
// Interleaved A/B at B = 64 (bit-identical): the occupancy target alone blocks 15-16 140 -> 139 us per step; with
// column batches one column ahead 140 -> 133, block 14 69 -> 66, blocks 8-13 unchanged (their expand role bounds the
// chunk period); 53.2k -> 53.5k img/s.
#ifndef SPEF_X2_DWB   // role-split depthwise: 0 = tap by tap, 1 = column batches, 2 = column batches one column ahead
#define SPEF_X2_DWB 2
#endif
#ifndef SPEF_X2_ROWS   // column batches share input rows between a wave's vertically adjacent pixel tiles
#define SPEF_X2_ROWS 1
#endif
// DWB 2 on two-pixel-tile waves up to this block input width. Without ROWS blocks 12-13 spilled at 96 and blocks 8-10
// measured 143.6 -> 145.4 us per step at 64; with ROWS (4 row reads per column instead of 6, interleaved A/B,
// bit-identical): blocks 12-13 161.6 -> 149.8, 8-10 141.7 -> 137.8, 11 53.0 -> 50.7 us per step.
#ifndef SPEF_X2_DWB2_CIN
#define SPEF_X2_DWB2_CIN 96
#endif
// occupancy target: one 8-wave workgroup per CU = 2 waves per SIMD (the VGPR budget is held to it)
// Roles by SIMD pair (PAIR, block 17: project fragments from L2, two cout groups): a workgroup's waves go to SIMDs in the
// cyclic order 0 -> 2 -> 1 -> 3 from a varying start (MI355X_MICROARCH.md, LDS), so waves {0, 1, 4, 5} (expand) share
// two SIMDs and {2, 3, 6, 7} (depthwise / project) the other two, and the two roles' MFMAs no longer share a SIMD's
// matrix pipe. Interleaved A/B at B = 64 (bit-identical): block 17 109.5 -> 102.6 us per step; blocks 8-16 slower
// (8-10 131.8 -> 146.5, 12-13 149.7 -> 168.2, 15-16 132.8 -> 136.0), so they keep waves 0-3 expand, 4-7 depthwise.
template <int CIN, int HID, int COUT, int S, int TH, int TW, bool RES, int WCO, bool PST, int P = 1, bool PT = false>
__global__ __launch_bounds__(8 * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void x2_irw_kernel(
    const float* __restrict__ X, const _Float16* __restrict__ We, const float* __restrict__ be,
    const float* __restrict__ Wd, const float* __restrict__ bd, const _Float16* __restrict__ Wp,
    const float* __restrict__ bp, float* __restrict__ Y, int H, int W, int OH, int OW, int tiles_x, int tiles_y,
    uint32_t nwg, size_t pstride, uint32_t ntile) {
  using G = X2wGeom<CIN, HID, COUT, S, TH, TW, WCO, PST, P>;
  using SL = typename G::SL;
  static_assert(!PT || (P == 1 && G::NCL % 2 == 0), "persistent tiles: one hidden part, even chunk count");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  uint32_t L = xcd_remap(blockIdx.x, nwg);
  const bool stamp_wg = SPEF_X2_STAMP && L == 0;   // the workgroup of tile 0 (its output holds the stamps)
  auto stamp = [&](int c, int slot) {              // lane 0 of waves 0 / 4: shader clock into LDS slot (c, slot)
    if constexpr (SPEF_X2_STAMP) {
      if (stamp_wg && lane == 0 && c < 64)
        reinterpret_cast<uint32_t*>(smem + G::OFF_ST)[c * 8 + slot] = (uint32_t)__builtin_amdgcn_s_memtime();
    }
  };
  const uint32_t L0 = L;                           // first work item (PT: then L0 + nwg, ...)
  const int nt = PT ? (int)((ntile - L0 + nwg - 1) / nwg) : 1;   // tiles of this workgroup
  const int GT = nt * G::NCL;                      // chunks of this workgroup
  const int part = (int)(L % (uint32_t)P);        // hidden part (the parts of a tile share an XCD)
  L /= (uint32_t)P;
  const int cb = part * G::NCL;                    // first hidden chunk of this part
  auto tile_of = [&](uint32_t Lt, int& b_, int& oy0_, int& ox0_) {   // tile (without the part) -> image, origin
    const int tx_ = (int)(Lt % (uint32_t)tiles_x);
    Lt /= (uint32_t)tiles_x;
    b_ = (int)(Lt / (uint32_t)tiles_y);
    oy0_ = (int)(Lt % (uint32_t)tiles_y) * TH;
    ox0_ = tx_ * TW;
  };
  int b, oy0, ox0;
  tile_of(L, b, oy0, ox0);
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
  // local chunk of global chunk g (G::NCL: none, past this workgroup's last tile)
  auto kmod = [&](int g) { return PT ? (g < GT ? g % G::NCL : G::NCL) : g; };
  auto slab = [&](int i) { return reinterpret_cast<float*>(smem + i * G::SLAB_B); };
  if (wave == 0) stamp(0, 3);                      // kernel entry (expand wave 0)
  auto se = [&](int i) { return smem + G::OFF_SE + i * G::SE_STR; };
  auto sd = [&](int i) { return reinterpret_cast<float*>(smem + G::OFF_SD + i * G::SD_STR); };
  auto sp = [&](int i) { return reinterpret_cast<_Float16*>(smem + G::OFF_SP + i * G::SP_STR); };

  // 16-B stage piece u of chunk k: kind 0 = expand (weights + bias, chunk ke), 1 = depthwise (chunk kd),
  // 2 = project (chunk kd). Source / destination pointers; null source = nothing to stage (chunk out of range).
  auto piece = [&](int u, int ke, int kd, const void*& src, void*& dst) {
    src = nullptr;
    dst = nullptr;
    if (u < G::NPE) {
      if (ke >= G::NCL) return;
      if (u < G::NPE - 8) {
        constexpr int PPR = G::CINP / 8;
        const int pl = u / (32 * PPR), rr = (u / PPR) % 32, g = u % PPR;
        src = We + (size_t)pl * G::HIDP * G::CINP + (size_t)(32 * (cb + ke) + rr) * G::CINP + 8 * g;
        dst = se(ke & 1) + ((pl * 32 + rr) * G::WES + 8 * g) * 2;
      } else {
        const int g = u - (G::NPE - 8);
        src = be + 32 * (cb + ke) + 4 * g;
        dst = se(ke & 1) + 2 * 32 * G::WES * 2 + 16 * g;
      }
      return;
    }
    u -= G::NPE;
    if (u < G::NPD) {
      if (kd >= G::NCL) return;
      if (u < 72) {
        const int tap = u >> 3, g = u & 7;
        src = Wd + (size_t)tap * G::HIDP + 32 * (cb + kd) + 4 * g;
        dst = sd(kd & 1) + tap * 32 + 4 * g;
      } else {
        src = bd + 32 * (cb + kd) + 4 * (u - 72);
        dst = sd(kd & 1) + 288 + 4 * (u - 72);
      }
      return;
    }
    u -= G::NPD;
    if (PST && u < G::NPP) {
      if (kd >= G::NCL) return;
      const int pl = u / (G::NPC * 4), rr = (u >> 2) % G::NPC, q = u & 3;
      src = Wp + (size_t)pl * G::NPC * G::HIDP + (size_t)rr * G::HIDP + 32 * (cb + kd) + 8 * q;
      dst = sp(kd & 1) + (pl * G::NPC + rr) * G::WPS + 8 * q;
    }
  };

  // ---- LDS-DMA stage pieces (G::GL). Expand waves: pieces e + NE j of the expand stage (weights hi / lo + bias); depthwise
  // waves: pieces d + ND j of the depthwise + project stage. Lane l of piece i fills LDS slot 64 i + l of the region
  // from a source whose address at chunk k is src0 + k * kstr (pad slots read a valid address of the same tensor).
  constexpr bool PAIR = !PST;
  const bool ewave = PAIR ? ((wave >> 1) & 1) == 0 : wave < G::NE;
  const int wr = PAIR ? (wave & 1) | ((wave >> 2) << 1) : ewave ? wave : wave - G::NE;   // index within the role
  if (!ewave && wr == 0) stamp(1, 7);              // kernel entry (depthwise wave 0)
  constexpr int NJ = G::GL ? (G::IEW > G::IDW ? G::IEW : G::IDW) : 1;
  const char* gsrc[NJ];
  int kstr[NJ];
#pragma unroll
  for (int j = 0; j < (G::GL ? NJ : 0); ++j) {
    const int off = ((ewave ? wr + G::NE * j : wr + G::ND * j) * 64 + lane) * 16;   // byte offset in the region
    const char* src;
    int ks;
    if (ewave) {
      constexpr int EW_B = 2 * 32 * G::WES * 2, ROW_B = G::WES * 2;
      if (off < EW_B) {
        const int pl = off / (32 * ROW_B), rem = off - pl * (32 * ROW_B), rr = rem / ROW_B;
        const int col = (rem - rr * ROW_B) / 16;
        src = reinterpret_cast<const char*>(We + (size_t)pl * G::HIDP * G::CINP + (size_t)(32 * cb + rr) * G::CINP +
                                            (col < G::CINP / 8 ? 8 * col : 0));
        ks = 32 * G::CINP * 2;
      } else {
        const int g = (off - EW_B) / 16;
        src = reinterpret_cast<const char*>(be + 32 * cb + (g < 8 ? 4 * g : 0));
        ks = 128;
      }
    } else {
      if (off < G::SD_BQ) {
        if (off < 1152) {
          src = reinterpret_cast<const char*>(Wd + (size_t)(off / 128) * G::HIDP + 32 * cb + 4 * ((off % 128) / 16));
        } else {
          const int g = (off - 1152) / 16;
          src = reinterpret_cast<const char*>(bd + 32 * cb + (g < 8 ? 4 * g : 0));
        }
        ks = 128;
      } else {
        const int o2 = off - G::SD_BQ;
        constexpr int ROW_B = G::WPS * 2;
        const int pl = o2 / (G::NPC * ROW_B), rem = o2 - pl * (G::NPC * ROW_B), rr = rem / ROW_B;
        const int q = (rem - rr * ROW_B) / 16;
        const bool ok = PST && o2 < G::SP_B;
        src = reinterpret_cast<const char*>(Wp + (ok ? (size_t)pl * G::NPC * G::HIDP + (size_t)rr * G::HIDP : 0) + 32 * cb +
                                            (ok && q < 4 ? 8 * q : 0));
        ks = 64;
      }
    }
    gsrc[j] = src;
    kstr[j] = ks;
  }
  // issue this wave's pieces of chunk k's stage (expand waves: the expand stage; depthwise waves: depthwise + project)
  auto dma = [&](int k) {
    if constexpr (!G::GL) return;
    char* base = ewave ? smem + G::OFF_SE + (k & 1) * G::SE_STR : smem + G::OFF_SD + (k & 1) * G::SD_STR;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int i = ewave ? wr + G::NE * j : wr + G::ND * j;
      if ((ewave && j < G::IEW && i < G::NIE) || (!ewave && j < G::IDW && i < G::NID))
        __builtin_amdgcn_global_load_lds((const void*)(gsrc[j] + (size_t)k * kstr[j]),
                                         (__attribute__((address_space(3))) void*)(base + i * 1024), 16, 0, 0);
    }
  };
  if constexpr (G::GL) {
    if (ewave) {
      dma(0);
      dma(1);
    } else {
      dma(0);
    }
  } else {
  // ---- prologue (all waves): expand stages of chunks 0 and 1, depthwise / project stage of chunk 0
    constexpr int NP0 = 2 * G::NPE + G::NPD + G::NPP;
    constexpr int NIT = (NP0 + G::NW * 64 - 1) / (G::NW * 64);
    uint4 v[NIT];
    void* dst[NIT];
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      int u = tid + G::NW * 64 * i;
      const void* src = nullptr;
      dst[i] = nullptr;
      if (u < G::NPE) piece(u, 1, G::NCL, src, dst[i]);                     // expand chunk 1
      else if (u < NP0) piece(u - G::NPE, 0, 0, src, dst[i]);               // expand / dw / project chunk 0
      v[i] = src ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NIT; ++i)
      if (dst[i]) *reinterpret_cast<uint4*>(dst[i]) = v[i];
  }

  if (ewave) {
    // ================= expand waves
    const int e = wr;
    // this wave's input-tile pixel tiles pt = e + NE j: B fragments (hi / lo) for every K step, loaded and split once
    // per tile. The fp32 rows are loaded into the fragments' own registers (8 floats of (j, ks) in the bits of
    // bxh[j][ks] | bxl[j][ks]) and split in place: no second register set
    f16x8 bxh[G::EPT][G::KS], bxl[G::EPT][G::KS];
    uint32_t pvmask = 0;   // bit j: pixel tile j's pixel of this lane is inside the map
    int soff[G::EPT];      // slab store offset (floats) of this lane's pixel, or the dummy rows
    auto pix = [&](int j, int iy0_, int ix0_, int& iy, int& ix) {   // input pixel of pixel tile j: inside the map?
      const int p = (e + G::NE * j) * 16 + r16;
      if (p >= G::PIN) return false;
      const int py = p / G::IW, px = p - py * G::IW;
      iy = iy0_ + py;
      ix = ix0_ + px;
      return iy >= 0 && iy < H && ix >= 0 && ix < W;
    };
    auto load_raw = [&](int b_, int iy0_, int ix0_) {   // fp32 input rows of the tile (zero outside the map)
      const float* Xb = X + (size_t)b_ * H * W * CIN;
#pragma unroll
      for (int j = 0; j < G::EPT; ++j) {
        int iy = 0, ix = 0;
        const bool ok = pix(j, iy0_, ix0_, iy, ix);
#pragma unroll
        for (int ks = 0; ks < G::KS; ++ks) {
          const int ch = 32 * ks + 8 * kg;
          float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0;
          if (ok && ch < CIN) {
            const float* src = Xb + ((size_t)iy * W + ix) * CIN + ch;
            r0 = *reinterpret_cast<const float4*>(src);
            r1 = *reinterpret_cast<const float4*>(src + 4);
          }
          bxh[j][ks] = __builtin_bit_cast(f16x8, r0);
          bxl[j][ks] = __builtin_bit_cast(f16x8, r1);
        }
      }
    };
    auto split_raw = [&]() {
#pragma unroll
      for (int j = 0; j < G::EPT; ++j)
#pragma unroll
        for (int ks = 0; ks < G::KS; ++ks) {
          const float4 a = __builtin_bit_cast(float4, bxh[j][ks]), c = __builtin_bit_cast(float4, bxl[j][ks]);
          const float v8[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
          split8(v8, bxh[j][ks], bxl[j][ks]);
        }
    };
    auto set_mask = [&](int iy0_, int ix0_) {   // PT: slab slots for every pixel of the tile (invalid ones get zeros)
      pvmask = 0;
#pragma unroll
      for (int j = 0; j < G::EPT; ++j) {
        const int p = (e + G::NE * j) * 16 + r16;
        int iy, ix;
        const bool ok = pix(j, iy0_, ix0_, iy, ix);
        if (ok) pvmask |= 1u << j;
        soff[j] = (PT ? p < G::PINP : ok) ? SL::at(p, kg) : G::OFF_TR / 4 + r16 * 24 + 4 * kg;
        if (!PT && !ok && p < G::PINP) {   // zero padding of the depthwise: both slabs, once
#pragma unroll
          for (int sb = 0; sb < 2; ++sb)
#pragma unroll
            for (int h = 0; h < 2; ++h)
              *reinterpret_cast<float4*>(slab(sb) + SL::at(p, kg) + 8 * h) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    };
    load_raw(b, iy0, ix0);
    set_mask(iy0, ix0);
    split_raw();
    if (wave == 0) stamp(1, 3);   // input fragments loaded and split
    // expand of chunk k into slab k & 1 (stage k & 1)
    auto expand = [&](int k) {
      const char* S0 = se(k & 1);
      const float* eb = reinterpret_cast<const float*>(S0 + 2 * 32 * G::WES * 2);
      f32x4 acc[G::EPT][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 bb = *reinterpret_cast<const float4*>(eb + 16 * h + 4 * kg);
#pragma unroll
        for (int j = 0; j < G::EPT; ++j) acc[j][h] = f32x4{bb.x, bb.y, bb.z, bb.w};
      }
      const _Float16* Ws = reinterpret_cast<const _Float16*>(S0);
#pragma unroll
      for (int ks = 0; ks < G::KS; ++ks) {
        f16x8 ah[2], al[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          ah[h] = *reinterpret_cast<const f16x8*>(Ws + (16 * h + r16) * G::WES + 32 * ks + 8 * kg);
          al[h] = *reinterpret_cast<const f16x8*>(Ws + (32 + 16 * h + r16) * G::WES + 32 * ks + 8 * kg);
        }
#pragma unroll
        for (int j = 0; j < G::EPT; ++j) {
#pragma unroll
          for (int h = 0; h < 2; ++h) acc[j][h] = mfma_x2(ah[h], al[h], bxh[j][ks], bxl[j][ks], acc[j][h]);
        }
      }
      // valid pixels -> slab k & 1; invalid ones -> the dummy rows (PT: zeros into their slab slots; slab offsets
      // are relative to slab 0, the dummy rows' to the LDS base, which is slab 0)
      float* Sl = reinterpret_cast<float*>(smem) + ((k & 1) ? G::SLAB_B / 4 : 0);
#pragma unroll
      for (int j = 0; j < G::EPT; ++j) {
        const bool pv = (pvmask >> j) & 1u;
        const int p = (e + G::NE * j) * 16 + r16;
        float* dst = (PT ? p < G::PINP : pv) ? Sl + soff[j] : reinterpret_cast<float*>(smem) + soff[j];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float4 v = make_float4(fmaxf(acc[j][h][0], 0.f), fmaxf(acc[j][h][1], 0.f), fmaxf(acc[j][h][2], 0.f),
                                 fmaxf(acc[j][h][3], 0.f));
          if (PT && !pv) v = make_float4(0.f, 0.f, 0.f, 0.f);
          *reinterpret_cast<float4*>(dst + 8 * h) = v;
        }
      }
    };
    // PT, around the expand of global chunk gn: after a tile's last expand its successor's rows are loaded into the
    // (now dead) fragment registers, after that iteration's stage loads so the stage stores' vmcnt waits do not cover
    // them; chunk 0 of the next tile splits them. (An L2 prefetch chunks earlier by LDS-DMA into the dummy rows made
    // the compiler wait vmcnt(0) at every barrier, which serialises the register-staged weight loads.)
    auto next_tile = [&](int gn) {   // before expand(gn)
      if constexpr (PT) {
        if (gn % G::NCL == 0) {
          int b_, oy_, ox_;
          tile_of(L0 + (uint32_t)(gn / G::NCL) * nwg, b_, oy_, ox_);
          set_mask(oy_ * S - 1, ox_ * S - 1);
          split_raw();
        }
      }
    };
    auto fetch_tile = [&](int gn) {   // after expand(gn)
      if constexpr (PT) {
        const int cn = gn % G::NCL, tn = gn / G::NCL + 1;
        if (tn < nt && cn == G::NCL - 1) {
          int b_, oy_, ox_;
          tile_of(L0 + (uint32_t)tn * nwg, b_, oy_, ox_);
          load_raw(b_, oy_ * S - 1, ox_ * S - 1);
        }
      }
    };
    // Stage data is loaded one iteration before it is stored: the pieces of expand chunk c + 2 and depthwise /
    // project chunk c + 1 are fetched in iteration c - 1 (a whole chunk period of L2 latency hidden) and written to
    // LDS at the start of iteration c (the same buffers and barriers as a load-and-store in iteration c).
    if constexpr (G::GL) {
    __syncthreads();                 // prologue stages landed (vmcnt(0) + barrier)
    expand(0);
    __syncthreads();                 // slab 0 visible
#pragma unroll 1
    for (int c = 0; c < GT; ++c) {
      if (wave == 0) stamp(c, 0);
      if (c + 2 < GT) dma(kmod(c + 2));   // expand stage of chunk c + 2 into the buffer chunk c's expand released
      if (c + 1 < GT) {
        next_tile(c + 1);
        expand(kmod(c + 1));
        fetch_tile(c + 1);
      }
      if (wave == 0) stamp(c, 1);
      __syncthreads();                  // (waits for this wave's pieces: visible to every wave after the barrier)
    }
    } else {
    uint4 v[G::NPIECE];
    auto load_stage = [&](int c) {
#pragma unroll
      for (int i = 0; i < G::NPIECE; ++i) {
        const void* src;
        void* dst;
        piece(e * 64 + lane + G::NE * 64 * i, kmod(c + 2), kmod(c + 1), src, dst);
        v[i] = src ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
      }
    };
    auto store_stage = [&](int c) {
#pragma unroll
      for (int i = 0; i < G::NPIECE; ++i) {
        const void* src;
        void* dst;
        piece(e * 64 + lane + G::NE * 64 * i, kmod(c + 2), kmod(c + 1), src, dst);
        if (src) *reinterpret_cast<uint4*>(dst) = v[i];
      }
    };
    load_stage(0);
    __syncthreads();                 // prologue stages visible
    expand(0);
    __syncthreads();                 // slab 0 visible
#pragma unroll 1
    for (int c = 0; c < GT; ++c) {
      if (wave == 0) stamp(c, 0);
      store_stage(c);                // expand chunk c + 2, depthwise / project chunk c + 1
      if (wave == 0) stamp(c, 2);
      if (c + 1 < GT) {
        load_stage(c + 1);
        next_tile(c + 1);
        expand(kmod(c + 1));
        fetch_tile(c + 1);
      }
      if (wave == 0) stamp(c, 1);
      __syncthreads();
    }
    }
  } else {
    // ================= depthwise / project waves
    const int d = wr;
    const int wp = d % G::WP, wc = d / G::WP;
    f32x4 acc[G::QPW][G::NCTW];
    auto init_acc = [&]() {
#pragma unroll
      for (int t = 0; t < G::NCTW; ++t) {   // (P > 1: the bias is added once, by the reduce)
        const float4 bb = P == 1 ? *reinterpret_cast<const float4*>(bp + (wc * G::NCTW + t) * 16 + 4 * kg)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < G::QPW; ++q) acc[q][t] = f32x4{bb.x, bb.y, bb.z, bb.w};
      }
    };
    init_acc();
    int pbase[G::QPW];
#pragma unroll
    for (int q = 0; q < G::QPW; ++q) {
      const int o = (wp * G::QPW + q) * 16 + r16;
      const int oy = o / TW, ox = o - (o / TW) * TW;
      pbase[q] = oy * S * G::IW + ox * S;
    }
    const _Float16* WpLo = Wp + (size_t)G::NPC * G::HIDP;
    f16x8 pgh[PST ? 1 : G::NCTW], pgl[PST ? 1 : G::NCTW];   // !PST: this chunk's project fragments from L2
    auto load_pg = [&](int k) {
      if constexpr (!PST) {
#pragma unroll
        for (int t = 0; t < G::NCTW; ++t) {
          const size_t off = (size_t)((wc * G::NCTW + t) * 16 + r16) * G::HIDP + 32 * (cb + k) + 8 * kg;
          pgh[t] = *reinterpret_cast<const f16x8*>(Wp + off);
          pgl[t] = *reinterpret_cast<const f16x8*>(WpLo + off);
        }
      }
    };
    // epilogue of the tile at (b_, oy0_, ox0_): + residual (the block input, pytorch_layers.py:93-96, added after the
    // BN bias; PT: fetched two chunks earlier into rres) -> fp32 NHWC
    constexpr int NRES = (PT && RES) ? G::QPW * G::NCTW : 1;
    float4 rres[NRES];
    auto out_pix = [&](int q, int b_, int oy0_, int ox0_, size_t& pix_) {
      const int o = (wp * G::QPW + q) * 16 + r16;
      const int oy = o / TW, ox = o - (o / TW) * TW;
      const int gy = oy0_ + oy, gx = ox0_ + ox;
      pix_ = ((size_t)b_ * OH + gy) * OW + gx;
      return gy < OH && gx < OW;
    };
    auto fetch_res = [&](int b_, int oy0_, int ox0_) {
      if constexpr (PT && RES) {
#pragma unroll
        for (int q = 0; q < G::QPW; ++q) {
          size_t pix_;
          const bool in = out_pix(q, b_, oy0_, ox0_, pix_);
#pragma unroll
          for (int t = 0; t < G::NCTW; ++t) {
            const int co = (wc * G::NCTW + t) * 16 + 4 * kg;
            rres[q * G::NCTW + t] = in && co < COUT ? *reinterpret_cast<const float4*>(X + pix_ * CIN + co)
                                                    : make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
      }
    };
    auto epilogue = [&](int b_, int oy0_, int ox0_) {
#pragma unroll
      for (int q = 0; q < G::QPW; ++q) {
        size_t pix;
        if (!out_pix(q, b_, oy0_, ox0_, pix)) continue;
#pragma unroll
        for (int t = 0; t < G::NCTW; ++t) {
          const int co = (wc * G::NCTW + t) * 16 + 4 * kg;
          if (co >= COUT) continue;
          f32x4 v = acc[q][t];
          if constexpr (P > 1) {   // partial sum of this hidden part
            *reinterpret_cast<float4*>(Y + part * pstride + pix * COUT + co) = make_float4(v[0], v[1], v[2], v[3]);
            continue;
          }
          if constexpr (RES) {
            const float4 r = PT ? rres[q * G::NCTW + t] : *reinterpret_cast<const float4*>(X + pix * CIN + co);
            v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
          }
          *reinterpret_cast<float4*>(Y + pix * COUT + co) = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
    };
    load_pg(0);
    __syncthreads();
    __syncthreads();
#pragma unroll 1
    for (int g = 0; g < GT; ++g) {
      const int c = kmod(g);
      if (wr == 0) stamp(g, 4);
      if constexpr (G::GL)
        if (g + 1 < GT) dma(kmod(g + 1));   // depthwise + project stage of chunk g + 1 (buffer released by g - 1)
      const float* Sl = slab(c & 1);
      const float* D = sd(c & 1);
      f32x2 a[G::QPW][4];
      {
        const float4 d0 = *reinterpret_cast<const float4*>(D + 288 + 8 * kg);
        const float4 d1 = *reinterpret_cast<const float4*>(D + 288 + 8 * kg + 4);
#pragma unroll
        for (int q = 0; q < G::QPW; ++q) {
          a[q][0] = f32x2{d0.x, d0.y}; a[q][1] = f32x2{d0.z, d0.w};
          a[q][2] = f32x2{d1.x, d1.y}; a[q][3] = f32x2{d1.z, d1.w};
        }
      }
      // (block 17, !PST: no registers to spare for the batches; DWB 2 only where a wave owns one pixel tile)
      constexpr int DWB = !PST ? 0 : (SPEF_X2_DWB == 2 && G::QPW > 1 && CIN > SPEF_X2_DWB2_CIN) ? 1 : SPEF_X2_DWB;
      if constexpr (DWB > 0) {
      // column batches: the 3 taps' weights and slab rows of column kx issued together (sched_barrier keeps them
      // ahead of the FMAs), DWB 2: column kx + 1's batch issued before column kx's FMAs. Same FMA order.
      // ROWS: a wave's pixel tiles are consecutive output rows (16-wide tiles, stride 1), so tap (ky, q) reads input
      // row q + ky of the column: QPW + 2 row reads per column instead of 3 QPW
      constexpr bool ROWS = SPEF_X2_ROWS && S == 1 && TW == 16 && G::QPW > 1;
      constexpr int NR = ROWS ? G::QPW + 2 : 3 * G::QPW;
      float4 wv[DWB][3][2], sr[DWB][NR][2];
      auto col = [&](int kx, int bf) {
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const float* wt = D + (ky * 3 + kx) * 32 + 8 * kg;
          wv[bf][ky][0] = *reinterpret_cast<const float4*>(wt);
          wv[bf][ky][1] = *reinterpret_cast<const float4*>(wt + 4);
        }
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int p = ROWS ? pbase[0] + r * G::IW + kx : pbase[r % G::QPW] + (r / G::QPW) * G::IW + kx;
          sr[bf][r][0] = *reinterpret_cast<const float4*>(Sl + SL::at(p, 2 * kg));
          sr[bf][r][1] = *reinterpret_cast<const float4*>(Sl + SL::at(p, 2 * kg + 1));
        }
      };
      col(0, 0);
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int bf = DWB == 2 ? (kx & 1) : 0;
        if (DWB == 2 && kx < 2) col(kx + 1, bf ^ 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const float4 w0 = wv[bf][ky][0], w1 = wv[bf][ky][1];
          const f32x2 w4[4] = {f32x2{w0.x, w0.y}, f32x2{w0.z, w0.w}, f32x2{w1.x, w1.y}, f32x2{w1.z, w1.w}};
#pragma unroll
          for (int q = 0; q < G::QPW; ++q) {
            const int r = ROWS ? q + ky : ky * G::QPW + q;
            dw_tap8(a[q], sr[bf][r][0], sr[bf][r][1], w4);
          }
        }
        if (DWB == 1 && kx < 2) {
          __builtin_amdgcn_sched_barrier(0);
          col(kx + 1, 0);
        }
      }
      } else {
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const float* wt = D + (ky * 3 + kx) * 32 + 8 * kg;
          const float4 w0 = *reinterpret_cast<const float4*>(wt), w1 = *reinterpret_cast<const float4*>(wt + 4);
          const f32x2 w4[4] = {f32x2{w0.x, w0.y}, f32x2{w0.z, w0.w}, f32x2{w1.x, w1.y}, f32x2{w1.z, w1.w}};
#pragma unroll
          for (int q = 0; q < G::QPW; ++q) {
            const int p = pbase[q] + ky * G::IW + kx;
            dw_tap8(a[q], *reinterpret_cast<const float4*>(Sl + SL::at(p, 2 * kg)),
                    *reinterpret_cast<const float4*>(Sl + SL::at(p, 2 * kg + 1)), w4);
          }
        }
      }
      f16x8 bh[G::QPW], bl[G::QPW];
#pragma unroll
      for (int q = 0; q < G::QPW; ++q) relu_split8(a[q], bh[q], bl[q]);
      if (wr == 0) stamp(g, 5);
      if constexpr (PST) {
        const _Float16* Ps = sp(c & 1);
#pragma unroll
        for (int t = 0; t < G::NCTW; ++t) {
          const int row = (wc * G::NCTW + t) * 16 + r16;
          const f16x8 ph = *reinterpret_cast<const f16x8*>(Ps + row * G::WPS + 8 * kg);
          const f16x8 pl = *reinterpret_cast<const f16x8*>(Ps + (G::NPC + row) * G::WPS + 8 * kg);
#pragma unroll
          for (int q = 0; q < G::QPW; ++q) acc[q][t] = mfma_x2(ph, pl, bh[q], bl[q], acc[q][t]);
        }
      } else {
#pragma unroll
        for (int t = 0; t < G::NCTW; ++t)
#pragma unroll
          for (int q = 0; q < G::QPW; ++q) acc[q][t] = mfma_x2(pgh[t], pgl[t], bh[q], bl[q], acc[q][t]);
        if (g + 1 < GT) load_pg(kmod(g + 1));   // next chunk's fragments: in flight across the barrier and its depthwise
      }
      if constexpr (PT) {
        if (c == G::NCL - SPEF_X2_RES_AHEAD || c == G::NCL - 1) {
          int b_, oy_, ox_;
          tile_of(L0 + (uint32_t)(g / G::NCL) * nwg, b_, oy_, ox_);
          if (c == G::NCL - SPEF_X2_RES_AHEAD) {
            fetch_res(b_, oy_, ox_);
          } else {
            // the next tile's bias loads go out before the epilogue's stores: vmcnt counts both in order, so a
            // wait for loads issued after the stores would wait for the stores too
            float4 bn[G::NCTW];
#pragma unroll
            for (int t = 0; t < G::NCTW; ++t)
              bn[t] = *reinterpret_cast<const float4*>(bp + (wc * G::NCTW + t) * 16 + 4 * kg);
            epilogue(b_, oy_, ox_);
#pragma unroll
            for (int t = 0; t < G::NCTW; ++t)
#pragma unroll
              for (int q = 0; q < G::QPW; ++q) acc[q][t] = f32x4{bn[t].x, bn[t].y, bn[t].z, bn[t].w};
          }
        }
      }
      if (wr == 0) stamp(g, 6);
      __syncthreads();
    }
    if constexpr (!PT) epilogue(b, oy0, ox0);
    if (wr == 0) stamp(0, 7);   // epilogue stores issued
  }
  if constexpr (SPEF_X2_STAMP) {   // every wave: the last barrier, then the stamps over the start of tile 0's output
    __syncthreads();
    if (stamp_wg && tid < 8 * 64) {
      const int n = 8 * (GT < 64 ? GT : 64);
      if (tid < n) reinterpret_cast<uint32_t*>(Y)[tid] = reinterpret_cast<const uint32_t*>(smem + G::OFF_ST)[tid];
    }
  }
}

// ------------------------------------------------------------------------------------------ three-stage form
// Blocks 15-16 (16x16 maps at 512^2: one 8x8 tile per CU, 30 hidden chunks), a three-stage pipeline with one barrier
// per chunk (the fp16 schedule's k_irp.hip structure with fp16x2 arithmetic):
//
//   MFMA waves [0, 4):  P(c-1)  project of chunk c - 1: B fragments (hi / lo depthwise outputs) from Ds[(c-1) & 1],
//                               A fragments from L2 (each wave its own output-channel tiles, one chunk ahead)
//                       E(c+1)  expand of chunk c + 1 into slab (c+1) & 1 (input fragments in registers, weights
//                               from the LDS stage that the same waves fill by LDS-DMA two chunks ahead)
//   VALU waves [4, 8):  V(c)    depthwise of chunk c from slab c & 1 (its weights by LDS-DMA one chunk ahead),
//                               ReLU, hi / lo split -> Ds[c & 1]
//
// Every double buffer is a separate static __shared__ array and the chunk loop is unrolled by two, so each LDS access
// names its buffer at compile time: the compiler's wait tracking (SIInsertWaitcnts, the LDS-DMA stores' alias scopes)
// then sees that a stage read does not alias the stage the same wave's LDS-DMA is filling, and does not drain vmcnt --
// i.e. the DMA just issued and the next project fragments -- before it (with one dynamic LDS array it waited there, and
// each chunk's 43 KB of weights were fetched synchronously: tools/kstamp_irp.py). The VALU waves hold no accumulators.
// Same operations per output, in the same order (fp32 depthwise kx outer / ky inner, relu_split8, three MFMAs per
// product accumulated over the chunks in order): bit-identical to the slab and role-split kernels. Ds: per buffer a hi
// and a lo plane of 64-B pixel rows (32 fp16 channels); granule kg of pixel p at position kg ^ (3 ((p >> 3) & 1)),
// conflict-free for the project's ds_read_b128 lane groups.
// Workgroup barrier for LDS hand-offs only: this wave's LDS stores complete, then s_barrier -- without the vmcnt(0)
// that __syncthreads() gets when an LDS-DMA is in flight, so global loads and DMA pieces that are consumed later stay
// in flight across it (the callers wait with counted vmcnt for the pieces other waves read next).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int CIN, int HID, int COUT, int S, int TH, int TW>
struct X2pGeom {
  static constexpr int NE = 4, ND = 4, NW = NE + ND;
  static constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3;
  static constexpr int PIN = IH * IW, PIN16 = (PIN + 15) / 16, PINP = PIN16 * 16;
  static constexpr int CINP = (CIN + 31) / 32 * 32, KS = CINP / 32;
  static constexpr int WES = CINP + 16;                 // staged expand row (halves)
  using SL = X2Slab<S, PINP>;
  static constexpr int NCH = (HID + 31) / 32, HIDP = NCH * 32;
  static constexpr int NCT = (COUT + 15) / 16, NPC = NCT * 16;
  static constexpr int POUT16 = TH * TW / 16, QPV = POUT16 / ND;
  // the VALU waves' depthwise pixel tiles are consecutive output rows (16-wide tiles, stride 1): a column's input rows
  // are read once for both (4 row reads per column instead of 6)
  static constexpr bool ROWS = S == 1 && TW == 16 && QPV == 2;
  static constexpr int NCTW = (NCT + NE - 1) / NE;      // project output-channel tiles per MFMA wave
  static constexpr int EPT = (PIN16 + NE - 1) / NE;     // expand pixel tiles per MFMA wave
  static constexpr int SE_B = 2 * 32 * WES * 2 + 32 * 4, SE_BQ = (SE_B + 1023) / 1024 * 1024;
  static constexpr int SD_B = (9 * 32 + 32) * 4, SD_BQ = (SD_B + 1023) / 1024 * 1024;
  static constexpr int DS_PL = POUT16 * 16 * 64;        // one Ds plane (bytes)
  static constexpr int NIE = SE_BQ / 1024, NID = SD_BQ / 1024;
  static constexpr int SLF = SL::FLOATS + 16 * 24;    // a slab + its dummy rows (invalid pixels' expand stores)
  // PAL: the project A fragments staged in LDS, each MFMA wave's own tiles (by its own LDS-DMA, one chunk ahead),
  // instead of registers held across the expand -- where those registers (8 per output-channel tile) would spill:
  // block 17 (5 tiles per wave) 244 VGPRs, no spill, 101.5 -> 67.3 us per step at B = 64 on this kernel (from the
  // role-split kernel; tools/ktime.sh, bit-identical); blocks 15-16 (3 tiles) 102 -> 105 us with it, so they keep
  // the registers. Block 14 (EPT 5: 120 registers of input fragments) spills either way and has no LDS left for it.
  static constexpr int LDS_BASE = 2 * SLF * 4 + 2 * SE_BQ + 2 * SD_BQ + 4 * DS_PL;
  static constexpr bool PAL = NCTW >= 4 && POUT16 <= 4 && LDS_BASE + NE * NCTW * 2048 <= 163840;
  static constexpr int SP_B = PAL ? NE * NCTW * 2048 : 0;
  static constexpr int LDS_BYTES = LDS_BASE + SP_B;
  static_assert(CIN % 8 == 0 && COUT % 16 == 0 && HID % 32 == 0, "channel counts");
  static_assert(TH * TW % 16 == 0 && POUT16 % ND == 0 && NCH >= 4 && NCH % 2 == 0, "tile split / pipeline depth");
  static_assert(EPT <= 32 && LDS_BYTES <= 163840, "validity mask / LDS budget");
};

// PT (persistent tiles, the maps with more tiles than CUs): a workgroup runs tiles L, L + nwg, ... < ntile as ONE
// stream of global chunks g = t NCH + c (NCH even, so the parity of g is that of c): the MFMA waves load the next tile's
// input rows into their fragment registers after its predecessor's last expand and split them before its first, and
// store a tile's outputs right after its last project; invalid input pixels are stored as zeros by every expand (a
// pixel valid in one tile may be padding in the next).
template <int CIN, int HID, int COUT, int S, int TH, int TW, bool RES, bool PT>
__global__ __launch_bounds__(8 * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void x2_irp_kernel(
    const float* __restrict__ X, const _Float16* __restrict__ We, const float* __restrict__ be,
    const float* __restrict__ Wd, const float* __restrict__ bd, const _Float16* __restrict__ Wp,
    const float* __restrict__ bp, float* __restrict__ Y, int H, int W, int OH, int OW, int tiles_x, int tiles_y,
    uint32_t nwg, uint32_t ntile) {
  using G = X2pGeom<CIN, HID, COUT, S, TH, TW>;
  using SL = typename G::SL;
  __shared__ __attribute__((aligned(16))) float Sl0[G::SLF], Sl1[G::SLF];   // hidden chunk slabs (fp32) + dummy rows
  __shared__ __attribute__((aligned(1024))) char Se0[G::SE_BQ], Se1[G::SE_BQ];       // expand stages
  __shared__ __attribute__((aligned(1024))) char Sd0[G::SD_BQ], Sd1[G::SD_BQ];       // depthwise stages
  __shared__ __attribute__((aligned(16))) char Ds0[2 * G::DS_PL], Ds1[2 * G::DS_PL]; // depthwise outputs hi | lo
  __shared__ __attribute__((aligned(1024))) char Sp[G::PAL ? G::SP_B : 16];          // project A stage (PAL)
  __shared__ uint32_t Stamps[SPEF_X2_STAMP ? 8 * 64 : 1];
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  auto slab = [&](auto p) -> float* { if constexpr (decltype(p)::value) return Sl1; else return Sl0; };
  auto se = [&](auto p) -> char* { if constexpr (decltype(p)::value) return Se1; else return Se0; };
  auto sd = [&](auto p) -> char* { if constexpr (decltype(p)::value) return Sd1; else return Sd0; };
  auto dsb = [&](auto p) -> char* { if constexpr (decltype(p)::value) return Ds1; else return Ds0; };

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  const uint32_t L0 = xcd_remap(blockIdx.x, nwg);   // first tile (PT: then L0 + nwg, ...)
  const int nt = PT ? (int)((ntile - L0 + nwg - 1) / nwg) : 1;
  const int GT = nt * G::NCH;                        // global chunks of this workgroup
  auto kmod = [&](int g) { return PT ? g % G::NCH : g; };
  auto tile_of = [&](int t, int& b_, int& oy0_, int& ox0_) {
    uint32_t Lt = L0 + (uint32_t)t * nwg;
    const int tx_ = (int)(Lt % (uint32_t)tiles_x);
    Lt /= (uint32_t)tiles_x;
    b_ = (int)(Lt / (uint32_t)tiles_y);
    oy0_ = (int)(Lt % (uint32_t)tiles_y) * TH;
    ox0_ = tx_ * TW;
  };
  const int dsx = 16 * (kg ^ (3 * ((r16 >> 3) & 1)));                         // this lane's Ds granule (bytes)
  const bool stamp_wg = SPEF_X2_STAMP && blockIdx.x == 0;
  auto stamp = [&](int c, int slot) {   // timing builds (tools/kstamp_irp.py): lane 0's shader clock into slot (c, slot)
    if constexpr (SPEF_X2_STAMP) {
      if (stamp_wg && lane == 0 && c < 64) Stamps[c * 8 + slot] = (uint32_t)__builtin_amdgcn_s_memtime();
    }
  };
  if (wave == 0) stamp(0, 3);
  if (wave == G::NE) stamp(1, 7);

  // Stage pieces, all moved by LDS-DMA from the VALU waves (the MFMA waves' critical path then carries none of it): the
  // expand stage (weights hi / lo + bias, 1-KiB pieces d + ND j) and the depthwise stage (weights + bias); lane l of
  // piece i fills slot 64 i + l of the region from src0 + k * kstr at chunk k (pad slots read a valid address of the
  // same tensor). Measured per step at B = 64 (tools/ktime.sh): blocks 15-16 with the expand stage issued by the MFMA
  // waves 102.9 -> 116.6 us, register staging (global loads an iteration ahead + ds_write) instead of LDS-DMA 181 us.
  const bool ewave = wave < G::NE;
  const int wr = ewave ? wave : wave - G::NE;
  constexpr int NJE = (G::NIE + G::ND - 1) / G::ND, NJD = (G::NID + G::ND - 1) / G::ND;
  const char* esrc[NJE];
  const char* dsrc[NJD];
  int ekstr[NJE];
#pragma unroll
  for (int j = 0; j < NJE; ++j) {
    const int off = ((wr + G::ND * j) * 64 + lane) * 16;
    constexpr int EW_B = 2 * 32 * G::WES * 2, ROW_B = G::WES * 2;
    if (off < EW_B) {
      const int pl = off / (32 * ROW_B), rem = off - pl * (32 * ROW_B), rr = rem / ROW_B;
      const int col = (rem - rr * ROW_B) / 16;
      esrc[j] = reinterpret_cast<const char*>(We + (size_t)pl * G::HIDP * G::CINP + (size_t)rr * G::CINP +
                                              (col < G::CINP / 8 ? 8 * col : 0));
      ekstr[j] = 32 * G::CINP * 2;
    } else {
      const int g = (off - EW_B) / 16;
      esrc[j] = reinterpret_cast<const char*>(be + (g < 8 ? 4 * g : 0));
      ekstr[j] = 128;
    }
  }
#pragma unroll
  for (int j = 0; j < NJD; ++j) {
    const int off = ((wr + G::ND * j) * 64 + lane) * 16;
    dsrc[j] = off < 1152 ? reinterpret_cast<const char*>(Wd + (size_t)(off / 128) * G::HIDP + 4 * ((off % 128) / 16))
                         : reinterpret_cast<const char*>(bd + (off - 1152 < 128 ? 4 * ((off - 1152) / 16) : 0));
  }
  auto dma_e = [&](int k, char* base) {
#pragma unroll
    for (int j = 0; j < NJE; ++j)
      if (wr + G::ND * j < G::NIE)
        __builtin_amdgcn_global_load_lds((const void*)(esrc[j] + (size_t)k * ekstr[j]),
                                         (__attribute__((address_space(3))) void*)(base + (wr + G::ND * j) * 1024), 16,
                                         0, 0);
  };
  auto dma_d = [&](int k, char* base) {
#pragma unroll
    for (int j = 0; j < NJD; ++j)
      if (wr + G::ND * j < G::NID)
        __builtin_amdgcn_global_load_lds((const void*)(dsrc[j] + (size_t)k * 128),
                                         (__attribute__((address_space(3))) void*)(base + (wr + G::ND * j) * 1024), 16,
                                         0, 0);
  };
  if (!ewave) {
    dma_e(0, Se0);
    dma_e(1, Se1);
    dma_d(0, Sd0);
  }

  if (ewave) {
    // ================= MFMA waves: expand (pixel tiles e + NE j, both hidden halves) and project (output-channel tiles
    // e + NE t, every output pixel tile)
    const int e = wr;
    // input-tile B fragments (hi / lo) for every K step; the fp32 rows are loaded into the fragments' own registers (8
    // floats of (j, ks) in the bits of bxh[j][ks] | bxl[j][ks]) and split in place
    f16x8 bxh[G::EPT][G::KS], bxl[G::EPT][G::KS];
    uint32_t pvmask = 0;
    int soff[G::EPT];
    auto pix = [&](int j, int iy0_, int ix0_, int& iy, int& ix) {
      const int p = (e + G::NE * j) * 16 + r16;
      if (p >= G::PIN) return false;
      const int py = p / G::IW, px = p - py * G::IW;
      iy = iy0_ + py;
      ix = ix0_ + px;
      return iy >= 0 && iy < H && ix >= 0 && ix < W;
    };
    auto load_raw = [&](int t) {   // fp32 input rows of tile t (zero outside the map)
      int b_, oy_, ox_;
      tile_of(t, b_, oy_, ox_);
      const float* Xb = X + (size_t)b_ * H * W * CIN;
#pragma unroll
      for (int j = 0; j < G::EPT; ++j) {
        int iy = 0, ix = 0;
        const bool ok = e + G::NE * j < G::PIN16 && pix(j, oy_ * S - 1, ox_ * S - 1, iy, ix);
#pragma unroll
        for (int ks = 0; ks < G::KS; ++ks) {
          const int ch = 32 * ks + 8 * kg;
          float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0;
          if (ok && ch < CIN) {
            const float* src = Xb + ((size_t)iy * W + ix) * CIN + ch;
            r0 = *reinterpret_cast<const float4*>(src);
            r1 = *reinterpret_cast<const float4*>(src + 4);
          }
          bxh[j][ks] = __builtin_bit_cast(f16x8, r0);
          bxl[j][ks] = __builtin_bit_cast(f16x8, r1);
        }
      }
    };
    auto split_mask = [&](int t) {   // split tile t's loaded rows in place; slab slots / validity of its pixels
      int b_, oy_, ox_;
      tile_of(t, b_, oy_, ox_);
      pvmask = 0;
#pragma unroll
      for (int j = 0; j < G::EPT; ++j) {
        const int p = (e + G::NE * j) * 16 + r16;
        int iy, ix;
        const bool ok = pix(j, oy_ * S - 1, ox_ * S - 1, iy, ix);
        if (ok) pvmask |= 1u << j;
        // PT: every slot of the tile is stored by every expand (zeros where invalid); else invalid pixels hold the
        // zeros stored once below and their expand stores go to the dummy rows
        soff[j] = (PT ? p < G::PINP : ok) ? SL::at(p, kg) : SL::FLOATS + r16 * 24 + 4 * kg;
#pragma unroll
        for (int ks = 0; ks < G::KS; ++ks) {
          const float4 a = __builtin_bit_cast(float4, bxh[j][ks]), c = __builtin_bit_cast(float4, bxl[j][ks]);
          const float v8[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
          split8(v8, bxh[j][ks], bxl[j][ks]);
        }
        if (!PT && !ok && p < G::PINP) {   // the depthwise's zero padding: both slabs, once
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            *reinterpret_cast<float4*>(Sl0 + SL::at(p, kg) + 8 * h) = make_float4(0.f, 0.f, 0.f, 0.f);
            *reinterpret_cast<float4*>(Sl1 + SL::at(p, kg) + 8 * h) = make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
      }
    };
    load_raw(0);
    split_mask(0);
    // expand of a chunk: weights from stage `sp`, ReLU'd fp32 results into slab `sl`
    auto expand = [&](const char* sp, float* sl) {
      const float* eb = reinterpret_cast<const float*>(sp + 2 * 32 * G::WES * 2);
      f32x4 acc[G::EPT][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 bb = *reinterpret_cast<const float4*>(eb + 16 * h + 4 * kg);
#pragma unroll
        for (int j = 0; j < G::EPT; ++j) acc[j][h] = f32x4{bb.x, bb.y, bb.z, bb.w};
      }
      const _Float16* Ws = reinterpret_cast<const _Float16*>(sp);
#pragma unroll
      for (int ks = 0; ks < G::KS; ++ks) {
        f16x8 ah[2], al[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          ah[h] = *reinterpret_cast<const f16x8*>(Ws + (16 * h + r16) * G::WES + 32 * ks + 8 * kg);
          al[h] = *reinterpret_cast<const f16x8*>(Ws + (32 + 16 * h + r16) * G::WES + 32 * ks + 8 * kg);
        }
#pragma unroll
        for (int j = 0; j < G::EPT; ++j) {
          if (e + G::NE * j >= G::PIN16) continue;   // (wave-uniform)
#pragma unroll
          for (int h = 0; h < 2; ++h) acc[j][h] = mfma_x2(ah[h], al[h], bxh[j][ks], bxl[j][ks], acc[j][h]);
        }
      }
#pragma unroll
      for (int j = 0; j < G::EPT; ++j) {
        if (e + G::NE * j >= G::PIN16) continue;
        const bool pv = (pvmask >> j) & 1u;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float4 v = make_float4(fmaxf(acc[j][h][0], 0.f), fmaxf(acc[j][h][1], 0.f), fmaxf(acc[j][h][2], 0.f),
                                 fmaxf(acc[j][h][3], 0.f));
          if (PT && !pv) v = make_float4(0.f, 0.f, 0.f, 0.f);
          *reinterpret_cast<float4*>(sl + soff[j] + 8 * h) = v;
        }
      }
    };
    // project: accumulators (bias) of this wave's output-channel tiles, A fragments of chunk k from L2
    f32x4 acc[G::POUT16][G::NCTW];
    auto init_acc = [&]() {
#pragma unroll
      for (int t = 0; t < G::NCTW; ++t) {
        float4 bb = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e + G::NE * t < G::NCT) bb = *reinterpret_cast<const float4*>(bp + (e + G::NE * t) * 16 + 4 * kg);
#pragma unroll
        for (int q = 0; q < G::POUT16; ++q) acc[q][t] = f32x4{bb.x, bb.y, bb.z, bb.w};
      }
    };
    init_acc();
    const _Float16* WpLo = Wp + (size_t)G::NPC * G::HIDP;
    f16x8 pah[G::NCTW], pal[G::NCTW];
    char* const spw = Sp + wr * (G::NCTW * 2048);   // PAL: this wave's A stage (tile t: hi at 2048 t, lo + 1024)
    auto load_pa = [&](int k) {
#pragma unroll
      for (int t = 0; t < G::NCTW; ++t)
        if (e + G::NE * t < G::NCT) {
          const size_t off = (size_t)((e + G::NE * t) * 16 + r16) * G::HIDP + 32 * k + 8 * kg;
          if constexpr (G::PAL) {
            __builtin_amdgcn_global_load_lds((const void*)(Wp + off),
                                             (__attribute__((address_space(3))) void*)(spw + t * 2048), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void*)(WpLo + off),
                                             (__attribute__((address_space(3))) void*)(spw + t * 2048 + 1024), 16, 0,
                                             0);
          } else {
            pah[t] = *reinterpret_cast<const f16x8*>(Wp + off);
            pal[t] = *reinterpret_cast<const f16x8*>(WpLo + off);
          }
        }
    };
    // the B fragments of pixel tile q + 1 are read before tile q's MFMAs (each read pair's LDS latency hides behind
    // the previous tile's MFMAs instead of stalling the MFMA role)
    auto project = [&](const char* Dh) {
      if constexpr (G::PAL) {   // all pixel tiles' B fragments, then output-channel tile by tile (its A from the stage)
        f16x8 bh[G::POUT16], bl[G::POUT16];
#pragma unroll
        for (int q = 0; q < G::POUT16; ++q) {
          bh[q] = *reinterpret_cast<const f16x8*>(Dh + (q * 16 + r16) * 64 + dsx);
          bl[q] = *reinterpret_cast<const f16x8*>(Dh + G::DS_PL + (q * 16 + r16) * 64 + dsx);
        }
#pragma unroll
        for (int t = 0; t < G::NCTW; ++t) {
          if (e + G::NE * t >= G::NCT) continue;
          const f16x8 ah = *reinterpret_cast<const f16x8*>(spw + t * 2048 + 16 * lane);
          const f16x8 al = *reinterpret_cast<const f16x8*>(spw + t * 2048 + 1024 + 16 * lane);
#pragma unroll
          for (int q = 0; q < G::POUT16; ++q) acc[q][t] = mfma_x2(ah, al, bh[q], bl[q], acc[q][t]);
        }
        return;
      }
      f16x8 bh[2], bl[2];
      bh[0] = *reinterpret_cast<const f16x8*>(Dh + r16 * 64 + dsx);
      bl[0] = *reinterpret_cast<const f16x8*>(Dh + G::DS_PL + r16 * 64 + dsx);
#pragma unroll
      for (int q = 0; q < G::POUT16; ++q) {
        if (q + 1 < G::POUT16) {
          bh[(q + 1) & 1] = *reinterpret_cast<const f16x8*>(Dh + ((q + 1) * 16 + r16) * 64 + dsx);
          bl[(q + 1) & 1] = *reinterpret_cast<const f16x8*>(Dh + G::DS_PL + ((q + 1) * 16 + r16) * 64 + dsx);
        }
#pragma unroll
        for (int t = 0; t < G::NCTW; ++t)
          if (e + G::NE * t < G::NCT) acc[q][t] = mfma_x2(pah[t], pal[t], bh[q & 1], bl[q & 1], acc[q][t]);
      }
    };
    // + residual (the block input, pytorch_layers.py:93-96, added after the BN bias) -> fp32 NHWC, tile t; the residual
    // loads of four pixel tiles are issued together (one memory round trip per group, not per value)
    auto epilogue = [&](int t) {
      int b_, oy_, ox_;
      tile_of(t, b_, oy_, ox_);
      constexpr int QG = G::POUT16 < 4 ? G::POUT16 : 4;
#pragma unroll
      for (int q0 = 0; q0 < G::POUT16; q0 += QG) {
        float4 r[QG][G::NCTW];
        size_t pix_[QG];
        bool in[QG];
#pragma unroll
        for (int qq = 0; qq < QG; ++qq) {
          const int o = (q0 + qq) * 16 + r16;
          const int gy = oy_ + o / TW, gx = ox_ + o % TW;
          in[qq] = gy < OH && gx < OW;
          pix_[qq] = ((size_t)b_ * OH + gy) * OW + gx;
#pragma unroll
          for (int tt = 0; tt < G::NCTW; ++tt) {
            r[qq][tt] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (RES && in[qq] && e + G::NE * tt < G::NCT)
              r[qq][tt] = *reinterpret_cast<const float4*>(X + pix_[qq] * CIN + (e + G::NE * tt) * 16 + 4 * kg);
          }
        }
#pragma unroll
        for (int qq = 0; qq < QG; ++qq) {
          if (!in[qq]) continue;
#pragma unroll
          for (int tt = 0; tt < G::NCTW; ++tt) {
            if (e + G::NE * tt >= G::NCT) continue;
            f32x4 v = acc[q0 + qq][tt];
            if constexpr (RES) {
              v[0] += r[qq][tt].x; v[1] += r[qq][tt].y; v[2] += r[qq][tt].z; v[3] += r[qq][tt].w;
            }
            *reinterpret_cast<float4*>(Y + pix_[qq] * COUT + (e + G::NE * tt) * 16 + 4 * kg) =
                make_float4(v[0], v[1], v[2], v[3]);
          }
        }
      }
    };
    load_pa(0);
    if (wave == 0) stamp(1, 3);
    __syncthreads();   // prologue stages landed (the VALU waves waited for their LDS-DMA)
    expand(Se0, Sl0);
    __syncthreads();   // slab 0 visible
    // iteration g (parity p = g & 1): P(g - 1) from Ds[p ^ 1] and the fragments of its chunk (PT: then, at a tile's
    // last chunk, the tile's outputs); chunk g's project fragments (in flight across E(g + 1) and the barrier); E(g + 1)
    // from stage p ^ 1 into slab p ^ 1 (PT: the next tile's rows split before its first chunk, loaded after the previous
    // tile's last)
    auto iter = [&](auto par, int g) {
      using Q = std::integral_constant<int, decltype(par)::value ^ 1>;
      if (wave == 0) stamp(g, 0);
      if (g >= 1) {
        project(dsb(Q{}));
        if (PT && kmod(g - 1) == G::NCH - 1) {
          epilogue((g - 1) / G::NCH);
          init_acc();
        }
      }
      if (g >= 1) load_pa(kmod(g));
      if (wave == 0) stamp(g, 1);
      if (g + 1 < GT) {
        if (PT && kmod(g + 1) == 0) split_mask((g + 1) / G::NCH);
        expand(se(Q{}), slab(Q{}));
        if (PT && kmod(g + 1) == G::NCH - 1 && (g + 1) / G::NCH + 1 < nt) load_raw((g + 1) / G::NCH + 1);
      }
      if (wave == 0) stamp(g, 2);
      lds_barrier();
    };
#pragma unroll 1
    for (int g = 0; g < GT; g += 2) {
      iter(I0{}, g);
      iter(I1{}, g + 1);
    }
    project(dsb(I1{}));   // (GT is even: the last chunk's parity is 1)
    epilogue(nt - 1);
    if (wave == 0) stamp(0, 7);
  } else {
    // ================= VALU waves: depthwise of output pixel tiles QPV d .. QPV d + QPV - 1 -> Ds
    const int d = wr;
    int pbase[G::QPV];
#pragma unroll
    for (int i = 0; i < G::QPV; ++i) {
      const int o = (G::QPV * d + i) * 16 + r16;
      pbase[i] = (o / TW) * S * G::IW + (o % TW) * S;
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the prologue stages landed
    __syncthreads();
    __syncthreads();   // slab 0 visible
    // iteration g (parity p): expand chunk g + 2's stage into stage p (released by E(g) in iteration g - 1) and depthwise
    // chunk g + 1's into stage p ^ 1 (released by V(g - 1)), from the registers loaded an iteration ago; the loads of
    // expand chunk g + 3 and depthwise chunk g + 2; V(g) from slab p and stage p into Ds[p]
    auto iter = [&](auto par, int g) {
      using Q = std::integral_constant<int, decltype(par)::value ^ 1>;
      if (wave == G::NE) stamp(g, 4);
      if (g + 2 < GT) dma_e(kmod(g + 2), se(par));
      if (g + 1 < GT) dma_d(kmod(g + 1), sd(Q{}));
      if (wave == G::NE) stamp(g, 5);
      const float* Sl = slab(par);
      const float* D = reinterpret_cast<const float*>(sd(par));
      char* Dh = dsb(par);
      const float4 d0 = *reinterpret_cast<const float4*>(D + 288 + 8 * kg);
      const float4 d1 = *reinterpret_cast<const float4*>(D + 288 + 8 * kg + 4);
      f32x2 a[G::QPV][4];
#pragma unroll
      for (int i = 0; i < G::QPV; ++i) {
        a[i][0] = f32x2{d0.x, d0.y}; a[i][1] = f32x2{d0.z, d0.w};
        a[i][2] = f32x2{d1.x, d1.y}; a[i][3] = f32x2{d1.z, d1.w};
      }
      // every tap's weights and the window's slab rows issued together (the VALU waves hold no accumulators): QPV + 2
      // shared rows per column (ROWS) or 3 per pixel tile
      constexpr int NR = G::ROWS ? G::QPV + 2 : 3 * G::QPV;
      float4 wv[3][3][2], sv[3][NR][2];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const float* wt = D + (ky * 3 + kx) * 32 + 8 * kg;
          wv[kx][ky][0] = *reinterpret_cast<const float4*>(wt);
          wv[kx][ky][1] = *reinterpret_cast<const float4*>(wt + 4);
        }
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int p = G::ROWS ? pbase[0] + r * G::IW + kx : pbase[r / 3] + (r % 3) * G::IW + kx;
          sv[kx][r][0] = *reinterpret_cast<const float4*>(Sl + SL::at(p, 2 * kg));
          sv[kx][r][1] = *reinterpret_cast<const float4*>(Sl + SL::at(p, 2 * kg + 1));
        }
      }
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const f32x2 w4[4] = {f32x2{wv[kx][ky][0].x, wv[kx][ky][0].y}, f32x2{wv[kx][ky][0].z, wv[kx][ky][0].w},
                               f32x2{wv[kx][ky][1].x, wv[kx][ky][1].y}, f32x2{wv[kx][ky][1].z, wv[kx][ky][1].w}};
#pragma unroll
          for (int i = 0; i < G::QPV; ++i) {
            const int r = G::ROWS ? i + ky : 3 * i + ky;
            dw_tap8(a[i], sv[kx][r][0], sv[kx][r][1], w4);
          }
        }
#pragma unroll
      for (int i = 0; i < G::QPV; ++i) {
        f16x8 bh, bl;
        relu_split8(a[i], bh, bl);
        const int o = (G::QPV * d + i) * 16 + r16;
        *reinterpret_cast<f16x8*>(Dh + o * 64 + dsx) = bh;
        *reinterpret_cast<f16x8*>(Dh + G::DS_PL + o * 64 + dsx) = bl;
      }
      if (wave == G::NE) stamp(g, 6);
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the DMA pieces landed (read by every wave next)
      lds_barrier();
    };
#pragma unroll 1
    for (int g = 0; g < GT; g += 2) {
      iter(I0{}, g);
      iter(I1{}, g + 1);
    }
  }
  if constexpr (SPEF_X2_STAMP) {   // every wave: the last barrier, then the stamps over the start of tile 0's output
    __syncthreads();
    if (stamp_wg) {
      const int n = 8 * (G::NCH < 64 ? G::NCH : 64);
      if (tid < n) reinterpret_cast<uint32_t*>(Y)[tid] = Stamps[tid];
    }
  }
}

// Hidden-split join: y = ((part 0 + part 1) + ...) + bias (+ residual), in that order, 4 channels per thread.
template <int P, bool RES>
__global__ __launch_bounds__(256) void x2_split_reduce_kernel(const float* __restrict__ parts, size_t pstride,
                                                              const float* __restrict__ bias,
                                                              const float* __restrict__ X, float* __restrict__ Y,
                                                              size_t n4, int cout4) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 v = reinterpret_cast<const float4*>(parts)[i];
#pragma unroll
  for (int p = 1; p < P; ++p) {
    const float4 u = reinterpret_cast<const float4*>(parts + p * pstride)[i];
    v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
  }
  const float4 bb = reinterpret_cast<const float4*>(bias)[i % (size_t)cout4];
  v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
  if constexpr (RES) {
    const float4 r = reinterpret_cast<const float4*>(X)[i];
    v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
  }
  reinterpret_cast<float4*>(Y)[i] = v;
}

// (cin, hidden, cout, stride, expand, residual, TH, TW, waves, cout groups, kind): MobileNet-V2's 17 blocks
// (mobilenet_v2.py:240-249). kind 0: slab kernel with `waves` waves (tiles keep the hi / lo input tile + fp32 slab at
// 2+ workgroups per CU where the geometry allows); kind 1: role-split kernel (4 + 4 waves) with the project weights
// staged in LDS; kind 2: role-split, project weights from L2 (block 17: no two depthwise waves share a channel tile).
// Cout groups: with g groups the depthwise waves split into g sets that each run the whole depthwise for their pixels
// and project onto 1/g of the output channels, so g > 1 computes the depthwise g times. Interleaved A/B at B = 64
// (tools/x2_ab.sh, per launch): blocks 8-10 81 -> 54 us and block 11 84 -> 59 us with g 2 -> 1; blocks 12-13 158
// (8x8, g 2) -> 125 (8x16, g 2) -> 89 us (8x16, g 1); blocks 15-16 93 -> 91 us (g 2 -> 1); block 17 142 us at g 4,
// 125 at g 2, 322 at g 1 (80 accumulator registers per wave: spills). URSONet step 2.11 -> 1.85 ms, keypoint mode
// 1.27 -> 1.05 ms (with the small-map table below).
// Kind 3 = kind 1 with persistent tiles (x2_irw_kernel's PT: a second tile per CU streams on without a prologue):
// the maps with more tiles than CUs at 512^2 (blocks 8-14: 512 tiles at B = 64). Kind 5 / 6: the three-stage kernel
// (x2_irp_kernel) without / with persistent tiles. Measured per step at B = 64 (tools/ktime.sh, bit-identical
// outputs): blocks 15-16 131.4 -> 101.9 us on kind 5, blocks 12-13 147.9 -> 142.0 and block 11 51.8 -> 49.1 on kind
// 6; blocks 8-10 130.7 -> 138.5 on kind 6 (their VALU role is the longer one there), so they stay on kind 3.
#define SPEF_X2_MID(X)                                           \
  X(64, 384, 64, 1, true, true, 8, 16, 8, 1, 3)      /* 8-10 */   \
  X(64, 384, 96, 1, true, false, 8, 16, 8, 1, 6)     /* 11 */     \
  X(96, 576, 96, 1, true, true, 8, 16, 8, 1, 6)      /* 12-13 */
#define SPEF_X2_TABLE(X)                                         \
  X(32, 32, 16, 1, false, false, 8, 16, 4, 1, 0)    /* 1 */      \
  X(16, 96, 24, 2, true, false, 8, 8, 4, 1, 0)      /* 2 */      \
  X(24, 144, 24, 1, true, true, 8, 16, 4, 1, 0)     /* 3 */      \
  X(24, 144, 32, 2, true, false, 8, 8, 4, 1, 0)     /* 4 */      \
  X(32, 192, 32, 1, true, true, 8, 16, 4, 1, 0)     /* 5-6 */    \
  X(32, 192, 64, 2, true, false, 8, 8, 4, 1, 0)     /* 7 */      \
  SPEF_X2_MID(X)                                                 \
  X(96, 576, 160, 2, true, false, 4, 8, 8, 2, 3)    /* 14 */     \
  X(160, 960, 160, 1, true, true, 8, 8, 8, 1, 5)    /* 15-16 */  \
  X(160, 960, 320, 1, true, false, 8, 8, 8, 1, 5)    /* 17 */
// 16x16 tiles with 8 waves (2 workgroups per CU) where they tile the map exactly: block 3 at 512^2 (interleaved A/B,
// round 4: 165 -> 153 us per step); on maps they do not divide (60x96, 30x48 at 240x384) the partial tiles cost more
// than the occupancy gains. Blocks 5-6 left this table in round 5: behind the fp16mx front end 8 x 16 tiles measured
// 139 -> 117 us per step (round 4, fp16x2: 119 -> 115 the other way).
#define SPEF_X2_EXACT_TABLE(X)                                      \
  X(24, 144, 24, 1, true, true, 16, 16, 8, 1, 0)     /* 3 */
// Maps whose primary tiling leaves CUs idle (fewer workgroups than CUs; the role-split kernels run one workgroup
// per CU): blocks 15-17 at 240x384 (8x12 maps: 128 workgroups of 8x8 at B = 64) split the hidden dimension over P
// workgroups per tile (last field; partial sums joined by x2_split_reduce_kernel in the caller's scratch).
#define SPEF_X2_SMALL_TABLE(X)                                      \
  X(160, 960, 160, 1, true, true, 8, 8, 8, 1, 1, 2)    /* 15-16 */  \
  X(160, 960, 320, 1, true, false, 8, 8, 8, 2, 2, 2)   /* 17 */

template <typename K>
static hipError_t x2_set_lds(K k, int lds) {   // > 64 KiB dynamic LDS needs the attribute (once per instantiation)
  if (lds <= 65536) return hipSuccess;
  return hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}

template <int CIN, int HID, int COUT, int S, bool EXPAND, bool RES, int TH, int TW, int NW, int WCO, int KIND,
          int P = 1, int IO = 0>
static hipError_t x2_irb_go(const void* x, const void* we, const float* be, const float* wd, const float* bd,
                            const void* wp, const float* bp, void* y, int B, int H, int W, int OH, int OW,
                            hipStream_t s, float* scratch = nullptr, int num_cu = 256) {
  if constexpr (KIND != 0 && IO != 0) {
    return hipErrorNotSupported;   // fp16 block I/O: the slab kernels (the fp16mx schedule's blocks 1-7) only
  }
  const int tiles_x = (OW + TW - 1) / TW, tiles_y = (OH + TH - 1) / TH;
  const int64_t nwg64 = (int64_t)tiles_x * tiles_y * B * P;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  static DevOnce attr_set;
  if constexpr (KIND == 0) {
    using G = X2Geom<CIN, HID, COUT, S, TH, TW, EXPAND, NW, WCO>;
    auto k = x2_irb_kernel<CIN, HID, COUT, S, TH, TW, EXPAND, RES, NW, WCO, IO>;
    if (!attr_set.done()) {
      hipError_t e = x2_set_lds(k, G::LDS_BYTES);
      if (e != hipSuccess) return e;
      attr_set.set();
    }
    k<<<nwg, NW * 64, G::LDS_BYTES, s>>>(x, (const _Float16*)we, be, wd, bd, (const _Float16*)wp, bp, y, H, W, OH, OW,
                                        tiles_x, tiles_y, nwg);
  } else if constexpr ((KIND == 5 || KIND == 6) && IO == 0) {
    static_assert(EXPAND && P == 1, "three-stage blocks expand, one part");
    constexpr bool PT = KIND == 6;   // persistent tiles: ceil(tiles / CUs) tiles per workgroup
    using G = X2pGeom<CIN, HID, COUT, S, TH, TW>;   // static LDS (G::LDS_BYTES)
    auto k = x2_irp_kernel<CIN, HID, COUT, S, TH, TW, RES, PT>;
    uint32_t grid = nwg;
    if constexpr (PT) {
      const uint32_t per = (nwg + (uint32_t)num_cu - 1) / (uint32_t)num_cu;
      grid = (nwg + per - 1) / per;
    }
    k<<<grid, G::NW * 64, 0, s>>>((const float*)x, (const _Float16*)we, be, wd, bd, (const _Float16*)wp, bp, (float*)y, H,
                                  W, OH, OW, tiles_x, tiles_y, grid, nwg);
  } else if constexpr (IO == 0) {
    static_assert(EXPAND && NW == 8, "role-split blocks expand, 4 + 4 waves");
    constexpr bool PT = KIND == 3 && P == 1;   // persistent tiles (kind 3): ceil(tiles / CUs) tiles per workgroup
    using G = X2wGeom<CIN, HID, COUT, S, TH, TW, WCO, KIND != 2, P>;
    auto k = x2_irw_kernel<CIN, HID, COUT, S, TH, TW, RES, WCO, KIND != 2, P, PT>;
    if (!attr_set.done()) {
      hipError_t e = x2_set_lds(k, G::LDS_BYTES);
      if (e != hipSuccess) return e;
      attr_set.set();
    }
    const size_t pstride = (size_t)B * OH * OW * COUT;   // floats per hidden part (16-B multiple: COUT % 4 == 0)
    if (P > 1 && !scratch) return hipErrorInvalidValue;
    uint32_t grid = nwg;
    if constexpr (PT) {
      const uint32_t per = (nwg + (uint32_t)num_cu - 1) / (uint32_t)num_cu;
      grid = (nwg + per - 1) / per;
    }
    k<<<grid, G::NW * 64, G::LDS_BYTES, s>>>((const float*)x, (const _Float16*)we, be, wd, bd, (const _Float16*)wp, bp,
                                     P > 1 ? scratch : (float*)y, H, W, OH, OW, tiles_x, tiles_y, grid, pstride, nwg);
    if constexpr (P > 1) {
      const size_t n4 = pstride / 4;
      x2_split_reduce_kernel<P, RES><<<(unsigned)((n4 + 255) / 256), 256, 0, s>>>(scratch, pstride, bp,
                                                                                   (const float*)x, (float*)y, n4,
                                                                                   COUT / 4);
    }
  }
  return hipGetLastError();
}

bool x2_irb_supported(int cin, int hid, int cout, int stride, bool expand, bool res) {
#define SPEF_X2_HAS(CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_) \
  if (cin == CI && hid == HI && cout == CO && stride == ST && expand == EX && res == RS) return true;
  SPEF_X2_TABLE(SPEF_X2_HAS)
#undef SPEF_X2_HAS
  return false;
}

hipError_t launch_x2_irb(int cin, int hid, int cout, int stride, bool expand, bool res, const void* x, const void* we,
                         const float* be, const float* wd, const float* bd, const void* wp, const float* bp, void* y,
                         int B, int H, int W, int OH, int OW, hipStream_t s, float* scratch, int io) {
  if (!x || !y || !wd || !bd || !wp || !bp || (expand && (!we || !be)) || io < 0 || io > 3) return hipErrorInvalidValue;
  int num_cu = 0;
  {
    static int cus[32] = {};   // per device (first call on each)
    const int dev = DevOnce::dev();
    if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus[dev] = 256;
    num_cu = cus[dev];
  }
#define SPEF_X2_IO_SWITCH(CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_)                                    \
  switch (io) {                                                                                               \
    case 0: return x2_irb_go<CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_, 1, 0>(x, we, be, wd, bd, wp, bp, y, \
                                                                               B, H, W, OH, OW, s, nullptr,   \
                                                                               num_cu);                       \
    case 1: return x2_irb_go<CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_, 1, 1>(x, we, be, wd, bd, wp, bp, y, \
                                                                               B, H, W, OH, OW, s);           \
    case 2: return x2_irb_go<CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_, 1, 2>(x, we, be, wd, bd, wp, bp, y, \
                                                                               B, H, W, OH, OW, s);           \
    default: return x2_irb_go<CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_, 1, 3>(x, we, be, wd, bd, wp, bp, y, \
                                                                                B, H, W, OH, OW, s);          \
  }
#define SPEF_X2_TILES(TH_, TW_) ((int64_t)((OW + (TW_)-1) / (TW_)) * ((OH + (TH_)-1) / (TH_)) * B)
#define SPEF_X2_SMALL(CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_, P_)                                    \
  if (cin == CI && hid == HI && cout == CO && stride == ST && expand == EX && res == RS && scratch && !io &&  \
      SPEF_X2_TILES(8, 8) < num_cu && SPEF_X2_TILES(TH_, TW_) * P_ <= num_cu)                                \
    return x2_irb_go<CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_, P_>(x, we, be, wd, bd, wp, bp, y, B, H, W, OH, \
                                                                         OW, s, scratch, num_cu);
  SPEF_X2_SMALL_TABLE(SPEF_X2_SMALL)
#undef SPEF_X2_SMALL
#ifndef SPEF_X2_EXACT_ON   // A/B aid: 0 = the primary 8 x 16 tiles on exact maps too
#define SPEF_X2_EXACT_ON 1
#endif
#define SPEF_X2_EXACT(CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_)                                        \
  if (SPEF_X2_EXACT_ON && cin == CI && hid == HI && cout == CO && stride == ST && expand == EX && res == RS &&  \
      OH % (TH_) == 0 &&                                                                                        \
      OW % (TW_) == 0)                                                                                        \
    SPEF_X2_IO_SWITCH(CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_)
  SPEF_X2_EXACT_TABLE(SPEF_X2_EXACT)
#undef SPEF_X2_EXACT
#undef SPEF_X2_TILES
#define SPEF_X2_CASE(CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_)                                         \
  if (cin == CI && hid == HI && cout == CO && stride == ST && expand == EX && res == RS)                      \
    SPEF_X2_IO_SWITCH(CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_)
  SPEF_X2_TABLE(SPEF_X2_CASE)
#undef SPEF_X2_CASE
#undef SPEF_X2_IO_SWITCH
  return hipErrorNotSupported;
}

// The kernel launch_x2_irb runs for these arguments (the same table walk): "x2_irb_kernel" (slab), "x2_irw_kernel"
// (role-split), "x2_irp_kernel" (three-stage); nullptr when none. Profiling labels only.
const char* x2_irb_kernel_name(int cin, int hid, int cout, int stride, bool expand, bool res, int B, int OH, int OW,
                               bool scratch, int io, int num_cu) {
  auto name = [](int kind) { return kind == 0 ? "x2_irb_kernel" : kind >= 5 ? "x2_irp_kernel" : "x2_irw_kernel"; };
#define SPEF_X2_TILES(TH_, TW_) ((int64_t)((OW + (TW_)-1) / (TW_)) * ((OH + (TH_)-1) / (TH_)) * B)
#define SPEF_X2_SMALL(CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_, P_)                                    \
  if (cin == CI && hid == HI && cout == CO && stride == ST && expand == EX && res == RS && scratch && !io &&  \
      SPEF_X2_TILES(8, 8) < num_cu && SPEF_X2_TILES(TH_, TW_) * P_ <= num_cu)                                \
    return name(KD_);
  SPEF_X2_SMALL_TABLE(SPEF_X2_SMALL)
#undef SPEF_X2_SMALL
#undef SPEF_X2_TILES
#define SPEF_X2_NAME_EXACT(CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_)                                   \
  if (SPEF_X2_EXACT_ON && cin == CI && hid == HI && cout == CO && stride == ST && expand == EX && res == RS &&  \
      OH % (TH_) == 0 && OW % (TW_) == 0)                                                                     \
    return (KD_ != 0 && io) ? nullptr : name(KD_);
  SPEF_X2_EXACT_TABLE(SPEF_X2_NAME_EXACT)
#undef SPEF_X2_NAME_EXACT
#define SPEF_X2_NAME(CI, HI, CO, ST, EX, RS, TH_, TW_, NW_, WC_, KD_)                                         \
  if (cin == CI && hid == HI && cout == CO && stride == ST && expand == EX && res == RS)                      \
    return (KD_ != 0 && io) ? nullptr : name(KD_);
  SPEF_X2_TABLE(SPEF_X2_NAME)
#undef SPEF_X2_NAME
  return nullptr;
}

// ------------------------------------------------------------------------------------------ front: stem + block 1
// uint8 NHWC frames -> stem ConvBnAct 3 -> 32, 3x3 / 2 (mobilenet_v2.py:252-254; ToTensor's /255 folded into the
// weights) -> block 1 (depthwise 3x3 + project 32 -> 16, pytorch_layers.py:65-98) -> fp32 block-1 output, one kernel:
// the 32-channel stem map (8.4 MB/img at 512^2 in fp32) never reaches HBM. A u8 pixel is exact in fp16, so the stem is
// two MFMAs per product (W_hi x + W_lo x, the blob's split /255-folded operand x0). Its K runs over the 3 input rows
// of the stencil, one K step per row ky with k = 4 kx + ci (ci padded to 4; k >= 12 zero), so a lane's B fragment is
// one 16-B (kg 0) or 8-B (kg 1) LDS read of the staged input tile [row][col][4] (fp16). The stem map of the output
// tile + halo goes to the fp32 slab (zero outside the image: the depthwise's padding), then block 1 runs as in
// x2_irb_kernel.
template <int TH, int TW, int NW_ = 4>
struct X2FrontGeom {
  static constexpr int NW = NW_;
  static constexpr int PH = TH + 2, PW = TW + 2;        // stem pixels of the tile (+ block-1 halo)
  static constexpr int PIN = PH * PW, PIN16 = (PIN + 15) / 16, PINP = PIN16 * 16;
  static constexpr int IRW = 2 * PH + 1, ICL = 2 * PW + 1;   // input rows / columns of the stem stencil
  static constexpr int ICS = (ICL * 4 + 8 + 7) / 8 * 8;   // halves per staged input row (16-B rows; zero tail)
  using SL = X2Slab<1, PINP>;
  static constexpr int POUT16 = TH * TW / 16, QPW = POUT16 / NW;
  static constexpr int EPT = (PIN16 + NW - 1) / NW;
  static constexpr int XI_H = (IRW * ICS + 7) / 8 * 8;   // staged input (halves)
  static constexpr int DWS = 9 * 32 + 32;               // block-1 depthwise weights + bias (floats)
  static constexpr int TRASH = 16 * 24;                 // dummy rows: stem stores of pixels outside the stem map
  static constexpr int LDS_BYTES = XI_H * 2 + (SL::FLOATS + DWS + TRASH) * 4;
  static_assert(TW == 16 && POUT16 % NW == 0 && EPT <= 32, "front tile");
};

template <int TH, int TW, int NW_ = 4, bool OUT16 = false>
__global__ __launch_bounds__(NW_ * 64) __attribute__((amdgpu_waves_per_eu(NW_ == 4 ? 3 : 4, 8))) void x2_front_kernel(
    const uint8_t* __restrict__ X, const _Float16* __restrict__ Wsx, const float* __restrict__ bs,
    const float* __restrict__ Wd, const float* __restrict__ bd, const _Float16* __restrict__ Wp,
    const float* __restrict__ bp, void* __restrict__ Y, int H, int W, int OH, int OW, int tiles_x, int tiles_y,
    uint32_t nwg) {
  using G = X2FrontGeom<TH, TW, NW_>;
  using SL = typename G::SL;
  constexpr int NW = G::NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  _Float16* Xi = reinterpret_cast<_Float16*>(smem);                     // [IRW][ICS] input tile, fp16
  float* Sl = reinterpret_cast<float*>(smem + G::XI_H * 2);             // stem map of the tile (+halo), plane layout
  float* Ds = Sl + SL::FLOATS;                                          // [9][32] depthwise weights, [32] bias

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  uint32_t L = xcd_remap(blockIdx.x, nwg);
  const int tx = (int)(L % (uint32_t)tiles_x);
  L /= (uint32_t)tiles_x;
  const int ty = (int)(L % (uint32_t)tiles_y);
  const int b = (int)(L / (uint32_t)tiles_y);
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int sy0 = oy0 - 1, sx0 = ox0 - 1;              // stem pixel of tile position (0, 0)
  const int iy0 = 2 * sy0 - 1, ix0 = 2 * sx0 - 1;      // input pixel of staged position (0, 0)

  // ---- staging: the input rows of the stencil as aligned dword loads (a row segment is 3 ICL bytes at any byte
  // alignment), bytes scattered to fp16 [row][col][4] over a zero-filled tile (zero outside the frame: the stem's
  // padding; the ci = 3 pad); block-1 depthwise weights + bias
  // Interior tiles (every staged row and column inside the frame, 4-byte aligned rows): the row's dwords load one per
  // lane, and lane c builds stem pixel column c from two of them (two lane shuffles + one v_alignbyte), converts the
  // three bytes exactly to fp16 (0x6400 | byte = 1024 + byte, minus 1024) and writes its 4 halves with one 8-B store.
  const bool fast = (W & 3) == 0 && ix0 >= 0 && ix0 + G::ICL <= W && iy0 >= 0 && iy0 + G::IRW <= H;
  if (fast) {
    constexpr int RPW = (G::IRW + NW - 1) / NW;
    static_assert(G::ICL <= 64 && (3 * G::ICL + 3 + 3) / 4 < 64, "one row per wave");
    const int off = (3 * ix0) & 3;                      // rows start `off` bytes into their dword (W % 4 == 0)
    const int nl = (off + 3 * G::ICL + 3) / 4;          // dwords holding the row segment
    const uint8_t* Xb = X + (size_t)b * H * W * 3;
    uint32_t v[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int r = wave + NW * i;
      v[i] = 0;
      if (r < G::IRW && lane < nl)
        v[i] = *reinterpret_cast<const uint32_t*>(Xb + (((size_t)(iy0 + r) * W + ix0) * 3 - off) + 4 * lane);
    }
    float4 dwv[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int u = tid + NW * 64 * i;   // 72 pieces of the [9][32] weights, 8 of the bias
      dwv[i] = u < 72 ? *reinterpret_cast<const float4*>(Wd + 4 * u)
                      : u < 80 ? *reinterpret_cast<const float4*>(bd + 4 * (u - 72)) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const int q = 3 * lane + off, d = q >> 2, sh = q & 3;   // lane c = pixel column c: segment bytes q .. q + 2
    const f16x2 k1024 = {(_Float16)1024.0f, (_Float16)1024.0f};
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int r = wave + NW * i;
      const uint32_t lo = __shfl(v[i], d, 64), hi = __shfl(v[i], d + 1 < 64 ? d + 1 : 63, 64);
      if (r < G::IRW && lane < G::ICL) {
        const uint32_t by = __builtin_amdgcn_alignbyte(hi, lo, sh);   // bytes ci 0, 1, 2 of the pixel
        const f16x2 h01 = __builtin_bit_cast(f16x2, __builtin_amdgcn_perm(0u, by, 0x0c010c00u) | 0x64006400u) - k1024;
        const f16x2 h2 = __builtin_bit_cast(f16x2, __builtin_amdgcn_perm(0u, by, 0x0c0c0c02u) | 0x64006400u) - k1024;
        *reinterpret_cast<uint2*>(Xi + r * G::ICS + 4 * lane) =
            make_uint2(__builtin_bit_cast(uint32_t, h01), __builtin_bit_cast(uint32_t, h2));
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int u = tid + NW * 64 * i;
      if (u < 80) *reinterpret_cast<float4*>(Ds + 4 * u) = dwv[i];
    }
  } else {
    constexpr int NDW = (3 * G::ICL + 3 + 3) / 4 + 1;   // dwords covering one row segment at any alignment
    constexpr int NPC = G::IRW * NDW;
    constexpr int NIT = (NPC + NW * 64 - 1) / (NW * 64);
    constexpr int NZ = G::XI_H / 8;                     // 16-B pieces of the staged tile
    const size_t img = (size_t)b * H * W * 3;
    uint32_t v[NIT];
    bool ld[NIT];
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int u = tid + NW * 64 * i;
      const int r = u / NDW, j = u - r * NDW;
      const int iy = iy0 + r;
      v[i] = 0;
      ld[i] = false;
      if (u < NPC && iy >= 0 && iy < H) {
        const int64_t rb = (int64_t)(img + (size_t)iy * W * 3);
        const int64_t vs = rb + 3 * (int64_t)(ix0 > 0 ? ix0 : 0);
        const int64_t ve = rb + 3 * (int64_t)(ix0 + G::ICL < W ? ix0 + G::ICL : W);
        const int64_t a = ((rb + 3 * (int64_t)ix0) & ~(int64_t)3) + 4 * j;   // may start left of the frame row
        if (a + 4 > vs && a < ve) {
          v[i] = *reinterpret_cast<const uint32_t*>(X + a);
          ld[i] = true;
        }
      }
    }
    float4 dwv[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int u = tid + NW * 64 * i;   // 72 pieces of the [9][32] weights, 8 of the bias
      dwv[i] = u < 72 ? *reinterpret_cast<const float4*>(Wd + 4 * u)
                      : u < 80 ? *reinterpret_cast<const float4*>(bd + 4 * (u - 72)) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int u = tid; u < NZ; u += NW * 64) reinterpret_cast<uint4*>(Xi)[u] = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int u = tid + NW * 64 * i;
      if (u < 80) *reinterpret_cast<float4*>(Ds + 4 * u) = dwv[i];
    }
    __syncthreads();
    // dword j's first byte is segment byte 4 j - off (off = the segment start's offset in its dword); valid bytes:
    // segment bytes [rlo, rhi), the frame row's part of the segment
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      if (!ld[i]) continue;
      const int u = tid + NW * 64 * i;
      const int r = u / NDW, j = u - r * NDW;
      const int64_t rb = (int64_t)(img + (size_t)(iy0 + r) * W * 3);
      const int off = (int)((rb + 3 * (int64_t)ix0) & 3);      // segment start within its dword
      const int rlo = ix0 < 0 ? -3 * ix0 : 0, rhi = 3 * ((ix0 + G::ICL < W ? ix0 + G::ICL : W) - ix0);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int rel = 4 * j + k - off;   // byte of the segment: column rel / 3, channel rel % 3
        if (rel < rlo || rel >= rhi) continue;
        Xi[r * G::ICS + 4 * (rel / 3) + rel % 3] = (_Float16)(float)((v[i] >> (8 * k)) & 0xffu);
      }
    }
  }
  // stem A fragments for the 3 K steps (ky) and 2 channel halves: lane (r16 = output channel, kg) holds k = 8kg + e,
  // k = 4 kx + ci. The blob's x0 is already in this order: [2 planes][3 ky][32 ch][32 k] (spef_blob.hpp).
  auto stem_a = [&](int h, int ky, f16x8& ah, f16x8& al) {
    const int off = (ky * 32 + 16 * h + r16) * 32 + 8 * kg;
    ah = *reinterpret_cast<const f16x8*>(Wsx + off);
    al = *reinterpret_cast<const f16x8*>(Wsx + 3 * 32 * 32 + off);
  };
  float sb[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float4 t = *reinterpret_cast<const float4*>(bs + 16 * h + 4 * kg);
    sb[h][0] = t.x; sb[h][1] = t.y; sb[h][2] = t.z; sb[h][3] = t.w;
  }
  __syncthreads();

  // ---- stem of the tile's stem pixels p = 16 pt + r16 -> slab (ReLU; zero outside the stem map); K steps (ky)
  // outermost so one (ky, half) A fragment pair is live at a time
  {
    f32x4 e[G::EPT][2];
    int xo[G::EPT], soff[G::EPT];
#pragma unroll
    for (int j = 0; j < G::EPT; ++j) {
      const int p = (wave + NW * j) * 16 + r16;
      const int pc = p < G::PIN ? p : G::PIN - 1;
      const int py = pc / G::PW, px = pc - (pc / G::PW) * G::PW;
      const int sy = sy0 + py, sx = sx0 + px;
      const bool ok = p < G::PIN && sy >= 0 && sy < OH && sx >= 0 && sx < OW;
      // pixels outside the stem map (the depthwise's zero padding) get zeros once; their stem results go to a dummy row
      soff[j] = ok ? SL::at(p, kg) : SL::FLOATS + G::DWS + r16 * 24 + 4 * kg;
      if (!ok && p < G::PIN) {
        *reinterpret_cast<float4*>(Sl + SL::at(p, kg)) = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4*>(Sl + SL::at(p, kg) + 8) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      xo[j] = 2 * py * G::ICS + 8 * px + (kg == 1 ? 8 : 0);   // stem pixel px reads input cols 2px .. 2px + 2
#pragma unroll
      for (int h = 0; h < 2; ++h) e[j][h] = f32x4{sb[h][0], sb[h][1], sb[h][2], sb[h][3]};
    }
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      f16x8 bx[G::EPT];
#pragma unroll
      for (int j = 0; j < G::EPT; ++j) {
        const _Float16* xr = Xi + xo[j] + ky * G::ICS;
        if (kg == 0) {
          bx[j] = *reinterpret_cast<const f16x8*>(xr);
        } else if (kg == 1) {
          const uint2 t = *reinterpret_cast<const uint2*>(xr);
          bx[j] = __builtin_bit_cast(f16x8, make_uint4(t.x, t.y, 0u, 0u));
        } else {
          bx[j] = __builtin_bit_cast(f16x8, make_uint4(0u, 0u, 0u, 0u));
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f16x8 ah, al;
        stem_a(h, ky, ah, al);
#pragma unroll
        for (int j = 0; j < G::EPT; ++j) {
          e[j][h] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bx[j], e[j][h], 0, 0, 0);
          e[j][h] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bx[j], e[j][h], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < G::EPT; ++j) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
        *reinterpret_cast<float4*>(Sl + soff[j] + 8 * h) = make_float4(
            fmaxf(e[j][h][0], 0.f), fmaxf(e[j][h][1], 0.f), fmaxf(e[j][h][2], 0.f), fmaxf(e[j][h][3], 0.f));
    }
  }
  __syncthreads();

  // ---- block 1: depthwise 3x3 (fp32, kx outer / ky inner) + BN + ReLU -> hi / lo -> project 32 -> 16
  f32x2 a[G::QPW][4];
  int pbase[G::QPW];
  {
    const float4 d0 = *reinterpret_cast<const float4*>(Ds + 288 + 8 * kg);
    const float4 d1 = *reinterpret_cast<const float4*>(Ds + 288 + 8 * kg + 4);
#pragma unroll
    for (int q = 0; q < G::QPW; ++q) {
      a[q][0] = f32x2{d0.x, d0.y}; a[q][1] = f32x2{d0.z, d0.w};
      a[q][2] = f32x2{d1.x, d1.y}; a[q][3] = f32x2{d1.z, d1.w};
      const int o = (wave * G::QPW + q) * 16 + r16;
      pbase[q] = (o / TW) * G::PW + (o % TW);
    }
  }
#pragma unroll 1   // (one kernel column in flight: fully unrolled, the 36 tap loads hoist and cost an occupancy step)
  for (int kx = 0; kx < 3; ++kx)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const float* wt = Ds + (ky * 3 + kx) * 32 + 8 * kg;
      const float4 w0 = *reinterpret_cast<const float4*>(wt), w1 = *reinterpret_cast<const float4*>(wt + 4);
      const f32x2 w4[4] = {f32x2{w0.x, w0.y}, f32x2{w0.z, w0.w}, f32x2{w1.x, w1.y}, f32x2{w1.z, w1.w}};
#pragma unroll
      for (int q = 0; q < G::QPW; ++q) {
        const int p = pbase[q] + ky * G::PW + kx;
        dw_tap8(a[q], *reinterpret_cast<const float4*>(Sl + SL::at(p, 2 * kg)),
                *reinterpret_cast<const float4*>(Sl + SL::at(p, 2 * kg + 1)), w4);
      }
    }
  const f16x8 ph = *reinterpret_cast<const f16x8*>(Wp + r16 * 32 + 8 * kg);
  const f16x8 pl = *reinterpret_cast<const f16x8*>(Wp + 16 * 32 + r16 * 32 + 8 * kg);
  const float4 bb = *reinterpret_cast<const float4*>(bp + 4 * kg);
#pragma unroll
  for (int q = 0; q < G::QPW; ++q) {
    f16x8 bh, bl;
    relu_split8(a[q], bh, bl);
    const f32x4 v = mfma_x2(ph, pl, bh, bl, f32x4{bb.x, bb.y, bb.z, bb.w});
    const int o = (wave * G::QPW + q) * 16 + r16;
    const int gy = oy0 + o / TW, gx = ox0 + o % TW;
    if (gy < OH && gx < OW) st_act4(Y, (((size_t)b * OH + gy) * OW + gx) * 16 + 4 * kg, v, OUT16);
  }
}

#ifndef SPEF_X2_FRONT_TH
#define SPEF_X2_FRONT_TH 16
#define SPEF_X2_FRONT_NW 8
#endif
template <bool OUT16>
static hipError_t x2_front_go(const void* x, const void* wsx, const float* bs, const float* wd, const float* bd,
                              const void* wp, const float* bp, void* y, int B, int H, int W, int OH, int OW,
                              hipStream_t s) {
  constexpr int TH = SPEF_X2_FRONT_TH, TW = 16, NW = SPEF_X2_FRONT_NW;
  using G = X2FrontGeom<TH, TW, NW>;
  if (!x || !wsx || !bs || !wd || !bd || !wp || !bp || !y) return hipErrorInvalidValue;
  const int tiles_x = (OW + TW - 1) / TW, tiles_y = (OH + TH - 1) / TH;
  const int64_t nwg64 = (int64_t)tiles_x * tiles_y * B;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  static DevOnce attr_set;
  if (!attr_set.done()) {
    hipError_t e = x2_set_lds(x2_front_kernel<TH, TW, NW, OUT16>, G::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set.set();
  }
  x2_front_kernel<TH, TW, NW, OUT16><<<nwg, NW * 64, G::LDS_BYTES, s>>>((const uint8_t*)x, (const _Float16*)wsx, bs,
                                                                      wd, bd, (const _Float16*)wp, bp, y, H, W, OH, OW,
                                                                      tiles_x, tiles_y, nwg);
  return hipGetLastError();
}
hipError_t launch_x2_front(const void* x, const void* wsx, const float* bs, const float* wd, const float* bd,
                           const void* wp, const float* bp, void* y, int B, int H, int W, int OH, int OW,
                           hipStream_t s, bool out16) {
  return out16 ? x2_front_go<true>(x, wsx, bs, wd, bd, wp, bp, y, B, H, W, OH, OW, s)
               : x2_front_go<false>(x, wsx, bs, wd, bd, wp, bp, y, B, H, W, OH, OW, s);
}

// ------------------------------------------------------------------------------------------ 1x1 conv, fp32 I/O
// C^T = W X^T as pw_kernel: a wave owns NT output-channel tiles x MT pixel tiles; 4 waves on 64 MT consecutive
// pixels; channel chunks fastest-varying so one pixel block's chunks share an XCD L2. B fragments: 8 fp32 values
// per lane from HBM / L2, split once and used by all NT channel tiles. POOL (URSONetHead's x.mean([2,3]),
// ursonet.py:30, when HW % 64 == 0): the 1280-channel map is never stored -- each wave sums the ReLU'd outputs of its
// 64 pixels (one image) over its pixel tiles and then over the 16 pixel lanes (xor shuffles, fixed order) into
// Y = partial [M / 64][N]; x2_pool_reduce_kernel adds an image's partials in order and divides by HW.
template <int NT, int MT, bool POOL>
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
  if constexpr (POOL) {   // MT = 4: the wave's 64 pixels m0 .. m0 + 63, all valid when m0 < M (M % 64 == 0)
#pragma unroll
    for (int a = 0; a < NT; ++a) {
      float sm[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = 0.f;
#pragma unroll
        for (int m = 0; m < MT; ++m) t += fmaxf(acc[a][m][r], 0.f);
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) t += __shfl_xor(t, o, 64);
        sm[r] = t;
      }
      const int i = n0 + 16 * a + 4 * kg;
      if (r16 == 0 && i < N && m0 < M)   // (a workgroup's last waves may lie past M: no partial for them)
        *reinterpret_cast<float4*>(Y + (size_t)(m0 / 64) * N + i) = make_float4(sm[0], sm[1], sm[2], sm[3]);
    }
    return;
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

// Staged form (the last conv, K = 320): 64 pixels x 256 output channels per workgroup. The 64 x K fp32 input block is
// split into hi / lo fp16 once per workgroup and staged in LDS (80 KB at K = 320: two workgroups per CU), instead of
// once per wave and 64-channel chunk from L2 as above (4x the split VALU and 4x the activation reads); the four waves
// take 64 channels each and stream their hi / lo weight fragments from L2 one K step ahead. Same products, same
// accumulation order, same pool partials as x2_pw_kernel<4, 4, POOL> (bit-identical). LDS rows of Kp halves with the
// 16-B granule index XOR-ed by (row & 7): the 8 rows a ds_read_b128 lane group reads hit disjoint banks.
#ifndef SPEF_X2_PWS
#define SPEF_X2_PWS 1
#endif
// Waves (64 output channels each) per workgroup. 5: 1280 / 320 = 4 channel chunks, 1024 workgroups at B = 64 (two
// full rounds at two per CU instead of 2.5) -- measured 64 -> 71 us per step (ten waves per CU load the four SIMDs
// 3 / 3 / 2 / 2): kept at 4.
#ifndef SPEF_X2_PWS_NWV
#define SPEF_X2_PWS_NWV 4
#endif
template <bool POOL, int NWV = 4>
__global__ __launch_bounds__(NWV * 64) void x2_pws_kernel(const float* __restrict__ X, const _Float16* __restrict__ Wt,
                                                     const float* __restrict__ bias, float* __restrict__ Y, int64_t M,
                                                     int K, int N, int Np, int Kp, int n_chunks, uint32_t nwg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  _Float16* Xh = reinterpret_cast<_Float16*>(smem);   // [64][Kp] hi halves (swizzled granules)
  _Float16* Xl = Xh + 64 * Kp;                         // [64][Kp] lo halves
  const uint32_t L = xcd_remap(blockIdx.x, nwg);
  const int chunk = (int)(L % (uint32_t)n_chunks);
  const int64_t m0 = (int64_t)(L / (uint32_t)n_chunks) * 64;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  const int n0 = chunk * (64 * NWV) + wave * 64;
  const _Float16* Wlo = Wt + (size_t)Np * Kp;
  // ---- stage: 64 rows x Kp / 8 granules, 8 fp32 -> hi / lo per piece (batches of 5 pieces per thread, loads first)
  {
    const int GP = Kp >> 3, NP = 64 * GP;
    for (int u0 = 0; u0 < NP; u0 += NWV * 64 * 5) {
      float4 v[5][2];
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const int u = u0 + tid + NWV * 64 * i;
        const int px = u / GP, g = u - px * GP;
        const int64_t p = m0 + px;
        v[i][0] = v[i][1] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (u < NP && p < M && 8 * g < K) {
          const float* xp = X + (size_t)p * K + 8 * g;
          v[i][0] = *reinterpret_cast<const float4*>(xp);
          v[i][1] = *reinterpret_cast<const float4*>(xp + 4);
        }
      }
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const int u = u0 + tid + NWV * 64 * i;
        if (u >= NP) break;
        const int px = u / GP, g = u - px * GP;
        const float f[8] = {v[i][0].x, v[i][0].y, v[i][0].z, v[i][0].w, v[i][1].x, v[i][1].y, v[i][1].z, v[i][1].w};
        f16x8 hi, lo;
        split8(f, hi, lo);
        const int o = px * Kp + 8 * (g ^ (px & 7));
        *reinterpret_cast<f16x8*>(Xh + o) = hi;
        *reinterpret_cast<f16x8*>(Xl + o) = lo;
      }
    }
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const float4 bb = *reinterpret_cast<const float4*>(bias + n0 + 16 * a + 4 * kg);
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[a][m] = f32x4{bb.x, bb.y, bb.z, bb.w};
  }
  f16x8 ah[4], al[4];
  auto load_a = [&](int k0) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const size_t off = (size_t)(n0 + 16 * a + r16) * Kp + k0 + 8 * kg;
      ah[a] = *reinterpret_cast<const f16x8*>(Wt + off);
      al[a] = *reinterpret_cast<const f16x8*>(Wlo + off);
    }
  };
  load_a(0);
  __syncthreads();
#pragma unroll 1
  for (int k0 = 0; k0 < Kp; k0 += 32) {
    f16x8 bh[4], bl[4];
    const int g = (k0 >> 3) + kg;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int px = 16 * m + r16;
      const int o = px * Kp + 8 * (g ^ (px & 7));
      bh[m] = *reinterpret_cast<const f16x8*>(Xh + o);
      bl[m] = *reinterpret_cast<const f16x8*>(Xl + o);
    }
    f16x8 ch[4], cl[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      ch[a] = ah[a];
      cl[a] = al[a];
    }
    if (k0 + 32 < Kp) load_a(k0 + 32);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[a][m] = mfma_x2(ch[a], cl[a], bh[m], bl[m], acc[a][m]);
  }
  if constexpr (POOL) {   // the 64 pixels m0 .. m0 + 63, all valid (M % 64 == 0)
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      float sm[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = 0.f;
#pragma unroll
        for (int m = 0; m < 4; ++m) t += fmaxf(acc[a][m][r], 0.f);
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) t += __shfl_xor(t, o, 64);
        sm[r] = t;
      }
      const int i = n0 + 16 * a + 4 * kg;
      if (r16 == 0 && i < N && m0 < M)   // (a workgroup's last waves may lie past M: no partial for them)
        *reinterpret_cast<float4*>(Y + (size_t)(m0 / 64) * N + i) = make_float4(sm[0], sm[1], sm[2], sm[3]);
    }
    return;
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int i = n0 + 16 * a + 4 * kg;
    if (i >= N) continue;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int64_t p = m0 + 16 * m + r16;
      if (p >= M) continue;
      const f32x4 v = acc[a][m];
      *reinterpret_cast<float4*>(Y + (size_t)p * N + i) =
          make_float4(fmaxf(v[0], 0.f), fmaxf(v[1], 0.f), fmaxf(v[2], 0.f), fmaxf(v[3], 0.f));
    }
  }
}

static bool x2_pws_ok(int Kp, int Np) {
  return SPEF_X2_PWS && Kp % 64 == 0 && Kp <= 320 && Np % 256 == 0;   // (NWV 5 falls back to 4 unless Np % 320 == 0)
}

template <bool POOL>
static hipError_t x2_pws_go(const void* x, const void* wt, const float* bias, float* y, int64_t M, int K, int N, int Np,
                            int Kp, hipStream_t s) {
  const bool five = SPEF_X2_PWS_NWV == 5 && Np % 320 == 0;
  const int n_chunks = Np / (five ? 320 : 256);
  const int64_t nwg64 = (M + 63) / 64 * n_chunks;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  const int lds = 64 * Kp * 2 * (int)sizeof(_Float16);
  static DevOnce attr_set;
  if (!attr_set.done()) {
    for (auto k : {x2_pws_kernel<POOL, 4>, x2_pws_kernel<POOL, 5>}) {
      hipError_t e = x2_set_lds(k, 64 * 320 * 2 * (int)sizeof(_Float16));   // the largest Kp
      if (e != hipSuccess) return e;
    }
    attr_set.set();
  }
  if (five)
    x2_pws_kernel<POOL, 5><<<nwg, 320, lds, s>>>((const float*)x, (const _Float16*)wt, bias, y, M, K, N, Np, Kp,
                                                 n_chunks, nwg);
  else
    x2_pws_kernel<POOL, 4><<<nwg, 256, lds, s>>>((const float*)x, (const _Float16*)wt, bias, y, M, K, N, Np, Kp,
                                                 n_chunks, nwg);
  return hipGetLastError();
}

// pooled[b][c] = (sum over the image's HW / 64 wave partials, in order) / HW
__global__ __launch_bounds__(256) void x2_pool_reduce_kernel(const float* __restrict__ part, float* __restrict__ pooled,
                                                             int B, int nblk, int N, float inv_hw) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)B * N) return;
  const int b = (int)(i / N), c = (int)(i % N);
  const float* p = part + (size_t)b * nblk * N + c;
  float t = 0.f;
  for (int j = 0; j < nblk; ++j) t += p[(size_t)j * N];
  pooled[i] = t * inv_hw;
}

hipError_t launch_x2_pw_relu(const void* x, const void* wt, const float* bias, float* y, int64_t M, int K, int N,
                             hipStream_t s) {
  if (M <= 0) return hipSuccess;
  const int Kp = (K + 31) & ~31, Np = (N + 15) & ~15;
  if ((K & 7) || (N & 3) || Np % 64) return hipErrorInvalidValue;
  if (x2_pws_ok(Kp, Np)) return x2_pws_go<false>(x, wt, bias, y, M, K, N, Np, Kp, s);
  constexpr int NT = 4, MT = 4;
  const int n_chunks = Np / (16 * NT);
  const int64_t nwg64 = (M + 64 * MT - 1) / (64 * MT) * n_chunks;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  x2_pw_kernel<NT, MT, false><<<nwg, 256, 0, s>>>((const float*)x, (const _Float16*)wt, bias, y, M, K, N, Np, Kp,
                                                  n_chunks, nwg);
  return hipGetLastError();
}

bool x2_pw_pool_supported(int HW, int N) { return HW % 64 == 0 && N % 64 == 0; }

hipError_t launch_x2_pw_pool(const void* x, const void* wt, const float* bias, float* part, float* pooled, int B,
                             int HW, int K, int N, hipStream_t s) {
  const int Kp = (K + 31) & ~31, Np = (N + 15) & ~15;
  if ((K & 7) || !x2_pw_pool_supported(HW, N) || B <= 0) return hipErrorInvalidValue;
  constexpr int NT = 4, MT = 4;
  const int64_t M = (int64_t)B * HW;
  hipError_t e;
  if (x2_pws_ok(Kp, Np)) {
    e = x2_pws_go<true>(x, wt, bias, part, M, K, N, Np, Kp, s);
  } else {
    const int n_chunks = Np / (16 * NT);
    const int64_t nwg64 = (M + 64 * MT - 1) / (64 * MT) * n_chunks;
    if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
    const uint32_t nwg = (uint32_t)nwg64;
    x2_pw_kernel<NT, MT, true><<<nwg, 256, 0, s>>>((const float*)x, (const _Float16*)wt, bias, part, M, K, N, Np, Kp,
                                                   n_chunks, nwg);
    e = hipGetLastError();
  }
  if (e != hipSuccess) return e;
  x2_pool_reduce_kernel<<<(unsigned)(((int64_t)B * N + 255) / 256), 256, 0, s>>>(part, pooled, B, HW / 64, N,
                                                                                 1.0f / (float)HW);
  return hipGetLastError();
}

}  // namespace spef
