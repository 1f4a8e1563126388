// Role-split fused INT8 inverted-residual block (QInvertedResidual, src/modeling/common/brevitas_layers.py:57-136)
// for the low-resolution MobileNet-V2 blocks 8-17 (32x32 and 16x16 maps, 384-960 hidden channels). Integer
// semantics of oracle/int8_ref.py, identical to the slab kernel (k_q8irb.hip) and the unfused k_q8.hip kernels.
//
// The slab kernel runs expand, barrier, depthwise + project on every wave in lock step, with every wave fetching the
// whole chunk's expand and project weights. Here the workgroup's waves take fixed roles and pipeline the 32-channel
// hidden chunks (the fp16 k_irw.hip structure):
//
//   expand waves    [0, NE):   chunk c+1: acc = sum q_x q_we (int8 MFMA) -> requant + ReLU -> u8 n as fp16 1024 + n
//                               -> LDS slab Es[(c+1) & 1]; they also stage the requant tables of chunk c+2
//   depthwise waves [NE, NW):  chunk c: 3x3 depthwise (exact fp32 sums of integer products) -> requant -> offset int8
//                               B fragment -> project int8 MFMA into int32 accumulators
//
// with one barrier per chunk. Every product and sum is an integer (the depthwise partial sums stay below 2^21, exact
// in fp32), so the result does not depend on the order of the sums: bit-identical to the slab and unfused schedules.
#include "spef_common.hpp"
#include "spef_kernels.hpp"
#include "q8_common.hpp"

namespace spef {

namespace {

using namespace q8;

template <int CIN, int HID, int COUT, int S, int TH, int TW, int NE, int ND>
struct QwGeom {
  static constexpr int NW = NE + ND;
  static constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3;
  static constexpr int PIN = IH * IW, PIN16 = (PIN + 15) / 16, PINP = PIN16 * 16;
  static constexpr int CINP = (CIN + 31) / 32 * 32, KSE = CINP / 32;
  static constexpr int XSB = CINP + 8;                 // Xs row stride (bytes)
  static constexpr int ES = 40;                        // hidden slab row stride (fp16 elements, 80 B)
  static constexpr int NCH = HID / 32;
  static constexpr int KPE = (CIN + 63) / 64 * 64;     // blob row length of the expand weights
  static constexpr int KPP = (HID + 63) / 64 * 64;     // blob row length of the project weights
  static constexpr int NPO = (COUT + 15) / 16 * 16, NCT = NPO / 16;
  static constexpr int EPT = (PIN16 + NE - 1) / NE;    // expand pixel tiles per expand wave
  static constexpr int POUT16 = TH * TW / 16, QPW = POUT16 / ND;
  static constexpr bool PAIR = S == 1 && TW == 16 && QPW % 2 == 0;   // a wave's tiles qi, qi+1 = rows oy, oy+1
  static constexpr int TAB = 32 * 16 * 2 + 9 * 32 * 2;   // bytes per chunk: RQ16 expand + depthwise, fp16 weights
  static constexpr int NTB = 3;                          // table buffers: chunk c (depthwise), c+1 (expand), c+2
  static constexpr int SLAB = PINP * ES * 2;
  static constexpr int LDS_BYTES = PINP * XSB + 2 * SLAB + NTB * TAB + NPO * 16;
  static_assert(HID % 32 == 0 && CIN % 8 == 0 && NCH >= 2, "channel counts");
  static_assert(POUT16 % ND == 0 && QPW >= 1, "tile split");
  static_assert(EPT <= 32, "validity mask is 32 bits");
  static_assert(NE * 64 >= 100, "one table piece per expand thread");
  static_assert(LDS_BYTES <= 163840, "LDS budget");
  static_assert(!(S == 2) || TW != 16, "stride-2 tiles use the unpaired depthwise");
};

template <int CIN, int HID, int COUT, int S, int TH, int TW, bool RES, int NE, int ND, bool SH32>
__global__ __launch_bounds__((NE + ND) * 64) void q_irw_kernel(
    const int8_t* __restrict__ X, const int8_t* __restrict__ We, const int8_t* __restrict__ Wp,
    const int32_t* __restrict__ pinit, const uint8_t* __restrict__ tabs, int64_t RM, int64_t RB, int RSH,
    int eh, int dh, int slo, int shi, int8_t* __restrict__ Y, int H, int W, int OH, int OW, int tiles_x, int tiles_y,
    uint32_t nwg) {
  using G = QwGeom<CIN, HID, COUT, S, TH, TW, NE, ND>;
  constexpr int NW = G::NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int8_t* Xs = reinterpret_cast<int8_t*>(smem);
  _Float16* Es0 = reinterpret_cast<_Float16*>(smem + G::PINP * G::XSB);       // [2][PINP][ES]
  uint8_t* Tb = reinterpret_cast<uint8_t*>(smem + G::PINP * G::XSB + 2 * G::SLAB);   // [NTB][TAB]
  RQ16* RqP = reinterpret_cast<RQ16*>(Tb + G::NTB * G::TAB);                   // [NPO]

  // table layout (spef_blob.hpp): RQ16 expand [HID] | RQ16 depthwise [HID] | RQ16 project [NPO] | fp16 [9][HID]
  const RQ16* gRqE = reinterpret_cast<const RQ16*>(tabs);
  const RQ16* gRqD = gRqE + HID;
  const RQ16* gRqP = gRqD + HID;
  const _Float16* gWd = reinterpret_cast<const _Float16*>(gRqP + G::NPO);

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  uint32_t L = xcd_remap(blockIdx.x, nwg);
  const int tx = (int)(L % (uint32_t)tiles_x);
  L /= (uint32_t)tiles_x;
  const int ty = (int)(L % (uint32_t)tiles_y);
  const int b = (int)(L / (uint32_t)tiles_y);
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;

  // chunk cc's tables: piece u < 100 of 16 B (RQ16 expand 32, RQ16 depthwise 32, fp16 weights 36)
  auto tab_src = [&](int cc, int u) -> const uint4* {
    const void* src = gRqE;
    if (u < 32) src = gRqE + 32 * cc + u;
    else if (u < 64) src = gRqD + 32 * cc + (u - 32);
    else if (u < 100) {
      const int f = (u - 64) * 8, tap = f >> 5, ch = f & 31;   // 8 fp16 weights of one tap
      src = gWd + tap * HID + 32 * cc + ch;
    }
    return reinterpret_cast<const uint4*>(src);
  };
  auto tab_buf = [&](int cc) { return Tb + (cc % G::NTB) * G::TAB; };

  // ---- 1. prologue (all waves): input tile (+halo) -> Xs, project requant records, tables of chunks 0 and 1
  {
    constexpr int GPR = G::CINP / 8, CG = CIN / 8;
    constexpr int NU = G::PINP * GPR, NIT = (NU + NW * 64 - 1) / (NW * 64);
    const int8_t* Xb = X + (size_t)b * H * W * CIN;
    long xin[NIT];
    uint32_t okm = 0;
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int u = tid + NW * 64 * i;
      const int p = u / GPR, g = u - p * GPR;
      const int py = p / G::IW, px = p - py * G::IW;
      const int iy = iy0 + py, ix = ix0 + px;
      const bool ok = u < NU && p < G::PIN && g < CG && iy >= 0 && iy < H && ix >= 0 && ix < W;
      xin[i] = *reinterpret_cast<const long*>(Xb + (ok ? ((size_t)iy * W + ix) * CIN + g * 8 : 0));
      okm |= (uint32_t)ok << i;
    }
    constexpr int NRQ = (G::NPO + NW * 64 - 1) / (NW * 64);
    RQ16 rqp[NRQ];
#pragma unroll
    for (int j = 0; j < NRQ; ++j) {
      const int u = tid + NW * 64 * j;
      rqp[j] = gRqP[u < G::NPO ? u : 0];
    }
    const int tc = tid < 100 ? 0 : 1, tu = tid < 100 ? tid : tid - 100;   // threads 0..199: tables of chunks 0, 1
    const uint4 tv = *tab_src(tc, tu < 100 ? tu : 0);
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int u = tid + NW * 64 * i;
      if (u < NU) {
        const int p = u / GPR, g = u - p * GPR;
        *reinterpret_cast<long*>(Xs + p * G::XSB + g * 8) = ((okm >> i) & 1u) ? xin[i] : 0;
      }
    }
#pragma unroll
    for (int j = 0; j < NRQ; ++j) {
      const int u = tid + NW * 64 * j;
      if (u < G::NPO) RqP[u] = rqp[j];
    }
    if (tid < 200) reinterpret_cast<uint4*>(tab_buf(tc))[tu] = tv;
  }

  if (wave < NE) {
    // =============================================================================== expand waves
    const int e = wave;
    const bool interior = iy0 >= 0 && ix0 >= 0 && iy0 + G::IH <= H && ix0 + G::IW <= W;
    uint32_t pvmask = 0;
#pragma unroll
    for (int j = 0; j < G::EPT; ++j) {
      if (interior) break;
      const int p = (e + NE * j) * 16 + r16;
      if (p < G::PIN) {
        const int py = p / G::IW, px = p - py * G::IW;
        const int iy = iy0 + py, ix = ix0 + px;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) pvmask |= 1u << j;
      }
    }
    // expand weight fragments, one chunk ahead (branch-free: the last chunk reloads itself)
    long ca0[G::KSE], ca1[G::KSE];
    auto ew_load = [&](int cc, long* a0_, long* a1_) {
      cc = cc < G::NCH ? cc : G::NCH - 1;
      const int h0 = 32 * cc + r16, h1 = 32 * cc + 16 + r16;
#pragma unroll
      for (int ks = 0; ks < G::KSE; ++ks) {
        a0_[ks] = *reinterpret_cast<const long*>(We + (size_t)h0 * G::KPE + 32 * ks + 8 * kg);
        a1_[ks] = *reinterpret_cast<const long*>(We + (size_t)h1 * G::KPE + 32 * ks + 8 * kg);
      }
    };
    // expand of chunk k -> Es[k & 1] (requant records from the chunk's table buffer)
    auto expand = [&](int k) {
      long a0[G::KSE], a1[G::KSE];
#pragma unroll
      for (int ks = 0; ks < G::KSE; ++ks) {
        a0[ks] = ca0[ks];
        a1[ks] = ca1[ks];
      }
      ew_load(k + 1, ca0, ca1);   // next chunk's fragments, in flight across this expand and the barrier
      const RQ16* rqE = reinterpret_cast<const RQ16*>(tab_buf(k));
      RQR<SH32> r0[4], r1[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        r0[r].set(rqE[4 * kg + r], 0x6400);
        r1[r].set(rqE[16 + 4 * kg + r], 0x6400);
      }
      _Float16* Es = Es0 + (k & 1) * (G::SLAB / 2);
#pragma unroll
      for (int j = 0; j < G::EPT; ++j) {
        const int pt = e + NE * j;
        if (pt >= G::PIN16) break;
        i32x4_t e0 = {0, 0, 0, 0}, e1 = {0, 0, 0, 0};
#pragma unroll
        for (int ks = 0; ks < G::KSE; ++ks) {
          const long bx = *reinterpret_cast<const long*>(Xs + (pt * 16 + r16) * G::XSB + 32 * ks + 8 * kg);
          e0 = mfma_i8(a0[ks], bx, e0);
          e1 = mfma_i8(a1[ks], bx, e1);
        }
        uint2 u0 = {expand_pair(r0[0], e0[0], r0[1], e0[1], eh), expand_pair(r0[2], e0[2], r0[3], e0[3], eh)};
        uint2 u1 = {expand_pair(r1[0], e1[0], r1[1], e1[1], eh), expand_pair(r1[2], e1[2], r1[3], e1[3], eh)};
        if (!interior && !((pvmask >> j) & 1u)) {   // pixel outside the image: the depthwise zero padding (n = 0)
          u0 = make_uint2(kF16Bias2, kF16Bias2);
          u1 = u0;
        }
        _Float16* er = Es + (pt * 16 + r16) * G::ES + 4 * kg;
        *reinterpret_cast<uint2*>(er) = u0;
        *reinterpret_cast<uint2*>(er + 16) = u1;
      }
    };
    ew_load(0, ca0, ca1);
    __syncthreads();                 // B0: input tile, tables of chunks 0 and 1, project records visible
    expand(0);
    __syncthreads();                 // B1: Es[0] visible
#pragma unroll 1
    for (int c = 0; c < G::NCH; ++c) {
      // tables of chunk c + 2 -> buffer (c + 2) % 3 (last read by the depthwise of chunk c - 1, before this period)
      const int et = e * 64 + lane;
      const bool st = c + 2 < G::NCH && et < 100;
      const uint4 tv = *tab_src(c + 2 < G::NCH ? c + 2 : c, et < 100 ? et : 0);
      if (c + 1 < G::NCH) expand(c + 1);   // into Es[(c+1) & 1]: last read by the depthwise of chunk c-1
      if (st) reinterpret_cast<uint4*>(tab_buf(c + 2))[et] = tv;
      __syncthreads();
    }
  } else {
    // =============================================================================== depthwise + project waves
    const int d = wave - NE;
    int oyq[G::QPW], oxq[G::QPW];
#pragma unroll
    for (int qi = 0; qi < G::QPW; ++qi) {
      const int o = (d * G::QPW + qi) * 16 + r16;
      oyq[qi] = o / TW;
      oxq[qi] = o - oyq[qi] * TW;
    }
    i32x4_t acc[G::QPW][G::NCT];   // project accumulators start at the offset correction 128 * sum_k q_wp
#pragma unroll
    for (int t = 0; t < G::NCT; ++t) {
      const int4 v = *reinterpret_cast<const int4*>(pinit + 16 * t + 4 * kg);
#pragma unroll
      for (int qi = 0; qi < G::QPW; ++qi) acc[qi][t] = i32x4_t{v.x, v.y, v.z, v.w};
    }
    long pa[G::NCT], pb[G::NCT];   // project fragments of the chunk being consumed / the next one
    auto load_p = [&](int cc, long (&dst)[G::NCT]) {
      cc = cc < G::NCH ? cc : G::NCH - 1;
#pragma unroll
      for (int t = 0; t < G::NCT; ++t)
        dst[t] = *reinterpret_cast<const long*>(Wp + (size_t)(16 * t + r16) * G::KPP + 32 * cc + 8 * kg);
    };
    load_p(0, pa);
    __syncthreads();                 // B0
    __syncthreads();                 // B1
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): no fragment load in flight across the loop header
    auto dw_chunk = [&](const int c, long (&pcur)[G::NCT], long (&pnext)[G::NCT]) {
      load_p(c + 1, pnext);          // in flight across this chunk's depthwise and the barrier
      const uint8_t* tb = tab_buf(c);
      const RQ16* rqD = reinterpret_cast<const RQ16*>(tb) + 32;
      const _Float16* wd = reinterpret_cast<const _Float16*>(rqD + 32);
      const _Float16* Es = Es0 + (c & 1) * (G::SLAB / 2);
      RQR<SH32> rd[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) rd[e].set(rqD[8 * kg + e], -128);
      // a8 = exact sum of (1024 + n) * w: the biased depthwise offset in rd[] removes the 1024 * sum w. Output: the
      // project MFMA's offset int8 u8 - 128 (SH32: the offset already carries the -128)
      auto bfrag = [&](const float* a8) -> long {
        uint32_t lo, hi;
        if constexpr (SH32) {
          int q[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) q[e] = med3i(rd[e].hi((int)a8[e]), -128, dh - 128);
          const uint32_t p01 = __builtin_amdgcn_perm((uint32_t)q[1], (uint32_t)q[0], 0x0c0c0400u);
          const uint32_t p23 = __builtin_amdgcn_perm((uint32_t)q[3], (uint32_t)q[2], 0x0c0c0400u);
          const uint32_t p45 = __builtin_amdgcn_perm((uint32_t)q[5], (uint32_t)q[4], 0x0c0c0400u);
          const uint32_t p67 = __builtin_amdgcn_perm((uint32_t)q[7], (uint32_t)q[6], 0x0c0c0400u);
          lo = __builtin_amdgcn_perm(p23, p01, 0x05040100u);
          hi = __builtin_amdgcn_perm(p67, p45, 0x05040100u);
        } else {
          lo = 0;
          hi = 0;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const uint32_t q = (uint32_t)med3i(rd[e].hi((int)a8[e]), 0, dh);
            if (e < 4) lo |= q << (8 * e);
            else hi |= q << (8 * (e - 4));
          }
          lo ^= 0x80808080u;
          hi ^= 0x80808080u;
        }
        return (long)(((uint64_t)hi << 32) | lo);
      };
      if constexpr (G::PAIR) {
#pragma unroll
        for (int qi = 0; qi < G::QPW; qi += 2) {
          float a0[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, a1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            f16x8 w[3], v[4];
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) w[ky] = *reinterpret_cast<const f16x8*>(wd + (ky * 3 + kx) * 32 + 8 * kg);
#pragma unroll
            for (int r = 0; r < 4; ++r)
              v[r] = *reinterpret_cast<const f16x8*>(Es + ((oyq[qi] + r) * G::IW + oxq[qi] + kx) * G::ES + 8 * kg);
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                a0[e] = fmaf((float)v[ky][e], (float)w[ky][e], a0[e]);
                a1[e] = fmaf((float)v[ky + 1][e], (float)w[ky][e], a1[e]);
              }
          }
          const long bf0 = bfrag(a0), bf1 = bfrag(a1);
#pragma unroll
          for (int t = 0; t < G::NCT; ++t) {
            acc[qi][t] = mfma_i8(pcur[t], bf0, acc[qi][t]);
            acc[qi + 1][t] = mfma_i8(pcur[t], bf1, acc[qi + 1][t]);
          }
        }
      } else {
#pragma unroll
        for (int qi = 0; qi < G::QPW; ++qi) {
          float a8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kx = 0; kx < 3; ++kx)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
              const int p = (oyq[qi] * S + ky) * G::IW + (oxq[qi] * S + kx);
              const f16x8 v = *reinterpret_cast<const f16x8*>(Es + p * G::ES + 8 * kg);
              const f16x8 w = *reinterpret_cast<const f16x8*>(wd + (ky * 3 + kx) * 32 + 8 * kg);
#pragma unroll
              for (int e = 0; e < 8; ++e) a8[e] = fmaf((float)v[e], (float)w[e], a8[e]);
            }
          const long bf = bfrag(a8);
#pragma unroll
          for (int t = 0; t < G::NCT; ++t) acc[qi][t] = mfma_i8(pcur[t], bf, acc[qi][t]);
        }
      }
      __syncthreads();
    };
#pragma unroll 1
    for (int c = 0; c + 1 < G::NCH; c += 2) {
      dw_chunk(c, pa, pb);
      dw_chunk(c + 1, pb, pa);
    }
    if constexpr (G::NCH % 2 == 1) dw_chunk(G::NCH - 1, pa, pb);

    // ---- epilogue: requant to the block's output scale (+ residual join + rescale) -> int8 NHWC
#pragma unroll
    for (int qi = 0; qi < G::QPW; ++qi) {
      const int oy = oyq[qi], ox = oxq[qi];
      const int gy = oy0 + oy, gx = ox0 + ox;
      if (gy >= OH || gx >= OW) continue;
      int8_t* yr = Y + (((size_t)b * OH + gy) * OW + gx) * COUT;
#pragma unroll
      for (int t = 0; t < G::NCT; ++t) {
        const int o = 16 * t + 4 * kg;
        if (o >= COUT) continue;
        uint32_t packed = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int q = rq_apply(acc[qi][t][r], RqP[o + r], slo, shi);
          if constexpr (RES) {
            q += (int)Xs[((oy + 1) * G::IW + (ox + 1)) * G::XSB + o + r];
            const int64_t v = ((int64_t)q * RM + RB) >> RSH;
            q = (int)(v < slo ? slo : (v > shi ? shi : v));
          }
          packed |= ((uint32_t)q & 0xffu) << (8 * r);
        }
        *reinterpret_cast<uint32_t*>(yr + o) = packed;
      }
    }
  }
}

template <int CIN, int HID, int COUT, int S, int TH, int TW, bool RES, int NE, int ND, bool SH32>
hipError_t q_irw_go(const int8_t* x, const int8_t* we, const int8_t* wp, const int32_t* pinit, const uint8_t* tabs,
                    int64_t rm, int64_t rb, int rs, QBits qb, int8_t* y, int B, int H, int W, int OH, int OW,
                    hipStream_t s) {
  if (qb.eb < 2 || qb.eb > 8 || qb.db < 2 || qb.db > 8 || qb.sb < 2 || qb.sb > 8) return hipErrorInvalidValue;
  using G = QwGeom<CIN, HID, COUT, S, TH, TW, NE, ND>;
  const int tiles_x = (OW + TW - 1) / TW, tiles_y = (OH + TH - 1) / TH;
  const int64_t nwg64 = (int64_t)tiles_x * tiles_y * B;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  auto k = q_irw_kernel<CIN, HID, COUT, S, TH, TW, RES, NE, ND, SH32>;
  static DevOnce attr_set;
  if (!attr_set.done() && G::LDS_BYTES > 65536) {
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set.set();
  }
  k<<<nwg, G::NW * 64, G::LDS_BYTES, s>>>(x, we, wp, pinit, tabs, rm, rb, rs, (1 << qb.eb) - 1, (1 << qb.db) - 1,
                                          -(1 << (qb.sb - 1)), (1 << (qb.sb - 1)) - 1, y, H, W, OH, OW, tiles_x,
                                          tiles_y, nwg);
  return hipGetLastError();
}

// (cin, hidden, cout, stride, TH, TW, residual, expand waves, depthwise waves): MobileNet-V2 blocks 8-17.
// Interleaved A/B against the slab kernel (tools/i8_ab.sh, per launch at B = 64): blocks 8-10 34.3 -> 32.8 us,
// block 11 38.1 -> 35.5, blocks 12-13 56.1 -> 49.8, block 14 46.8 -> 33.8, blocks 15-16 57.8 -> 47.6, block 17 73.8 ->
// 70.2; int8 kernel sum 1.28 -> 1.22 ms. 8x16 tiles for blocks 8-13 (512 workgroups; 134-170 VGPRs, so still one
// workgroup per CU): +3 to +5 us per launch.
#define SPEF_QIRW_TABLE(X)                                                  \
  X(64, 384, 64, 1, 16, 16, true, 4, 4)       /* blocks 8-10  */           \
  X(64, 384, 96, 1, 16, 16, false, 4, 4)      /* block 11     */           \
  X(96, 576, 96, 1, 16, 16, true, 4, 4)       /* blocks 12-13 */           \
  X(96, 576, 160, 2, 8, 8, false, 4, 4)       /* block 14     */           \
  X(160, 960, 160, 1, 8, 8, true, 4, 4)       /* blocks 15-16 */ \
  X(160, 960, 320, 1, 8, 8, false, 4, 4)      /* block 17     */

}  // namespace

bool q_irw_supported(int cin, int hid, int cout, int stride, bool res) {
#define SPEF_QIRW_HAS(CI, HI, CO, ST, TH_, TW_, RS, NE_, ND_) \
  if (cin == CI && hid == HI && cout == CO && stride == ST && res == RS) return true;
  SPEF_QIRW_TABLE(SPEF_QIRW_HAS)
#undef SPEF_QIRW_HAS
  return false;
}

hipError_t launch_q_irw(int cin, int hid, int cout, int stride, bool res, bool sh32, const int8_t* x, const int8_t* we,
                        const int8_t* wp, const int32_t* pinit, const uint8_t* tabs, int64_t rm, int64_t rb, int rs,
                        QBits qb, int8_t* y, int B, int H, int W, int OH, int OW, hipStream_t s) {
  if (!x || !we || !wp || !pinit || !tabs || !y) return hipErrorInvalidValue;
#define SPEF_QIRW_CASE(CI, HI, CO, ST, TH_, TW_, RS, NE_, ND_)                                                     \
  if (cin == CI && hid == HI && cout == CO && stride == ST && res == RS)                                           \
    return sh32 ? q_irw_go<CI, HI, CO, ST, TH_, TW_, RS, NE_, ND_, true>(x, we, wp, pinit, tabs, rm, rb, rs, qb, y, \
                                                                         B, H, W, OH, OW, s)                       \
                : q_irw_go<CI, HI, CO, ST, TH_, TW_, RS, NE_, ND_, false>(x, we, wp, pinit, tabs, rm, rb, rs, qb, y, \
                                                                          B, H, W, OH, OW, s);
  SPEF_QIRW_TABLE(SPEF_QIRW_CASE)
#undef SPEF_QIRW_CASE
  return hipErrorNotSupported;
}

}  // namespace spef
