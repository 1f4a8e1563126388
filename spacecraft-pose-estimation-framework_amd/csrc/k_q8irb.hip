// Fused INT8 inverted-residual block (QInvertedResidual, src/modeling/common/brevitas_layers.py:57-136) with
// the integer semantics of oracle/int8_ref.py, bit-exact like the unfused k_q8.hip kernels:
//
//   expand   acc = sum q_x q_we (v_mfma_i32_16x16x32_i8) -> requant + ReLU -> u8 n, kept in LDS as fp16 1024 + n
//   depthwise acc = sum (1024 + n) * q_wd over 9 taps by v_fma_mix_f32 on fp16 operands: every product and
//            partial sum is an integer below 2^21, so the fp32 accumulation is exact -> requant (offset carries
//            -1024 * M * sum q_wd, blob_q8.py) + ReLU -> u8
//   project  acc = 128 * sum q_wp + sum (u8 - 128) q_wp (int8 MFMA, unsigned operand offset by -128)
//            -> requant to the shared signed quantizer (+ residual join + rescale) -> int8
//
// Structure follows the fp16 fused kernel (k_irb.hip): the input tile + halo is staged in LDS once, the hidden
// tensor is produced 32 channels at a time into an LDS slab, the depthwise writes the project MFMA's B fragment
// directly in registers, the project accumulates in int32 MFMA accumulators over hidden chunks. Per chunk the
// workgroup stages its requant tables (RQ16 {int32 M, int32 S, int64 B}) and fp16 depthwise weights in LDS.
#include "spef_common.hpp"
#include "spef_kernels.hpp"
#include "q8_common.hpp"

namespace spef {

namespace {

using namespace q8;

template <int CIN, int HID, int COUT, int S, int TH, int TW, bool RES, int NW>
struct QGeom {
  static constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3;
  static constexpr int PIN = IH * IW, PIN16 = (PIN + 15) / 16, PINP = PIN16 * 16;
  static constexpr int CINP = (CIN + 31) / 32 * 32, KSE = CINP / 32;
  static constexpr int XSB = CINP + 8;                 // Xs row stride (bytes)
  static constexpr int ES = 40;                        // hidden slab row stride (fp16 elements, 80 B)
  static constexpr int H32 = (HID + 31) / 32 * 32, NCH = H32 / 32;
  static constexpr int KPE = (CIN + 63) / 64 * 64;     // blob row length of the expand weights
  static constexpr int KPP = (HID + 63) / 64 * 64;     // blob row length of the project weights
  static constexpr int NPO = (COUT + 15) / 16 * 16, NCT = NPO / 16;
  static constexpr int EPT = (PIN16 + NW - 1) / NW;
  static constexpr int POUT16 = TH * TW / 16, QPW = POUT16 / NW;
  // depthwise row pairs: a wave's consecutive pixel tiles are vertically adjacent rows (16-wide, stride 1)
  static constexpr bool PAIR = S == 1 && TW == 16 && QPW % 2 == 0;
  static constexpr int TAB = 32 * 16 * 2 + 9 * 32 * 2;   // bytes per chunk: RQ16 expand + depthwise, fp16 weights
  static constexpr int LDS_BYTES = PINP * XSB + PINP * ES * 2 + 2 * TAB + NPO * 16;
  static_assert(POUT16 % NW == 0, "tile split");
  static_assert(EPT <= 32, "validity mask is 32 bits");
  static_assert(LDS_BYTES <= 163840, "LDS budget");
  static_assert(!RES || (S == 1 && CIN == COUT), "residual geometry");
};

template <int CIN, int HID, int COUT, int S, int TH, int TW, bool RES, int NW, bool EXPAND, bool SH32>
__global__ __launch_bounds__(NW * 64) void q_irb_kernel(
    const int8_t* __restrict__ X, const int8_t* __restrict__ We, const int8_t* __restrict__ Wp,
    const int32_t* __restrict__ pinit, const uint8_t* __restrict__ tabs, int64_t RM, int64_t RB, int RSH,
    int eh, int dh, int slo, int shi, int8_t* __restrict__ Y, int H, int W, int OH, int OW, int tiles_x, int tiles_y,
    uint32_t nwg) {
  // eh, dh: top levels of the expand / depthwise ReLU quantizers (2^b - 1); [slo, shi]: the shared signed quantizer
  using G = QGeom<CIN, HID, COUT, S, TH, TW, RES, NW>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // t == 1 without residual (block 1) never reads an int8 input copy: no Xs region, more workgroups per CU
  constexpr int XREG = (EXPAND || RES) ? G::PINP * G::XSB : 0;
  int8_t* Xs = reinterpret_cast<int8_t*>(smem);
  _Float16* Es = reinterpret_cast<_Float16*>(smem + XREG);
  uint8_t* Tb = reinterpret_cast<uint8_t*>(Es + G::PINP * G::ES);          // [2][TAB]
  RQ16* RqP = reinterpret_cast<RQ16*>(Tb + 2 * G::TAB);                      // [NPO]

  // x2 table layout (spef_blob.hpp): RQ16 expand [H32] | RQ16 depthwise [H32] | RQ16 project [NPO] | fp16 [9][H32]
  const RQ16* gRqE = reinterpret_cast<const RQ16*>(tabs);
  const RQ16* gRqD = gRqE + G::H32;
  const RQ16* gRqP = gRqD + G::H32;
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

  // per-chunk tables -> LDS buffer (cc & 1): 16-B pieces, RQ16 expand (32), RQ16 depthwise (32), weights (36); one
  // piece per thread. Loads are branch-free and issued a chunk ahead of their store: a load under a condition, or
  // one stored right away, is waited for at once (a full memory round trip per chunk).
  static_assert(NW * 64 >= 100, "one table piece per thread");
  auto tab_load = [&](int cc) -> uint4 {
    const int u = tid;
    const void* src = gRqE;
    if (u < 32) src = gRqE + 32 * cc + u;
    else if (u < 64) src = gRqD + 32 * cc + (u - 32);
    else if (u < 100) {
      const int f = (u - 64) * 8, tap = f >> 5, ch = f & 31;   // 8 fp16 weights of one tap
      src = gWd + tap * G::H32 + 32 * cc + ch;
    }
    return *reinterpret_cast<const uint4*>(src);
  };
  auto tab_store = [&](int cc, uint4 v) {
    if (tid < 100) reinterpret_cast<uint4*>(Tb + (cc & 1) * G::TAB)[tid] = v;
  };

  // ---- 1. input tile (+halo) -> LDS (int8; zero outside the image and in the K padding), tables of chunk 0
  {
    constexpr int GPR = G::CINP / 8, CG = CIN / 8;
    constexpr int NU = G::PINP * GPR, NIT = (NU + NW * 64 - 1) / (NW * 64);
    const int8_t* Xb = X + (size_t)b * H * W * CIN;
    // every prologue load issued branch-free before the first LDS store (see tab_load)
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
    const uint4 tab0 = tab_load(0);
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int u = tid + NW * 64 * i;
      if (u < NU) {
        const int p = u / GPR, g = u - p * GPR;
        const long v = ((okm >> i) & 1u) ? xin[i] : 0;
        if constexpr (EXPAND) {
          *reinterpret_cast<long*>(Xs + p * G::XSB + g * 8) = v;
        } else {   // t == 1 (block 1): the hidden tensor is the u8 input itself, straight into the slab as fp16 1024 + n
          const uint32_t lo = (uint32_t)v, hi = (uint32_t)((uint64_t)v >> 32);
          uint4 o;
          o.x = (lo & 0xffu) | ((lo & 0xff00u) << 8) | kF16Bias2;
          o.y = ((lo >> 16) & 0xffu) | ((lo >> 8) & 0xff0000u) | kF16Bias2;
          o.z = (hi & 0xffu) | ((hi & 0xff00u) << 8) | kF16Bias2;
          o.w = ((hi >> 16) & 0xffu) | ((hi >> 8) & 0xff0000u) | kF16Bias2;
          *reinterpret_cast<uint4*>(Es + p * G::ES + 8 * g) = o;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NRQ; ++j) {
      const int u = tid + NW * 64 * j;
      if (u < G::NPO) RqP[u] = rqp[j];
    }
    tab_store(0, tab0);
  }

  // validity of this lane's expand pixels (inside the image): the depthwise zero padding. Interior tiles (whole
  // input tile inside the image) need no mask (workgroup-uniform branch).
  const bool interior = iy0 >= 0 && ix0 >= 0 && iy0 + G::IH <= H && ix0 + G::IW <= W;
  uint32_t pvmask = 0;
#pragma unroll
  for (int j = 0; j < G::EPT; ++j) {
    if (interior) break;
    const int p = (wave + NW * j) * 16 + r16;
    if (p < G::PIN) {
      const int py = p / G::IW, px = p - py * G::IW;
      const int iy = iy0 + py, ix = ix0 + px;
      if (iy >= 0 && iy < H && ix >= 0 && ix < W) pvmask |= 1u << j;
    }
  }
  int oyq[G::QPW], oxq[G::QPW];
#pragma unroll
  for (int qi = 0; qi < G::QPW; ++qi) {
    const int o = (wave * G::QPW + qi) * 16 + r16;
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
  __syncthreads();

  // expand weight fragments prefetched one chunk ahead (branch-free: rows past HID reload a valid row and are zeroed
  // at use)
  long ca0[G::KSE], ca1[G::KSE];
  auto ew_load = [&](int cc, long* a0_, long* a1_) {
    cc = cc < G::NCH ? cc : G::NCH - 1;
    const int h0 = 32 * cc + r16 < HID ? 32 * cc + r16 : r16, h1 = 32 * cc + 16 + r16 < HID ? 32 * cc + 16 + r16 : r16;
#pragma unroll
    for (int ks = 0; ks < G::KSE; ++ks) {
      a0_[ks] = *reinterpret_cast<const long*>(We + (size_t)h0 * G::KPE + 32 * ks + 8 * kg);
      a1_[ks] = *reinterpret_cast<const long*>(We + (size_t)h1 * G::KPE + 32 * ks + 8 * kg);
    }
  };
  if constexpr (EXPAND) ew_load(0, ca0, ca1);

#pragma unroll 1
  for (int c = 0; c < G::NCH; ++c) {
    const uint4 tab_next = tab_load(c + 1 < G::NCH ? c + 1 : c);   // stored after this chunk's depthwise
    const uint8_t* tb = Tb + (c & 1) * G::TAB;
    const RQ16* rqE = reinterpret_cast<const RQ16*>(tb);
    const RQ16* rqD = rqE + 32;
    const _Float16* wd = reinterpret_cast<const _Float16*>(rqD + 32);
    // project weight fragments of this chunk, in flight across the expand
    long pa[G::NCT];
#pragma unroll
    for (int t = 0; t < G::NCT; ++t)
      pa[t] = *reinterpret_cast<const long*>(Wp + (size_t)(16 * t + r16) * G::KPP + 32 * c + 8 * kg);
    if (c > 0) __syncthreads();   // every wave's depthwise reads of the previous chunk's slab are done

    // ---- 2. expand (32 hidden channels) -> requant -> u8 as fp16 in the slab. t == 1 (block 1): the hidden
    // tensor is the unsigned stem output itself, converted to fp16 (zero outside the image from the staging).
    if constexpr (!EXPAND) {
      static_assert(HID == 32 && CIN == 32, "t == 1 is MobileNet-V2 block 1");   // slab filled by the prologue
    } else {
      long a0[G::KSE], a1[G::KSE], na0[G::KSE], na1[G::KSE];
      const int h0 = 32 * c + r16, h1 = 32 * c + 16 + r16;
      ew_load(c + 1, na0, na1);   // next chunk's fragments, in flight across this chunk
#pragma unroll
      for (int ks = 0; ks < G::KSE; ++ks) {
        a0[ks] = h0 < HID ? ca0[ks] : 0;
        a1[ks] = h1 < HID ? ca1[ks] : 0;
        ca0[ks] = na0[ks];
        ca1[ks] = na1[ks];
      }
      RQR<SH32> r0[4], r1[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        r0[r].set(rqE[4 * kg + r], 0x6400);
        r1[r].set(rqE[16 + 4 * kg + r], 0x6400);
      }
#pragma unroll
      for (int j = 0; j < G::EPT; ++j) {
        const int pt = wave + NW * j;
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
    }
    __syncthreads();   // slab and this chunk's tables visible

    // ---- 3. depthwise (exact fp32 sums of integer products) -> requant -> offset int8 B fragment; 4. project
    {
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
        // Two vertically adjacent output rows per step (tiles qi, qi+1 = rows oy, oy+1 of the same 16 columns): per
        // tap column the 3 weights and the 4 input rows are read once and feed both rows (21 instead of 36
        // ds_read_b128 per 2 x 16 pixels x 8 channels), as in the fp16 kernel
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
            acc[qi][t] = mfma_i8(pa[t], bf0, acc[qi][t]);
            acc[qi + 1][t] = mfma_i8(pa[t], bf1, acc[qi + 1][t]);
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
          for (int t = 0; t < G::NCT; ++t) acc[qi][t] = mfma_i8(pa[t], bf, acc[qi][t]);
        }
      }
    }
    if (c + 1 < G::NCH) tab_store(c + 1, tab_next);   // buffer (c+1)&1 was last read in chunk c-1
  }

  // ---- 5. epilogue: requant to the block's output scale (+ residual join + rescale) -> int8 NHWC
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

template <int CIN, int HID, int COUT, int S, int TH, int TW, bool RES, int NW, bool EXPAND, bool SH32>
hipError_t q_irb_go(const int8_t* x, const int8_t* we, const int8_t* wp, const int32_t* pinit, const uint8_t* tabs,
                    int64_t rm, int64_t rb, int rs, QBits qb, int8_t* y, int B, int H, int W, int OH, int OW,
                    hipStream_t s) {
  if (qb.eb < 2 || qb.eb > 8 || qb.db < 2 || qb.db > 8 || qb.sb < 2 || qb.sb > 8) return hipErrorInvalidValue;
  using G = QGeom<CIN, HID, COUT, S, TH, TW, RES, NW>;
  const int tiles_x = (OW + TW - 1) / TW, tiles_y = (OH + TH - 1) / TH;
  const int64_t nwg64 = (int64_t)tiles_x * tiles_y * B;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  auto k = q_irb_kernel<CIN, HID, COUT, S, TH, TW, RES, NW, EXPAND, SH32>;
  constexpr int lds = G::LDS_BYTES - ((EXPAND || RES) ? 0 : G::PINP * G::XSB);   // see XREG in the kernel
  static DevOnce attr_set;
  if (!attr_set.done() && lds > 65536) {
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr_set.set();
  }
  k<<<nwg, NW * 64, lds, s>>>(x, we, wp, pinit, tabs, rm, rb, rs, (1 << qb.eb) - 1, (1 << qb.db) - 1,
                              -(1 << (qb.sb - 1)), (1 << (qb.sb - 1)) - 1, y, H, W, OH, OW, tiles_x, tiles_y, nwg);
  return hipGetLastError();
}

// (cin, hidden, cout, stride, TH, TW, residual, waves) for MobileNet-V2 blocks 2-17
#define SPEF_QIRB_TABLE(X)                                                              \
  X(32, 32, 16, 1, 16, 16, false, 8, false)     /* block 1 (t = 1) */                  \
  X(16, 96, 24, 2, 4, 16, false, 4, true)       /* block 2      */                     \
  X(24, 144, 24, 1, 8, 16, true, 4, true)       /* block 3      */                     \
  X(24, 144, 32, 2, 8, 8, false, 4, true)       /* block 4      */                     \
  X(32, 192, 32, 1, 8, 16, true, 4, true)       /* blocks 5-6   */                     \
  X(32, 192, 64, 2, 8, 8, false, 4, true)       /* block 7      */                     \
  X(64, 384, 64, 1, 8, 16, true, 4, true)       /* blocks 8-10  */                     \
  X(64, 384, 96, 1, 8, 16, false, 4, true)      /* block 11     */                     \
  X(96, 576, 96, 1, 8, 16, true, 4, true)       /* blocks 12-13 */                     \
  X(96, 576, 160, 2, 4, 8, false, 2, true)      /* block 14     */                     \
  X(160, 960, 160, 1, 4, 8, true, 2, true)      /* blocks 15-16 */                     \
  X(160, 960, 320, 1, 4, 8, false, 2, true)     /* block 17     */

}  // namespace

bool q_irb_supported(int cin, int hid, int cout, int stride, bool res, bool expand) {
#define SPEF_QIRB_HAS(CI, HI, CO, ST, TH_, TW_, RS, NW_, EX) \
  if (cin == CI && hid == HI && cout == CO && stride == ST && res == RS && expand == EX) return true;
  SPEF_QIRB_TABLE(SPEF_QIRB_HAS)
#undef SPEF_QIRB_HAS
  return false;
}

hipError_t launch_q_irb(int cin, int hid, int cout, int stride, bool res, bool expand, bool sh32, const int8_t* x,
                        const int8_t* we, const int8_t* wp, const int32_t* pinit, const uint8_t* tabs, int64_t rm,
                        int64_t rb, int rs, QBits qb, int8_t* y, int B, int H, int W, int OH, int OW, hipStream_t s) {
#define SPEF_QIRB_CASE(CI, HI, CO, ST, TH_, TW_, RS, NW_, EX)                                                         \
  if (cin == CI && hid == HI && cout == CO && stride == ST && res == RS && expand == EX)                                \
    return sh32 ? q_irb_go<CI, HI, CO, ST, TH_, TW_, RS, NW_, EX, true>(x, we, wp, pinit, tabs, rm, rb, rs, qb, y, B,  \
                                                                        H, W, OH, OW, s)                                \
                : q_irb_go<CI, HI, CO, ST, TH_, TW_, RS, NW_, EX, false>(x, we, wp, pinit, tabs, rm, rb, rs, qb, y, B, \
                                                                         H, W, OH, OW, s);
  SPEF_QIRB_TABLE(SPEF_QIRB_CASE)
#undef SPEF_QIRB_CASE
  return hipErrorNotSupported;
}

}  // namespace spef
