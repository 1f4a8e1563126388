// Front kernel: stem ConvBnAct 3->32 3x3/s2 (mobilenet_v2.py:252-254) fused with inverted-residual block 1
// (t=1: depthwise 3x3 32ch + BN + ReLU -> project 32->16 + BN; pytorch_layers.py:65-98), uint8 NHWC frames in.
//
// The 32-channel 256x256 stem map (the largest activation of the network) never reaches HBM: per 16x16 block-1
// output tile the kernel stages the 37x37x3 input bytes in LDS, computes the 18x18 stem tile (+1 halo for the
// depthwise) on MFMA, keeps it in LDS, and runs the block-1 depthwise + project from there.
//
// Stem on MFMA: K = 27 taps (ky, kx, ci) padded to 32, A = weights [32 ch][k], B = image patch [k][pixel].
// uint8 pixels are exact in fp16/bf16; ToTensor's /255 is folded into the weights, which are split into
// hi + lo halves (w = hi + lo, two MFMAs) so the stem keeps ~fp32 weight precision.
#include "spef_common.hpp"
#include "spef_kernels.hpp"

namespace spef {

template <typename DT, int TH, int TW, int NW>
__global__ __launch_bounds__(NW * 64) void front_kernel(
    const uint8_t* __restrict__ X, const typename DT::T* __restrict__ wsp, const float* __restrict__ bs,
    const typename DT::DW* __restrict__ Wd, const float* __restrict__ bd, const typename DT::T* __restrict__ Wp,
    const float* __restrict__ bp, typename DT::T* __restrict__ Y, int H, int W, int SH_img, int SW_img,
    int tiles_x, int tiles_y, uint32_t nwg) {
  using T = typename DT::T;
  using x8 = typename DT::x8;
  using x4 = typename DT::x4;
  constexpr int SH = TH + 2, SW = TW + 2;          // stem tile (block-1 output tile + depthwise halo)
  constexpr int IH = 2 * SH + 1, IW = 2 * SW + 1;  // input tile
  constexpr int IRS = ((IW * 3 + 3) / 4 * 4 + 4 + 15) / 16 * 16;   // input LDS row stride (bytes)
  constexpr int PS = SH * SW, PS16 = (PS + 15) / 16, PSP = PS16 * 16;
  constexpr int XS = 48;                           // stem-map row stride: 96 B, conflict-free b128 reads
  constexpr int POUT16 = TH * TW / 16, QPW = POUT16 / NW;
  static_assert(POUT16 % NW == 0, "tile split");
  __shared__ __attribute__((aligned(16))) uint8_t In[IH * IRS];
  __shared__ __attribute__((aligned(16))) T Xs[PSP * XS];
  using DW = typename DT::DW;
  __shared__ __attribute__((aligned(16))) DW Sl[9 * 32];     // block-1 depthwise weights
  __shared__ __attribute__((aligned(16))) float Sb[32];      // block-1 depthwise bias

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  uint32_t L = xcd_remap(blockIdx.x, nwg);
  const int tx = (int)(L % (uint32_t)tiles_x);
  L /= (uint32_t)tiles_x;
  const int ty = (int)(L % (uint32_t)tiles_y);
  const int b = (int)(L / (uint32_t)tiles_y);
  const int oy0 = ty * TH, ox0 = tx * TW;            // block-1 output (= stem output) coordinates
  const int sy0 = oy0 - 1, sx0 = ox0 - 1;            // stem tile origin
  const int iy0 = 2 * sy0 - 1, ix0 = 2 * sx0 - 1;    // input tile origin

  // ---- 1. input bytes -> LDS (zero outside the image = the stem's padding). Each input row is a contiguous
  // IW*3-byte run of the NHWC frame, fetched as aligned dwords with ALL of a thread's loads issued before any
  // LDS store. Interior tiles (every column inside the image, W % 4 == 0) copy the dwords as they are and the
  // reader offsets by the common misalignment `mis`; edge tiles scatter bytes and zero the outside columns.
  int mis = 0;
  {
    // Half a wave per input row (lane & 31 = dword k of the row, rows 2 (wave + NW i) + (lane >> 5)): no
    // divisions, and 32-bit in-frame byte offsets (the launcher checks H * W * 3 < 2^31).
    constexpr int RB = IW * 3;                        // bytes per input-tile row
    constexpr int DPR = (RB + 3) / 4 + 1;             // dwords covering a row at any byte alignment
    constexpr int NIT = (IH + 2 * NW - 1) / (2 * NW);
    static_assert(4 * DPR <= IRS && DPR <= 32, "LDS row holds the dword-aligned run; one half-wave per row");
    const uint8_t* Xb = X + (size_t)b * H * W * 3;
    const int img_bytes = H * W * 3;
    const int k = lane & 31;
    const bool fast = (W & 3) == 0 && ix0 >= 0 && ix0 + IW <= W;
    uint32_t v[NIT];
    int a[NIT], rs[NIT];
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int r = 2 * (wave + NW * i) + (lane >> 5);
      const int iy = iy0 + r;
      rs[i] = (iy * W + ix0) * 3;
      a[i] = (rs[i] & ~3) + 4 * k;
      v[i] = 0;
      if (r < IH && k < DPR && iy >= 0 && iy < H && a[i] >= 0) {
        if (a[i] + 4 <= img_bytes) {
          v[i] = *reinterpret_cast<const uint32_t*>(Xb + a[i]);
        } else {
          for (int j = 0; j < 4; ++j)
            if (a[i] + j < img_bytes) v[i] |= (uint32_t)Xb[a[i] + j] << (8 * j);
        }
      }
    }
    if (fast) {
      mis = ((iy0 * W + ix0) * 3) & 3;   // the same for every row when W % 4 == 0
#pragma unroll
      for (int i = 0; i < NIT; ++i) {
        const int r = 2 * (wave + NW * i) + (lane >> 5);
        if (r < IH && k < DPR) *reinterpret_cast<uint32_t*>(In + r * IRS + 4 * k) = v[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < NIT; ++i) {
        const int r = 2 * (wave + NW * i) + (lane >> 5);
        if (r >= IH || k >= DPR) continue;
        const int iy = iy0 + r;
        const bool row_ok = iy >= 0 && iy < H;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int o = a[i] + j - rs[i];               // byte offset inside the tile row
          if (o < 0 || o >= RB) continue;
          const int ix = ix0 + o / 3;
          In[r * IRS + o] = (row_ok && ix >= 0 && ix < W) ? (uint8_t)(v[i] >> (8 * j)) : (uint8_t)0;
        }
      }
    }
    for (int u = tid; u < 9 * 32 + 32; u += NW * 64) {
      if (u < 9 * 32) Sl[u] = Wd[u];
      else Sb[u - 9 * 32] = bd[u - 9 * 32];
    }
  }
  // stem weight fragments: /255-folded weights split hi + lo, [2][32 ch][32 k] from the blob; tiles t = 0, 1
  x8 ahi[2], alo[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    ahi[t] = load8<DT>(wsp + (16 * t + r16) * 32 + 8 * kg);
    alo[t] = load8<DT>(wsp + 32 * 32 + (16 * t + r16) * 32 + 8 * kg);
  }
  const float4 sb0 = *reinterpret_cast<const float4*>(bs + 4 * kg);
  const float4 sb1 = *reinterpret_cast<const float4*>(bs + 16 + 4 * kg);
  // per-lane tap offsets inside the input tile for k = 8kg + e: (k / 9) * IRS + k % 9. The K padding slots
  // k = 27..31 have zero weights, so they may read any finite byte (offset 0): no per-tap select.
  int koff[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 8 * kg + e;
    koff[e] = k < 27 ? (k / 9) * IRS + (k % 9) : 0;
  }
  // interior tiles: every stem position of the tile lies inside the stem map (no zero padding to apply)
  const bool interior = sy0 >= 0 && sx0 >= 0 && sy0 + SH <= SH_img && sx0 + SW <= SW_img;
  __syncthreads();

  // ---- 2. stem tile on MFMA -> Xs (fp16/bf16, ReLU; zero outside the stem map = block-1 depthwise padding)
  for (int pt = wave; pt < PS16; pt += NW) {
    const int p = pt * 16 + r16;
    const int pc = p < PS ? p : PS - 1;             // padding lanes of the last tile: any in-tile address
    const int spy = pc / SW, spx = pc - spy * SW;
    const int base = (2 * spy) * IRS + 2 * spx * 3 + mis;
    x8 bx;
#pragma unroll
    for (int e = 0; e < 8; ++e) bx[e] = (T)(float)In[base + koff[e]];
    f32x4 e0 = {sb0.x, sb0.y, sb0.z, sb0.w}, e1 = {sb1.x, sb1.y, sb1.z, sb1.w};   // bias as MFMA C
    e0 = DT::mfma(ahi[0], bx, e0);
    e0 = DT::mfma(alo[0], bx, e0);
    e1 = DT::mfma(ahi[1], bx, e1);
    e1 = DT::mfma(alo[1], bx, e1);
    const x4 o0 = relu_cvt4<DT>(e0), o1 = relu_cvt4<DT>(e1);   // packed convert + ReLU (fp16)
    uint2 u0 = __builtin_bit_cast(uint2, o0), u1 = __builtin_bit_cast(uint2, o1);
    if (!interior) {
      const int gy = sy0 + spy, gx = sx0 + spx;
      const uint32_t m = (gy >= 0 && gy < SH_img && gx >= 0 && gx < SW_img) ? 0xffffffffu : 0u;
      u0.x &= m; u0.y &= m; u1.x &= m; u1.y &= m;
    }
    if (p < PS) {
      *reinterpret_cast<uint2*>(Xs + p * XS + 4 * kg) = u0;
      *reinterpret_cast<uint2*>(Xs + p * XS + 16 + 4 * kg) = u1;
    }
  }
  __syncthreads();

  // ---- 3. block 1: depthwise 3x3 (32 ch) -> project 32 -> 16 (+BN)
  const x8 pa = load8<DT>(Wp + (size_t)r16 * 32 + 8 * kg);
  const float4 pb = *reinterpret_cast<const float4*>(bp + 4 * kg);
  auto store = [&](int oy, int ox, const f32x4& acc) {
    const int gy = oy0 + oy, gx = ox0 + ox;
    if (gy < SH_img && gx < SW_img) {
      x4 out;
      out[0] = (T)acc[0];
      out[1] = (T)acc[1];
      out[2] = (T)acc[2];
      out[3] = (T)acc[3];
      *reinterpret_cast<x4*>(Y + (((size_t)b * SH_img + gy) * SW_img + gx) * 16 + 4 * kg) = out;
    }
  };
  if constexpr (TW == 16 && QPW % 2 == 0) {
    // Two vertically adjacent output rows per step (a wave's tiles qi, qi+1 are rows oy, oy+1 of the same 16
    // columns): per tap column the 3 weights and 4 stem rows are read once and feed both rows -- 21 instead of 36
    // ds_read_b128 per 2 x 16 pixels x 8 channels. Same tap order (kx outer, ky inner) as the one-row loop.
#pragma unroll
    for (int qi = 0; qi < QPW; qi += 2) {
      const int oy = wave * QPW + qi, ox = r16;
      const T* xb = Xs + (oy * SW + ox) * XS + 8 * kg;   // tap (r, kx) at a constant offset: ds_read immediates
      float a0[8], a1[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) a0[e] = a1[e] = Sb[8 * kg + e];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        DW8<DT> w[3];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) w[ky].load(Sl + (ky * 3 + kx) * 32 + 8 * kg);
        x8 v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = *reinterpret_cast<const x8*>(xb + (r * SW + kx) * XS);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            a0[e] = fmaf((float)v[ky][e], w[ky][e], a0[e]);
            a1[e] = fmaf((float)v[ky + 1][e], w[ky][e], a1[e]);
          }
      }
      const x8 bf0 = relu_cvt8<DT>(a0), bf1 = relu_cvt8<DT>(a1);
      f32x4 acc0 = {pb.x, pb.y, pb.z, pb.w}, acc1 = acc0;   // bias as MFMA C (same order as the block kernels)
      acc0 = DT::mfma(pa, bf0, acc0);
      acc1 = DT::mfma(pa, bf1, acc1);
      store(oy, ox, acc0);
      store(oy + 1, ox, acc1);
    }
    return;
  }
#pragma unroll
  for (int qi = 0; qi < QPW; ++qi) {
    const int o = (wave * QPW + qi) * 16 + r16;
    const int oy = o / TW, ox = o - (o / TW) * TW;
    float a8[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) a8[e] = Sb[8 * kg + e];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const x8 v = *reinterpret_cast<const x8*>(Xs + ((oy + ky) * SW + (ox + kx)) * XS + 8 * kg);
        DW8<DT> wt;
        wt.load(Sl + (ky * 3 + kx) * 32 + 8 * kg);
#pragma unroll
        for (int e = 0; e < 8; ++e) a8[e] = fmaf((float)v[e], wt[e], a8[e]);
      }
    const x8 bf = relu_cvt8<DT>(a8);
    f32x4 acc = {pb.x, pb.y, pb.z, pb.w};      // bias as MFMA C (same order as the block kernels)
    acc = DT::mfma(pa, bf, acc);
    store(oy, ox, acc);
  }
}

// fp16 front kernel with the vertical-pair block-1 depthwise (k_irb.hip, VP) and a gather-free stem.
//  * Input staging as above (bytes -> In), then one pass re-lays the tile out as Lr[stem row][col dword][ky]:
//    dword (cd, ky) = the two input bytes 2cd, 2cd+1 of input row 2*spy+ky as exact fp16. A stem pixel's 27 taps are
//    then 15 consecutive dwords (5 column dwords x 3 rows; the 16th is a zero-weight pad), so an MFMA B fragment is
//    4 dword reads at immediate offsets -- no per-tap byte gathers, address arithmetic or conversions (the blob's
//    fp16 stem operand is packed in this k order, blob.py).
//  * The stem runs in units of 16 (row pair, column) positions: the even- and odd-row pixel of each position are
//    two MFMA tiles whose outputs are stored as row-pair dwords, i.e. the block-1 depthwise input in VP layout.
//  * Block 1's depthwise takes two taps per v_dot2_f32_f16 (6 instead of 9 VALU per 3x3), two output rows per step.
// 374 instead of 457 VALU per wave (PMC), but only -2 % time: the kernel is bound by its staging latency and HBM
// traffic as much as by VALU issue. A persistent variant (tiles per workgroup, next tile's bytes prefetched during
// the stem) needed 106-122 VGPRs (2 workgroups per CU) and was slower at every tiles-per-workgroup setting
// (125-172 us; spilling versions at 6-8 waves per SIMD 200-330 us; measured with a one-kernel timing harness).
template <int TH, int TW, int NW>
__global__ __launch_bounds__(NW * 64) void front_vp_kernel(
    const uint8_t* __restrict__ X, const _Float16* __restrict__ wsp, const float* __restrict__ bs,
    const _Float16* __restrict__ Wd, const float* __restrict__ bd, const _Float16* __restrict__ Wp,
    const float* __restrict__ bp, _Float16* __restrict__ Y, int H, int W, int SH_img, int SW_img,
    int tiles_x, int tiles_y, uint32_t nwg) {
  using DT = F16;
  using T = _Float16;
  using x8 = f16x8;
  using x4 = f16x4;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  constexpr int SH = TH + 2, SW = TW + 2;          // stem tile (block-1 output tile + depthwise halo)
  constexpr int IH = 2 * SH + 1, IW = 2 * SW + 1;  // input tile
  constexpr int IRS = ((IW * 3 + 3) / 4 * 4 + 4 + 15) / 16 * 16;   // input LDS row stride (bytes)
  constexpr int NCD = 3 * SW + 3;                  // column dwords per Lr row (last stem pixel's pad dword included)
  constexpr int RSL = 3 * NCD;                     // dwords per stem row of Lr
  constexpr int PR = SH / 2, NQ = PR * SW, NU = (NQ + 15) / 16, NQP = NU * 16;
  constexpr int RSB = NQP * 32 + 16;               // bytes per channel-group region of the pair slab
  constexpr int EPU = (NU + NW - 1) / NW;
  constexpr int POUT16 = TH * TW / 16, QPW = POUT16 / NW;
  static_assert(SH % 2 == 0 && TW == 16 && QPW == 2 && NCD <= 64, "geometry");
  __shared__ __attribute__((aligned(16))) uint8_t In[IH * IRS];
  __shared__ __attribute__((aligned(16))) uint32_t Lr[SH * RSL + 4];
  __shared__ __attribute__((aligned(16))) char Ps[4 * RSB];
  __shared__ __attribute__((aligned(16))) uint32_t Sv[3 * 64];   // block-1 dw weight pairs [kx][(w0,w1)|(w1,w2)][32]
  __shared__ __attribute__((aligned(16))) float Sb[32];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  uint32_t L = xcd_remap(blockIdx.x, nwg);
  const int tx = (int)(L % (uint32_t)tiles_x);
  L /= (uint32_t)tiles_x;
  const int ty = (int)(L % (uint32_t)tiles_y);
  const int b = (int)(L / (uint32_t)tiles_y);
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int sy0 = oy0 - 1, sx0 = ox0 - 1;
  const int iy0 = 2 * sy0 - 1, ix0 = 2 * sx0 - 1;

  // ---- 1. input bytes -> Lr (interior tiles) or In (edge tiles, as front_kernel), dw weight pairs, biases
  const bool fast = (W & 3) == 0 && ix0 >= 0 && ix0 + IW <= W;
  {
    constexpr int RB = IW * 3;
    constexpr int DPR = (RB + 3) / 4 + 1;
    constexpr int NIT = (IH + 2 * NW - 1) / (2 * NW);
    static_assert(4 * DPR <= IRS && DPR <= 32, "LDS row holds the dword-aligned run; one half-wave per row");
    const uint8_t* Xb = X + (size_t)b * H * W * 3;
    const int img_bytes = H * W * 3;
    const int k = lane & 31;
    uint32_t v[NIT];
    int a[NIT], rs[NIT];
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int r = 2 * (wave + NW * i) + (lane >> 5);
      const int iy = iy0 + r;
      rs[i] = (iy * W + ix0) * 3;
      a[i] = (rs[i] & ~3) + 4 * k;
      v[i] = 0;
      if (r < IH && k < DPR && iy >= 0 && iy < H && a[i] >= 0) {
        if (a[i] + 4 <= img_bytes) {
          v[i] = *reinterpret_cast<const uint32_t*>(Xb + a[i]);
        } else {
          for (int j = 0; j < 4; ++j)
            if (a[i] + j < img_bytes) v[i] |= (uint32_t)Xb[a[i] + j] << (8 * j);
        }
      }
    }
    // dw weight pairs: the last wave's threads 0..47 (kx = t / 16, pair (ky, ky+1), ky = (t / 8) % 2, 4 channels)
    const int vt = NW * 64 - 1 - tid;
    uint2 wa = make_uint2(0, 0), wb = make_uint2(0, 0);
    if (vt < 48) {
      const int kx = vt >> 4, ky = (vt >> 3) & 1, ch = 4 * (vt & 7);
      wa = *reinterpret_cast<const uint2*>(Wd + (ky * 3 + kx) * 32 + ch);
      wb = *reinterpret_cast<const uint2*>(Wd + ((ky + 1) * 3 + kx) * 32 + ch);
    }
    if (fast) {
      // interior tiles: the rows go straight to Lr. Every row starts 3 bytes into its aligned dword (W % 4 == 0,
      // ix0 = 32 tx - 3), so lane k holds tile bytes 4k-3 .. 4k: column dword 2k-1 = its bytes 1, 2 and column
      // dword 2k = its byte 3 + the next lane's byte 0
      static_assert(TW == 16, "fast-path byte phase assumes 16-wide tiles");
#pragma unroll
      for (int i = 0; i < NIT; ++i) {
        const int r = 2 * (wave + NW * i) + (lane >> 5);
        const uint32_t vn = __shfl_down(v[i], 1, 32);
        if (r < IH && k < DPR) {
          const uint32_t p0 = __builtin_amdgcn_perm(0u, v[i], 0x0c020c01u);   // [b1, 0, b2, 0]
          const uint32_t p1 = __builtin_amdgcn_perm(vn, v[i], 0x0c040c03u);   // [b3, 0, next b0, 0]
          f16x2 h0 = __builtin_bit_cast(f16x2, p0 | 0x64006400u), h1 = __builtin_bit_cast(f16x2, p1 | 0x64006400u);
          h0 = h0 - f16x2{(_Float16)1024.0f, (_Float16)1024.0f};
          h1 = h1 - f16x2{(_Float16)1024.0f, (_Float16)1024.0f};
          const uint32_t d0 = __builtin_bit_cast(uint32_t, h0), d1 = __builtin_bit_cast(uint32_t, h1);
          // column dwords cd = 2k-1 (d0) and 2k (d1): Lr[spy][cd][ky] for every (spy, ky) with 2 spy + ky = r
          uint32_t* l0 = Lr + (r >> 1) * RSL + 3 * (2 * k) + (r & 1);     // (spy = r/2, ky = r%2)
          if ((r >> 1) < SH) {
            if (k > 0) l0[-3] = d0;
            l0[0] = d1;
          }
          if (!(r & 1) && r >= 2) {                                       // (spy = r/2 - 1, ky = 2)
            uint32_t* l2 = l0 - RSL + 2;
            if (k > 0) l2[-3] = d0;
            l2[0] = d1;
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NIT; ++i) {
        const int r = 2 * (wave + NW * i) + (lane >> 5);
        if (r >= IH || k >= DPR) continue;
        const int iy = iy0 + r;
        const bool row_ok = iy >= 0 && iy < H;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int o = a[i] + j - rs[i];
          if (o < 0 || o >= RB) continue;
          const int ix = ix0 + o / 3;
          In[r * IRS + o] = (row_ok && ix >= 0 && ix < W) ? (uint8_t)(v[i] >> (8 * j)) : (uint8_t)0;
        }
      }
    }
    if (vt < 48) {
      const int kx = vt >> 4, ky = (vt >> 3) & 1;
      *reinterpret_cast<uint4*>(Sv + kx * 64 + ky * 32 + 4 * (vt & 7)) =
          make_uint4((wa.x & 0xffffu) | (wb.x << 16), (wa.x >> 16) | (wb.x & 0xffff0000u),
                     (wa.y & 0xffffu) | (wb.y << 16), (wa.y >> 16) | (wb.y & 0xffff0000u));
    }
    if (tid < 32) Sb[tid] = bd[tid];
    if (tid < 4) Lr[SH * RSL + tid] = 0;   // pad dwords read (zero weight) by the last position of the last row
  }
  // stem weight fragments (blob k order = the Lr dword order), bias as the MFMA C operand
  x8 ahi[2], alo[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    ahi[t] = load8<DT>(wsp + (16 * t + r16) * 32 + 8 * kg);
    alo[t] = load8<DT>(wsp + 32 * 32 + (16 * t + r16) * 32 + 8 * kg);
  }
  const float4 sb0 = *reinterpret_cast<const float4*>(bs + 4 * kg);
  const float4 sb1 = *reinterpret_cast<const float4*>(bs + 16 + 4 * kg);
  const bool interior = sy0 >= 0 && sx0 >= 0 && sy0 + SH <= SH_img && sx0 + SW <= SW_img;
  __syncthreads();

  // ---- 2. edge tiles: In -> Lr, lane = column dword cd, rows r = wave + NW i; exact fp16 via 0x6400 | byte, minus 1024
  if (!fast) {
  if (lane < NCD) {
    const int cd = lane;
#pragma unroll
    for (int i = 0; i < (IH + NW - 1) / NW; ++i) {
      const int r = wave + NW * i;
      if (r >= IH) break;
      const uint8_t* src = In + r * IRS + 2 * cd;
      const uint32_t bv = (uint32_t)src[0] | ((uint32_t)src[1] << 16);
      f16x2 hv = __builtin_bit_cast(f16x2, bv | 0x64006400u);
      hv = hv - f16x2{(_Float16)1024.0f, (_Float16)1024.0f};
      const uint32_t dv = __builtin_bit_cast(uint32_t, hv);
      if (r & 1) {
        Lr[((r - 1) >> 1) * RSL + 3 * cd + 1] = dv;
      } else {
        if ((r >> 1) < SH) Lr[(r >> 1) * RSL + 3 * cd] = dv;
        if (r >= 2) Lr[((r >> 1) - 1) * RSL + 3 * cd + 2] = dv;
      }
    }
  }
  __syncthreads();
  }

  // ---- 3. stem on MFMA, units of 16 (row pair, column) positions -> pair slab Ps (ReLU, fp16; zero outside the
  // stem map = block-1 depthwise padding)
#pragma unroll
  for (int j = 0; j < EPU; ++j) {
    const int u = wave + NW * j;
    if (u >= NU) break;
    const int q = 16 * u + r16;
    const int qc = q < NQ ? q : NQ - 1;
    const int pr = qc / SW, col = qc - pr * SW;
    const uint32_t* lb = Lr + 2 * pr * RSL + 9 * col + 4 * kg;
    x8 bx[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t* p = lb + h * RSL;
      bx[h] = __builtin_bit_cast(x8, u32x4{p[0], p[1], p[2], p[3]});
    }
    f32x4 e[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      e[h][0] = f32x4{sb0.x, sb0.y, sb0.z, sb0.w};
      e[h][1] = f32x4{sb1.x, sb1.y, sb1.z, sb1.w};
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        e[h][t] = DT::mfma(ahi[t], bx[h], e[h][t]);
        e[h][t] = DT::mfma(alo[t], bx[h], e[h][t]);
      }
    }
    uint4 d[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
      d[t] = make_uint4(relu_pk2(e[0][t][0], e[1][t][0]), relu_pk2(e[0][t][1], e[1][t][1]),
                        relu_pk2(e[0][t][2], e[1][t][2]), relu_pk2(e[0][t][3], e[1][t][3]));
    if (!interior) {
      const int gy = sy0 + 2 * pr, gx = sx0 + col;
      const bool cx = gx >= 0 && gx < SW_img;
      const uint32_t m = ((cx && gy >= 0 && gy < SH_img) ? 0x0000ffffu : 0u) |
                         ((cx && gy + 1 >= 0 && gy + 1 < SH_img) ? 0xffff0000u : 0u);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        d[t].x &= m; d[t].y &= m; d[t].z &= m; d[t].w &= m;
      }
    }
    char* er = Ps + q * 32 + (kg & 1) * 16;
    *reinterpret_cast<u32x4*>(er + (kg >> 1) * RSB) = u32x4{d[0].x, d[0].y, d[0].z, d[0].w};
    *reinterpret_cast<u32x4*>(er + (2 + (kg >> 1)) * RSB) = u32x4{d[1].x, d[1].y, d[1].z, d[1].w};
  }
  const x8 pa = load8<DT>(Wp + (size_t)r16 * 32 + 8 * kg);
  const float4 pb = *reinterpret_cast<const float4*>(bp + 4 * kg);
  __syncthreads();

  // ---- 4. block 1: depthwise (rows oy = 2 wave, oy + 1; pairs m = wave, wave + 1) -> project 32 -> 16 (+BN)
  {
    const int oy = 2 * wave, ox = r16;
    const char* pbase = Ps + kg * RSB + (wave * SW + ox) * 32;
    const uint32_t* sv = Sv + 8 * kg;
    float a0[8], a1[8];
    {
      const float4 u0 = *reinterpret_cast<const float4*>(Sb + 8 * kg);
      const float4 u1 = *reinterpret_cast<const float4*>(Sb + 8 * kg + 4);
      a0[0] = u0.x; a0[1] = u0.y; a0[2] = u0.z; a0[3] = u0.w; a0[4] = u1.x; a0[5] = u1.y; a0[6] = u1.z; a0[7] = u1.w;
#pragma unroll
      for (int e = 0; e < 8; ++e) a1[e] = a0[e];
    }
    auto rd8 = [&](const void* p, uint32_t v[8]) {
      const uint4 x = *reinterpret_cast<const uint4*>(p), y = *(reinterpret_cast<const uint4*>(p) + 1);
      v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
    };
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      uint32_t pc[8], pn[8], w01[8], w12[8];
      rd8(pbase + kx * 32, pc);
      rd8(pbase + (SW + kx) * 32, pn);
      rd8(sv + kx * 64, w01);
      rd8(sv + kx * 64 + 32, w12);
#pragma unroll
      for (int e = 0; e < 8; ++e) {   // same operations and order as k_irb.hip's VP row pair
        a1[e] = fmaf(h_hi(pc[e]), h_lo(w01[e]), a1[e]);
        a0[e] = dot2h(pc[e], w01[e], a0[e]);
        a0[e] = fmaf(h_lo(pn[e]), h_hi(w12[e]), a0[e]);
        a1[e] = dot2h(pn[e], w12[e], a1[e]);
      }
    }
    const x8 bf0 = relu_cvt8<DT>(a0), bf1 = relu_cvt8<DT>(a1);
    f32x4 acc0 = {pb.x, pb.y, pb.z, pb.w}, acc1 = acc0;
    acc0 = DT::mfma(pa, bf0, acc0);
    acc1 = DT::mfma(pa, bf1, acc1);
    const int gy = oy0 + oy, gx = ox0 + ox;
    T* yr = Y + (((size_t)b * SH_img + gy) * SW_img + gx) * 16 + 4 * kg;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (gy + h < SH_img && gx < SW_img) {
        const f32x4& ac = h ? acc1 : acc0;
        x4 out;
        out[0] = (T)ac[0];
        out[1] = (T)ac[1];
        out[2] = (T)ac[2];
        out[3] = (T)ac[3];
        SPEF_KB_YSTORE(*reinterpret_cast<x4*>(yr + (size_t)h * SW_img * 16) = out, out);
      }
    }
  }
}

hipError_t launch_front(int dtype, const void* x, const void* wsp, const float* bs, const void* wd, const float* bd,
                        const void* wp, const float* bp, void* y, int B, int H, int W, int OH, int OW,
                        hipStream_t s) {
  constexpr int TH = 16, TW = 16, NW = 8;
  const int tiles_x = (OW + TW - 1) / TW, tiles_y = (OH + TH - 1) / TH;
  const int64_t ntiles64 = (int64_t)tiles_x * tiles_y * B;
  if (ntiles64 > 0x7fffffff) return hipErrorInvalidValue;
  if ((int64_t)H * W * 3 + 4 > 0x7fffffff) return hipErrorInvalidValue;   // 32-bit in-frame byte offsets
  const uint32_t nwg = (uint32_t)ntiles64;
  if (dtype == DT_F16)
    front_vp_kernel<TH, TW, NW><<<nwg, NW * 64, 0, s>>>((const uint8_t*)x, (const _Float16*)wsp, bs, (const _Float16*)wd, bd,
                                                     (const _Float16*)wp, bp, (_Float16*)y, H, W, OH, OW, tiles_x, tiles_y,
                                                     nwg);
  else
    front_kernel<BF16, TH, TW, NW><<<nwg, NW * 64, 0, s>>>((const uint8_t*)x, (const __bf16*)wsp, bs, (const float*)wd, bd, (const __bf16*)wp, bp,
                                                           (__bf16*)y, H, W, OH, OW, tiles_x, tiles_y, nwg);
  return hipGetLastError();
}

}  // namespace spef
