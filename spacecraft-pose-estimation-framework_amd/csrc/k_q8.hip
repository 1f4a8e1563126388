// INT8 path: the Brevitas-mirroring quantized MobileNet-V2 + URSONet head
// (src/modeling/backbone/mobilenet_v2.py:119-229, common/brevitas_layers.py:10-136, head/ursonet.py:36-93)
// with the integer semantics of oracle/int8_ref.py, which these kernels reproduce bit-exactly:
//
//   conv + BN + quant   acc = sum q_x q_w (int32, exact);  q = clip((acc * M[c] + B[c]) >> S[c], lo, hi)
//                       (int64 fixed point; M, B, S per output channel from the blob, B holds the rounding half)
//   residual join       q_sum = q_proj + q_in;  q_out = clip((q_sum * R + RB) >> RS, -128, 127)
//   pool                sum over the map >> tb (TruncTo8bit floor), u8
//   FC                  out = f32(acc + q_b[c]) * sc[c]
//
// MFMA: v_mfma_i32_16x16x64_i8 (signed x signed). Unsigned activations (depthwise outputs, pooled features)
// are stored offset by -128 (u ^ 0x80) so they are valid int8 operands; the exact correction 128 * sum_k q_w
// is the accumulator's initial value (`init`, per output channel). The K order inside one MFMA is irrelevant
// because A and B fragments use the same lane->k assignment (lane (r, g) element j <-> k = 16 g + j).
#include "spef_common.hpp"
#include "spef_kernels.hpp"

namespace spef {

typedef int i32x4 __attribute__((ext_vector_type(4)));

struct Rq {   // per-channel requant parameters, struct-of-arrays over Np channels
  const int64_t* M;
  const int64_t* B;
  const int32_t* S;
  int lo, hi;   // output quantizer range: [0, 2^b - 1] unsigned, [-2^(b-1), 2^(b-1) - 1] signed (bit width b <= 8)
};

__device__ __forceinline__ int requant(int acc, int64_t M, int64_t B, int S, int lo, int hi) {
  const int64_t v = ((int64_t)acc * M + B) >> S;
  return (int)(v < lo ? lo : (v > hi ? hi : v));
}

// clamp to [lo, hi] (lo <= hi) as one v_med3_i32 (the compiler forms med3 only for constant bounds)
__device__ __forceinline__ int q_med3(int x, int lo, int hi) {
  int r;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo), "v"(hi));
  return r;
}

// ------------------------------------------------------------------------------------------------ stem
// Input QuantIdentity + QConvBnAct 3->32 3x3/s2 (mobilenet_v2.py:177-182).
// A workgroup owns a 4 x 64 output tile. Its 9 x 129 input
// pixels are staged in LDS once, quantised (LUT / rint), one dword per pixel [q_r, q_g, q_b, 0], and the weights
// rearranged to [32][9] dwords of the same form (w28's k = ky*9 + kx*3 + ci order: the sums are the same integers).
// The conv is then a K = 64 MFMA (9 tap dwords + zero padding): one ds_read_b32 per tap per lane. 15 byte gathers
// per thread instead of 27 per pixel. Requant: the high word of one v_mad_i64_i32 shifted by S - 32 when every channel's
// S >= 32 and |M| < 2^31 (workgroup-uniform check), the 64-bit form otherwise.
constexpr int kStemTH = 4, kStemTW = 64, kStemIH = 2 * kStemTH + 1, kStemIW = 2 * kStemTW + 1;

template <bool F32IN>
__global__ __launch_bounds__(256) void q_stem_rows_kernel(const void* __restrict__ in, const int8_t* __restrict__ lut,
                                                          float s_img, int in_lo, int in_hi,
                                                          const int8_t* __restrict__ w28, Rq rq,
                                                          uint8_t* __restrict__ Y, int H, int W, int OH, int OW,
                                                          int tiles_x, int tiles_y, size_t nbytes) {
  __shared__ int Xs[kStemIH * kStemIW];
  constexpr int RAWDW = (3 * kStemIW + 6) / 4 + 1;   // dwords of one window row's aligned byte span
  __shared__ uint32_t Raw[F32IN ? 1 : kStemIH * RAWDW];
  __shared__ int Wl[32 * 9];
  __shared__ int8_t Ll[256];
  __shared__ int64_t Ml[32], Bl[32];
  __shared__ int Sl[32];
  const int tid = threadIdx.x;
  int L = blockIdx.x;
  const int tx = L % tiles_x;
  L /= tiles_x;
  const int ty = L % tiles_y, b = L / tiles_y;
  const int oy0 = ty * kStemTH, ox0 = tx * kStemTW;
  const int iy0 = 2 * oy0 - 1, ix0 = 2 * ox0 - 1;
  // staging: every load issued (clamped address) before any is used. u8 frames: each window row is one contiguous
  // byte span (clipped to the image row), moved as aligned dwords into Raw and unpacked from LDS below.
  const int cx0 = ix0 > 0 ? ix0 : 0, cx1 = ix0 + kStemIW < W ? ix0 + kStemIW : W;   // valid columns [cx0, cx1)
  constexpr int NRAW = kStemIH * RAWDW, NITR = (NRAW + 255) / 256;
  uint32_t rw[F32IN ? 1 : NITR];
  if constexpr (!F32IN) {
    const uint8_t* inb = reinterpret_cast<const uint8_t*>(in);
#pragma unroll
    for (int it = 0; it < NITR; ++it) {
      const int i = tid + 256 * it;
      const int r = i / RAWDW, d = i - r * RAWDW;
      const int iy = iy0 + r;
      const size_t rs = (((size_t)b * H + (iy >= 0 ? iy : 0)) * W + cx0) * 3, re = rs + (size_t)(cx1 - cx0) * 3;
      const size_t dw = (rs >> 2) + d;
      const bool ok = i < NRAW && (unsigned)iy < (unsigned)H && cx1 > cx0 && 4 * dw < re;
      if (ok && 4 * dw + 4 > nbytes) {   // the buffer's partial last dword: bytes one by one
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k)
          if (4 * dw + k < nbytes) v |= (uint32_t)inb[4 * dw + k] << (8 * k);
        rw[it] = v;
      } else {
        rw[it] = reinterpret_cast<const uint32_t*>(inb)[ok ? dw : 0];
      }
    }
  }
  constexpr int NS = kStemIH * kStemIW, NIT = (NS + 255) / 256;
  float fv[F32IN ? NIT * 3 : 1];
  uint32_t okm = 0;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int i = tid + 256 * it;
    const int r = i / kStemIW, cc = i - r * kStemIW;
    const int iy = iy0 + r, ix = ix0 + cc;
    const bool ok = i < NS && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    okm |= (uint32_t)ok << it;
#pragma unroll
    for (int ci = 0; ci < 3; ++ci) {
      if (F32IN) {
        const size_t off = ok ? (((size_t)b * 3 + ci) * H + iy) * W + ix : 0;
        fv[it * 3 + ci] = reinterpret_cast<const float*>(in)[off];
      }
    }
  }
  bool fast_ok = true;
  if (tid < 32) {
    Ml[tid] = rq.M[tid];
    Bl[tid] = rq.B[tid];
    Sl[tid] = rq.S[tid];
    fast_ok = rq.S[tid] >= 32 && rq.M[tid] > -(1LL << 31) && rq.M[tid] < (1LL << 31);
  }
  for (int i = tid; i < 32 * 9; i += 256) {   // [c][tap] dwords {w(ci 0), w(ci 1), w(ci 2), 0}
    const int c = i / 9, t = i - 9 * c;
    const uint8_t* w = reinterpret_cast<const uint8_t*>(w28) + c * 28 + 3 * t;
    Wl[i] = (int)((uint32_t)w[0] | ((uint32_t)w[1] << 8) | ((uint32_t)w[2] << 16));
  }
  if constexpr (!F32IN) {
    Ll[tid] = lut[tid];
#pragma unroll
    for (int it = 0; it < NITR; ++it) {
      const int i = tid + 256 * it;
      if (i < NRAW) Raw[i] = rw[it];
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int i = tid + 256 * it;
    if (i < NS) {
      uint32_t v = 0;
      if ((okm >> it) & 1u) {
        // u8: bytes (ix - cx0) * 3 + ci of window row r's span, which starts (rs & 3) bytes into Raw; rs mod 4 only
        // needs the low bits of the byte offset, so 32-bit arithmetic (wrapping) gives it exactly
        const int r = i / kStemIW, ix = ix0 + (i - r * kStemIW);
        const uint32_t rs = (((uint32_t)b * (uint32_t)H + (uint32_t)(iy0 + r)) * (uint32_t)W + (uint32_t)cx0) * 3u;
        const uint8_t* rb = reinterpret_cast<const uint8_t*>(Raw + r * RAWDW) + (rs & 3u) + (ix - cx0) * 3;
#pragma unroll
        for (int ci = 0; ci < 3; ++ci) {
          int q;
          if (F32IN) q = (int)fminf(fmaxf(rintf(fv[it * 3 + ci] / s_img), (float)in_lo), (float)in_hi);
          else q = Ll[rb[ci]];
          v |= ((uint32_t)q & 0xffu) << (8 * ci);
        }
      }
      Xs[i] = (int)v;
    }
  }
  const bool fast = __syncthreads_and(fast_ok);
  // ---- the 3x3/s2 conv on v_mfma_i32_16x16x64_i8: k = 4 * tap + byte (tap = ky*3 + kx, taps >= 9 zero), a wave
  // computes 16 pixels x 16 channels per MFMA; lane (r16, kg) holds taps 4 kg .. 4 kg + 3 of pixel / channel r16
  const int lane = tid & 63, wave = tid >> 6, r16 = lane & 15, kg = lane >> 4;
  int toff[4];
  uint32_t tv = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int t = 4 * kg + j, tc = t < 9 ? t : 0;
    toff[j] = (tc / 3) * kStemIW + tc % 3;
    tv |= (uint32_t)(t < 9) << j;
  }
  i32x4 a[2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = 4 * kg + j;
      const int v = Wl[(16 * h + r16) * 9 + (t < 9 ? t : 0)];
      a[h][j] = ((tv >> j) & 1u) ? v : 0;
    }
  int64_t Mr[8], Br[8];
  int Sr[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = (i < 4 ? 0 : 12) + 4 * kg + i;
    Mr[i] = Ml[c];
    Br[i] = Bl[c];
    Sr[i] = Sl[c];
  }
  constexpr int GPW = kStemTH * kStemTW / 16 / 4;   // 16-pixel groups per wave
#pragma unroll
  for (int gi = 0; gi < GPW; ++gi) {
    const int g = wave * GPW + gi;
    const int oy = g / (kStemTW / 16), ox = (g % (kStemTW / 16)) * 16 + r16;
    const int base = 2 * oy * kStemIW + 2 * ox;
    i32x4 bx;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int v = Xs[base + toff[j]];
      bx[j] = ((tv >> j) & 1u) ? v : 0;
    }
    const i32x4 z = {0, 0, 0, 0};
    const i32x4 acc0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[0], bx, z, 0, 0, 0);
    const i32x4 acc1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[1], bx, z, 0, 0, 0);
    uint32_t o[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t w = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int acc = h ? acc1[i] : acc0[i];
        const int e = 4 * h + i;
        int v;
        if (fast) {
          v = (int)(((int64_t)acc * (int)Mr[e] + Br[e]) >> 32) >> (Sr[e] - 32);
          v = q_med3(v, 0, rq.hi);
        } else {
          v = requant(acc, Mr[e], Br[e], Sr[e], 0, rq.hi);
        }
        w |= (uint32_t)v << (8 * i);
      }
      o[h] = w;
    }
    const int gy = oy0 + oy, gx = ox0 + ox;
    if (gy < OH && gx < OW) {
      uint8_t* y = Y + (((size_t)b * OH + gy) * OW + gx) * 32 + 4 * kg;
      *reinterpret_cast<uint32_t*>(y) = o[0];
      *reinterpret_cast<uint32_t*>(y + 16) = o[1];
    }
  }
}

// ------------------------------------------------------------------------------------------------ depthwise
// dw QConvBnAct (brevitas_layers.py:113-119): u8 in, int8 [9][C] weights, ReLU-quant; output stored offset
// (u - 128 as int8) for the projection MFMA. One thread = one output pixel x 8 channels.
__global__ __launch_bounds__(256) void q_dw_kernel(const uint8_t* __restrict__ X, const int8_t* __restrict__ W9,
                                                   Rq rq, int8_t* __restrict__ Y, int B, int H, int W, int C,
                                                   int stride, int OH, int OW) {
  const int cg = C >> 3;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)B * OH * OW * cg) return;
  const int g = (int)(t % cg);
  const int64_t p = t / cg;
  const int ox = (int)(p % OW);
  const int oy = (int)((p / OW) % OH);
  const int b = (int)(p / ((int64_t)OW * OH));
  const int c0 = 8 * g;
  int acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = oy * stride - 1 + ky;
    if (iy < 0 || iy >= H) continue;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int ix = ox * stride - 1 + kx;
      if (ix < 0 || ix >= W) continue;
      const uint2 xv = *reinterpret_cast<const uint2*>(X + (((size_t)b * H + iy) * W + ix) * C + c0);
      const uint2 wv = *reinterpret_cast<const uint2*>(W9 + (size_t)(ky * 3 + kx) * C + c0);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int xs = (int)(((e < 4 ? xv.x : xv.y) >> (8 * (e & 3))) & 0xff);
        const int ws = (int)(int8_t)(((e < 4 ? wv.x : wv.y) >> (8 * (e & 3))) & 0xff);
        acc[e] += xs * ws;
      }
    }
  }
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = c0 + e;
    const uint32_t q = (uint32_t)(requant(acc[e], rq.M[c], rq.B[c], rq.S[c], 0, rq.hi) ^ 0x80);
    if (e < 4) lo |= q << (8 * e);
    else hi |= q << (8 * (e - 4));
  }
  *reinterpret_cast<uint2*>(Y + p * C + c0) = make_uint2(lo, hi);
}

// ------------------------------------------------------------------------------------------------ GEMM
// 1x1 conv / FC as C^T = W X^T on v_mfma_i32_16x16x64_i8: W int8 [Np][Kp] (Kp multiple of 64), X int8 [M][K]
// (NHWC rows). Workgroup 4 waves = WN (channel) x WM (pixel); K advances 64 per double-buffered LDS step.
// LDS rows are 80 B (64 + 16 pad): the 16 rows of one ds_read_b128 phase hit disjoint banks.
template <int WN, int NT, int MT, int EPI>
__global__ __launch_bounds__(256) void q_gemm_kernel(const int8_t* __restrict__ X, const int8_t* __restrict__ Wt,
                                                     const int32_t* __restrict__ init, Rq rq,
                                                     const int8_t* __restrict__ R, int64_t RM, int64_t RB, int RS,
                                                     void* __restrict__ Y, float* __restrict__ Y1,
                                                     const float* __restrict__ sc, int n_split, int64_t M, int K,
                                                     int N, int Kp, int Np, int n_chunks, uint32_t nwg) {
  constexpr int WM = 4 / WN;
  constexpr int BN = 16 * WN * NT, BM = 16 * WM * MT;
  constexpr int RSB = 80;
  constexpr int XP = (BM * 4 + 255) / 256, WP = (BN * 4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) int8_t As[2][BN * RSB];
  __shared__ __attribute__((aligned(16))) int8_t Bs[2][BM * RSB];

  const uint32_t L = xcd_remap(blockIdx.x, nwg);
  const int chunk = (int)(L % (uint32_t)n_chunks);
  const int64_t mt0 = (int64_t)(L / (uint32_t)n_chunks) * BM;
  const int n0 = chunk * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  const int wn = wave % WN, wm = wave / WN;
  const bool k16 = (K & 15) == 0;

  i32x4 xr[XP], wr[WP];
  auto gload = [&](int ks) {
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int p = tid + 256 * i;
      const int row = p >> 2, g = p & 3;
      const int64_t m = mt0 + row;
      const int k = ks * 64 + 16 * g;
      i32x4 v = {0, 0, 0, 0};
      if (p < BM * 4 && m < M) {
        const int8_t* src = X + (size_t)m * K + k;
        if (k16) {
          if (k < K) v = *reinterpret_cast<const i32x4*>(src);
        } else {
          if (k < K) {
            const int2 a = *reinterpret_cast<const int2*>(src);
            v[0] = a.x;
            v[1] = a.y;
          }
          if (k + 8 < K) {
            const int2 a = *reinterpret_cast<const int2*>(src + 8);
            v[2] = a.x;
            v[3] = a.y;
          }
        }
      }
      xr[i] = v;
    }
#pragma unroll
    for (int i = 0; i < WP; ++i) {
      const int p = tid + 256 * i;
      const int row = p >> 2, g = p & 3;
      const int n = n0 + row;
      i32x4 v = {0, 0, 0, 0};
      if (p < BN * 4 && n < Np) v = *reinterpret_cast<const i32x4*>(Wt + (size_t)n * Kp + ks * 64 + 16 * g);
      wr[i] = v;
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int p = tid + 256 * i;
      if (p < BM * 4) *reinterpret_cast<i32x4*>(&Bs[buf][(p >> 2) * RSB + 16 * (p & 3)]) = xr[i];
    }
#pragma unroll
    for (int i = 0; i < WP; ++i) {
      const int p = tid + 256 * i;
      if (p < BN * 4) *reinterpret_cast<i32x4*>(&As[buf][(p >> 2) * RSB + 16 * (p & 3)]) = wr[i];
    }
  };

  i32x4 acc[NT][MT];
#pragma unroll
  for (int a = 0; a < NT; ++a) {
    const int i = n0 + (wn * NT + a) * 16 + 4 * kg;
    int4 b0 = make_int4(0, 0, 0, 0);
    if (init && i < Np) b0 = *reinterpret_cast<const int4*>(init + i);
#pragma unroll
    for (int b = 0; b < MT; ++b) acc[a][b] = i32x4{b0.x, b0.y, b0.z, b0.w};
  }

  const int KS = Kp >> 6;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int ks = 0; ks < KS; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < KS) gload(ks + 1);
    i32x4 af[NT], bf[MT];
#pragma unroll
    for (int a = 0; a < NT; ++a)
      af[a] = *reinterpret_cast<const i32x4*>(&As[buf][((wn * NT + a) * 16 + r16) * RSB + 16 * kg]);
#pragma unroll
    for (int b = 0; b < MT; ++b)
      bf[b] = *reinterpret_cast<const i32x4*>(&Bs[buf][((wm * MT + b) * 16 + r16) * RSB + 16 * kg]);
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int b = 0; b < MT; ++b) acc[a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[a], bf[b], acc[a][b], 0, 0, 0);
    if (ks + 1 < KS) {
      lstore(buf ^ 1);
      __syncthreads();
    }
  }

#pragma unroll
  for (int a = 0; a < NT; ++a) {
    const int i = n0 + (wn * NT + a) * 16 + 4 * kg;
    if (i >= N) continue;
#pragma unroll
    for (int b = 0; b < MT; ++b) {
      const int64_t m = mt0 + (wm * MT + b) * 16 + r16;
      if (m >= M) continue;
      const i32x4 v = acc[a][b];
      if constexpr (EPI == QEPI_FC) {   // float head outputs: columns [0, n_split) -> Y, the rest -> Y1
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = i + e;
          if (c >= N) break;
          const float o = (float)v[e] * sc[c];
          if (c < n_split) reinterpret_cast<float*>(Y)[(size_t)m * n_split + c] = o;
          else Y1[(size_t)m * (N - n_split) + (c - n_split)] = o;
        }
        continue;
      }
      uint32_t packed = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = i + e;
        int q;
        if constexpr (EPI == QEPI_RELU) {
          q = requant(v[e], rq.M[c], rq.B[c], rq.S[c], 0, rq.hi);
        } else if constexpr (EPI == QEPI_PROJ) {
          q = requant(v[e], rq.M[c], rq.B[c], rq.S[c], rq.lo, rq.hi);
        } else {   // QEPI_PROJ_RES: residual join, then requantise to the next consumer's scale (same width)
          const int p = requant(v[e], rq.M[c], rq.B[c], rq.S[c], rq.lo, rq.hi) + (int)R[(size_t)m * N + c];
          const int64_t t = ((int64_t)p * RM + RB) >> RS;
          q = (int)(t < rq.lo ? rq.lo : (t > rq.hi ? rq.hi : t));
        }
        packed |= ((uint32_t)q & 0xffu) << (8 * e);
      }
      *reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(Y) + (size_t)m * N + i) = packed;
    }
  }
}

// ------------------------------------------------------------------------------------------------ pool
// QuantAvgPool2d + TruncTo8bit over the whole map (ursonet.py:61-62, 88): pooled = (sum_hw q) >> tb, stored
// offset (u - 128) as the FC's int8 B operand. Workgroup = (image, 64 channels): 16 lanes x 4 channels per row
// of pixels, 16 pixel rows strided over the map, integer partial sums reduced through LDS (exact, any order).
__global__ __launch_bounds__(256) void q_pool_kernel(const uint8_t* __restrict__ X, int8_t* __restrict__ P, int B,
                                                     int HW, int C, int tb) {
  __shared__ int part[16][64];
  const int b = blockIdx.y, c0 = blockIdx.x * 64;
  const int cl = threadIdx.x & 15, pg = threadIdx.x >> 4;
  int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  for (int p = pg; p < HW; p += 16) {
    const uint32_t v = *reinterpret_cast<const uint32_t*>(X + ((size_t)b * HW + p) * C + c0 + 4 * cl);
    s0 += v & 0xff;
    s1 += (v >> 8) & 0xff;
    s2 += (v >> 16) & 0xff;
    s3 += v >> 24;
  }
  part[pg][4 * cl] = s0;
  part[pg][4 * cl + 1] = s1;
  part[pg][4 * cl + 2] = s2;
  part[pg][4 * cl + 3] = s3;
  __syncthreads();
  if (threadIdx.x < 64) {
    int t = 0;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += part[g][threadIdx.x];
    P[(size_t)b * C + c0 + threadIdx.x] = (int8_t)(uint8_t)(((uint32_t)(t >> tb) ^ 0x80) & 0xff);
  }
}

// int8 / u8 codes -> fp32 (probes, dequantized feature export): y = (code) * scale
__global__ void q_to_f32_kernel(const void* __restrict__ x, float* __restrict__ y, int64_t n, int is_unsigned,
                                float scale) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int v = is_unsigned ? (int)reinterpret_cast<const uint8_t*>(x)[i] : (int)reinterpret_cast<const int8_t*>(x)[i];
  y[i] = (float)v * scale;
}

// ------------------------------------------------------------------------------------------------ launchers

hipError_t launch_q_to_f32(const void* x, float* y, int64_t n, int is_unsigned, float scale, hipStream_t s) {
  const int64_t nb = (n + 255) / 256;
  if (nb > 0x7fffffff) return hipErrorInvalidValue;
  if (n > 0) q_to_f32_kernel<<<(unsigned)nb, 256, 0, s>>>(x, y, n, is_unsigned, scale);
  return hipGetLastError();
}

hipError_t launch_q_stem(const void* in, int f32in, const int8_t* lut, float s_img, int in_bits, const int8_t* w28,
                         const int64_t* M, const int64_t* Bq, const int32_t* S, int out_bits, uint8_t* y, int B, int H,
                         int W, int OH, int OW, hipStream_t s) {
  if (in_bits < 2 || in_bits > 8 || out_bits < 2 || out_bits > 8) return hipErrorInvalidValue;
  const int in_lo = -(1 << (in_bits - 1)), in_hi = (1 << (in_bits - 1)) - 1;
  const int tiles_x = (OW + kStemTW - 1) / kStemTW, tiles_y = (OH + kStemTH - 1) / kStemTH;
  const size_t nbytes = (size_t)B * H * W * 3;   // u8 NHWC frame buffer (the f32 form does not use it)
  const int64_t nb = (int64_t)tiles_x * tiles_y * B;
  if (nb > 0x7fffffff) return hipErrorInvalidValue;
  if (nb == 0) return hipSuccess;
  Rq rq{M, Bq, S, 0, (1 << out_bits) - 1};
  if (f32in)
    q_stem_rows_kernel<true><<<(unsigned)nb, 256, 0, s>>>(in, lut, s_img, in_lo, in_hi, w28, rq, y, H, W, OH, OW,
                                                           tiles_x, tiles_y, nbytes);
  else
    q_stem_rows_kernel<false><<<(unsigned)nb, 256, 0, s>>>(in, lut, s_img, in_lo, in_hi, w28, rq, y, H, W, OH, OW,
                                                            tiles_x, tiles_y, nbytes);
  return hipGetLastError();
}

hipError_t launch_q_dw(const uint8_t* x, const int8_t* w9, const int64_t* M, const int64_t* Bq, const int32_t* S,
                       int out_bits, int8_t* y, int B, int H, int W, int C, int stride, int OH, int OW, hipStream_t s) {
  if ((C & 7) || out_bits < 2 || out_bits > 8) return hipErrorInvalidValue;
  const int64_t n = (int64_t)B * OH * OW * (C >> 3);
  const int64_t nb = (n + 255) / 256;
  if (nb > 0x7fffffff) return hipErrorInvalidValue;
  q_dw_kernel<<<(unsigned)nb, 256, 0, s>>>(x, w9, Rq{M, Bq, S, 0, (1 << out_bits) - 1}, y, B, H, W, C, stride, OH, OW);
  return hipGetLastError();
}

template <int WN, int NT, int MT>
static hipError_t q_gemm_go(const QGemmArgs& a, hipStream_t s) {
  constexpr int WM = 4 / WN;
  constexpr int BN = 16 * WN * NT, BM = 16 * WM * MT;
  const int Kp = (a.K + 63) & ~63, Np = (a.N + 15) & ~15;
  const int n_chunks = (Np + BN - 1) / BN;
  const int64_t nwg64 = (a.M + BM - 1) / BM * n_chunks;
  if (nwg64 > 0x7fffffff) return hipErrorInvalidValue;
  const uint32_t nwg = (uint32_t)nwg64;
  if (a.out_bits < 2 || a.out_bits > 8) return hipErrorInvalidValue;
  const bool sgn = a.epi == QEPI_PROJ || a.epi == QEPI_PROJ_RES;
  const Rq rq{a.rqM, a.rqB, a.rqS, sgn ? -(1 << (a.out_bits - 1)) : 0,
              sgn ? (1 << (a.out_bits - 1)) - 1 : (1 << a.out_bits) - 1};
#define SPEF_QG(E)                                                                                             \
  q_gemm_kernel<WN, NT, MT, E><<<nwg, 256, 0, s>>>(a.x, a.w, a.init, rq, a.r, a.rm, a.rb, a.rs, a.y, a.y1, a.sc, \
                                                   a.n_split, a.M, a.K, a.N, Kp, Np, n_chunks, nwg)
  switch (a.epi) {
    case QEPI_RELU: SPEF_QG(QEPI_RELU); break;
    case QEPI_PROJ: SPEF_QG(QEPI_PROJ); break;
    case QEPI_PROJ_RES: SPEF_QG(QEPI_PROJ_RES); break;
    case QEPI_FC: SPEF_QG(QEPI_FC); break;
    default: return hipErrorInvalidValue;
  }
#undef SPEF_QG
  return hipGetLastError();
}

hipError_t launch_q_gemm(const QGemmArgs& a, hipStream_t s) {
  if (a.M <= 0) return hipSuccess;
  if ((a.K & 7) || (a.epi != QEPI_FC && (a.N & 3))) return hipErrorInvalidValue;
  const int n16 = ((a.N + 15) & ~15) / 16;
  if (a.M <= 256) return q_gemm_go<4, 1, 1>(a, s);          // FC: few rows (images), many channels
  switch (n16) {
    case 1: return q_gemm_go<1, 1, 2>(a, s);
    case 2: return q_gemm_go<2, 1, 4>(a, s);
    case 4: return q_gemm_go<2, 2, 4>(a, s);
    case 6: return q_gemm_go<2, 3, 4>(a, s);
    case 9: return q_gemm_go<1, 9, 1>(a, s);
    case 10: return q_gemm_go<2, 5, 2>(a, s);
    default: break;
  }
  if (n16 % 12 == 0) return q_gemm_go<2, 6, 2>(a, s);
  if (n16 % 10 == 0) return q_gemm_go<2, 5, 2>(a, s);
  if (n16 % 8 == 0) return q_gemm_go<2, 4, 4>(a, s);
  if (n16 % 4 == 0) return q_gemm_go<2, 2, 4>(a, s);
  if (n16 % 2 == 0) return q_gemm_go<2, 1, 4>(a, s);
  return q_gemm_go<1, 1, 2>(a, s);
}

hipError_t launch_q_pool(const uint8_t* x, int8_t* p, int B, int HW, int C, int tb, hipStream_t s) {
  if (C & 63) return hipErrorInvalidValue;
  q_pool_kernel<<<dim3(C / 64, B), 256, 0, s>>>(x, p, B, HW, C, tb);
  return hipGetLastError();
}

}  // namespace spef
