// Head and decode kernels on gfx950.
//
//   fc_kernel          URSONetHead Linear layers (src/modeling/head/ursonet.py:17-25), ori and pos weights
//                      concatenated into one fp32 GEMM on the exact f32-input MFMA (v_mfma_f32_16x16x4_f32)
//   decode_ori_kernel  SPEUtils.last_activ softmax (src/spe/spe_utils.py:75-76) fused with
//                      OrientationSoftClassification.decode (src/spe/classification_utils.py:113-146):
//                      a = sum_i p_i q_i q_i^T in fp64, top eigenvector by repeated squaring, normalised
//   decode_pos_kernel  softmax (spe_utils.py:78-79) + PositionSoftClassification.decode
//                      (classification_utils.py:242-267): 3-D soft-argmax over the bin grid
//   normalize_ori      orientation regression L2 normalisation (spe_utils.py:72)
// One 256-thread workgroup decodes one image (the reference loops over images in Python,
// classification_utils.py:163-164); the orientation decode supports up to 8192 bins.
#include <math.h>

#include "spef_common.hpp"
#include "spef_kernels.hpp"

namespace spef {

// ------------------------------------------------------------------------------------------ fc
// out[b][i] = sum_k X[b][k] W[i][k] + bias[i]. One workgroup per 16x16 output tile; its 4 waves take
// interleaved quarters of K (split-K inside the workgroup, reduced through LDS in a fixed order, so the
// result is deterministic). Lane l loads float4 W[i0+(l&15)][t+4(l>>4)..] and X[j0+(l&15)][t+4(l>>4)..];
// MFMA step e takes element e from both, so A and B see the same k.
// 1-D grid, XCD-aware: the nJ image groups of one 16-row weight tile are consecutive logical ids, which
// xcd_remap places on one XCD, so the fp32 weight (8.85 MB for 1728 bins) is fetched from HBM once per batch
// and re-read from that XCD's L2 by the other image groups (round-robin placement fetched it once per group).
__global__ __launch_bounds__(256) void fc_kernel(const float* __restrict__ X, const float* __restrict__ W,
                                                 const float* __restrict__ bias, float* __restrict__ out0, int n0,
                                                 float* __restrict__ out1, int n1, int B, int K, int Np) {
  __shared__ f32x4 part[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t nJ = (uint32_t)(B + 15) / 16;
  const uint32_t L = xcd_remap(blockIdx.x, gridDim.x);
  const int i0 = (int)(L / nJ) * 16;
  const int j0 = (int)(L % nJ) * 16;
  const int r16 = lane & 15, kg = lane >> 4;
  const float* wp = W + (size_t)(i0 + r16) * K + 4 * kg;
  const int j = j0 + r16;
  const bool jv = j < B;
  const float* xp = X + (size_t)(jv ? j : 0) * K + 4 * kg;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int t = 16 * wave; t < K; t += 64) {
    const float4 a = *reinterpret_cast<const float4*>(wp + t);
    float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
    if (jv) b = *reinterpret_cast<const float4*>(xp + t);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
  }
  part[wave][lane] = acc;
  __syncthreads();
  if (wave != 0 || !jv) return;
  const f32x4 s = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * kg + r;
    const float v = s[r] + bias[i];
    if (i < n0)
      out0[(size_t)j * n0 + i] = v;
    else if (i < n0 + n1)
      out1[(size_t)j * n1 + (i - n0)] = v;
  }
}

// Split-K form for very long K (KeypointRegressionHead: K = 1280*8*12 = 122880, keypoints.py:20): grid.z
// slices of K write fp32 partial tiles, fc_reduce_kernel sums them in slice order (deterministic).
__global__ __launch_bounds__(256) void fc_partial_kernel(const float* __restrict__ X, const float* __restrict__ W,
                                                         float* __restrict__ part, int B, int K, int Np, int kslice) {
  __shared__ f32x4 red[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t nJ = (uint32_t)(B + 15) / 16, nI = (uint32_t)Np / 16;
  uint32_t L = xcd_remap(blockIdx.x, gridDim.x);       // image groups of one (slice, row tile) on one XCD
  const int j0 = (int)(L % nJ) * 16;
  L /= nJ;
  const int i0 = (int)(L % nI) * 16, z = (int)(L / nI);
  const int r16 = lane & 15, kg = lane >> 4;
  const int j = j0 + r16;
  const bool jv = j < B;
  const float* wp = W + (size_t)(i0 + r16) * K + 4 * kg;
  const float* xp = X + (size_t)(jv ? j : 0) * K + 4 * kg;
  const int k0 = z * kslice, k1 = min(K, k0 + kslice);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int t = k0 + 16 * wave; t < k1; t += 64) {
    const float4 a = *reinterpret_cast<const float4*>(wp + t);
    float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
    if (jv) b = *reinterpret_cast<const float4*>(xp + t);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave != 0 || !jv) return;
  const f32x4 s = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
  float* o = part + ((size_t)z * B + j) * Np + i0 + 4 * kg;
  *reinterpret_cast<float4*>(o) = make_float4(s[0], s[1], s[2], s[3]);
}

__global__ void fc_reduce_kernel(const float* __restrict__ part, const float* __restrict__ bias,
                                 float* __restrict__ out, int n, int B, int Np, int splits) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * n) return;
  const int j = idx / n, i = idx - j * n;
  const float* p = part + (size_t)j * Np + i;
  const size_t zs = (size_t)B * Np;
  float v = bias[i];
  // 30 slices' loads in flight, then added in slice order (the sum order of one slice at a time: bit-identical);
  // one dependent load per slice made this 60-slice reduction latency-bound (15 us)
  constexpr int U = 30;
  int z = 0;
  for (; z + U <= splits; z += U) {
    float t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = p[(size_t)(z + u) * zs];
#pragma unroll
    for (int u = 0; u < U; ++u) v += t[u];
  }
  for (; z < splits; ++z) v += p[(size_t)z * zs];
  out[(size_t)j * n + i] = v;
}

// ------------------------------------------------------------------------------------------ reductions
// Workgroup (4 waves) max / sum of one float per thread: within a 16-lane row by DPP (quad swaps, half-row and row
// mirrors: every lane ends with its row's value, no LDS round trip), the 4 rows by readlane, the 4 waves through
// LDS with one barrier. sh[4] must not be reused by the caller. A fixed combination order: deterministic.
template <bool MAX>
__device__ __forceinline__ float dpp_op(float a, float b) { return MAX ? fmaxf(a, b) : a + b; }
template <bool MAX, int CTRL>
__device__ __forceinline__ float dpp_step(float v) {
  const float o = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
  return dpp_op<MAX>(v, o);
}
template <bool MAX>
__device__ __forceinline__ float block_reduce256(float v, float* sh) {
  v = dpp_step<MAX, 0xB1>(v);    // quad_perm [1,0,3,2]
  v = dpp_step<MAX, 0x4E>(v);    // quad_perm [2,3,0,1]
  v = dpp_step<MAX, 0x141>(v);   // row_half_mirror
  v = dpp_step<MAX, 0x140>(v);   // row_mirror
  const int u = __builtin_bit_cast(int, v);
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(u, 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(u, 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(u, 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(u, 48));
  const float w = dpp_op<MAX>(dpp_op<MAX>(r0, r1), dpp_op<MAX>(r2, r3));
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = w;
  __syncthreads();
  return dpp_op<MAX>(dpp_op<MAX>(sh[0], sh[1]), dpp_op<MAX>(sh[2], sh[3]));
}
template <int CTRL>
__device__ __forceinline__ double dpp_add_d(double v) {   // v + (v of the DPP source lane), fp64 as two dword moves
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xf, 0xf, false);
  return v + __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ float block_max256(float v, float* sh) { return block_reduce256<true>(v, sh); }
__device__ __forceinline__ float block_sum256(float v, float* sh) { return block_reduce256<false>(v, sh); }

// Top eigenvector of the symmetric PSD 4x4 a (fp64, packed upper triangle t) by repeated squaring: each step
// M <- M^2 multiplies the eigenvalue ratios (l_i / l_1) by themselves, so after k steps M is l_1-dominated to
// (l_2 / l_1)^(2^k); M is rescaled by a power of two each step (exact, no division) and the loop stops when M is
// rank one to fp64 precision (tr(M^2) = tr(M)^2), at most 40 steps. The eigenvector is M's column of largest
// diagonal entry, polished by two power steps with a. Replaces np.linalg.eig (classification_utils.py:137-141):
// <= 8 squarings after the Gershgorin shift below (<= 11 without it on every golden/random/near-uniform case; equal to
// numpy's eigenvector in float32), a short dependent chain of independent FMAs where cyclic Jacobi spent ~20 us of
// fp64 divides and square roots on one lane.
__device__ void sym4_top_eigvec(const double t[10], double out[4]) {
  // packed upper triangle: 0:00 1:01 2:02 3:03 4:11 5:12 6:13 7:22 8:23 9:33
  double m[10];
  {
    // shift by (just under) the Gershgorin lower bound g <= l_4 of a: the eigenvectors stay, every shifted
    // eigenvalue stays >= 0 and the ratio (l_2 - g) / (l_1 - g) < l_2 / l_1 -- near-flat softmaxes (a ~ I/4, the
    // slow case) converge in ~7 squarings instead of ~10; peaked ones have g <= 0 and keep sigma = 0
    const double g0 = t[0] - (fabs(t[1]) + fabs(t[2]) + fabs(t[3]));
    const double g1 = t[4] - (fabs(t[1]) + fabs(t[5]) + fabs(t[6]));
    const double g2 = t[7] - (fabs(t[2]) + fabs(t[5]) + fabs(t[8]));
    const double g3 = t[9] - (fabs(t[3]) + fabs(t[6]) + fabs(t[8]));
    const double sg = fmax(0.0, fmin(fmin(g0, g1), fmin(g2, g3))) * (1.0 - 0x1p-10);
#pragma unroll
    for (int k = 0; k < 10; ++k) m[k] = t[k];
    m[0] -= sg; m[4] -= sg; m[7] -= sg; m[9] -= sg;
    int e;
    frexp((m[0] + m[4]) + (m[7] + m[9]), &e);
#pragma unroll
    for (int k = 0; k < 10; ++k) m[k] = ldexp(m[k], -e);
  }
  for (int it = 0; it < 40; ++it) {
    const double m00 = m[0], m01 = m[1], m02 = m[2], m03 = m[3], m11 = m[4], m12 = m[5], m13 = m[6], m22 = m[7],
                 m23 = m[8], m33 = m[9];
    const double trm = (m00 + m11) + (m22 + m33);
    double q[10];
    q[0] = m00 * m00 + m01 * m01 + m02 * m02 + m03 * m03;
    q[1] = m00 * m01 + m01 * m11 + m02 * m12 + m03 * m13;
    q[2] = m00 * m02 + m01 * m12 + m02 * m22 + m03 * m23;
    q[3] = m00 * m03 + m01 * m13 + m02 * m23 + m03 * m33;
    q[4] = m01 * m01 + m11 * m11 + m12 * m12 + m13 * m13;
    q[5] = m01 * m02 + m11 * m12 + m12 * m22 + m13 * m23;
    q[6] = m01 * m03 + m11 * m13 + m12 * m23 + m13 * m33;
    q[7] = m02 * m02 + m12 * m12 + m22 * m22 + m23 * m23;
    q[8] = m02 * m03 + m12 * m13 + m22 * m23 + m23 * m33;
    q[9] = m03 * m03 + m13 * m13 + m23 * m23 + m33 * m33;
    const double tr = (q[0] + q[4]) + (q[7] + q[9]);
    int e;
    frexp(tr, &e);
#pragma unroll
    for (int k = 0; k < 10; ++k) m[k] = ldexp(q[k], -e);
    if (tr >= (1.0 - 1e-15) * (trm * trm)) break;   // M was rank one: tr(M^2) = tr(M)^2
  }
  // column of the largest diagonal entry (static indices only: no scratch)
  double v[4] = {m[0], m[1], m[2], m[3]}, bd = m[0];
  if (m[4] > bd) { bd = m[4]; v[0] = m[1]; v[1] = m[4]; v[2] = m[5]; v[3] = m[6]; }
  if (m[7] > bd) { bd = m[7]; v[0] = m[2]; v[1] = m[5]; v[2] = m[7]; v[3] = m[8]; }
  if (m[9] > bd) { v[0] = m[3]; v[1] = m[6]; v[2] = m[8]; v[3] = m[9]; }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const double w0 = t[0] * v[0] + t[1] * v[1] + t[2] * v[2] + t[3] * v[3];
    const double w1 = t[1] * v[0] + t[4] * v[1] + t[5] * v[2] + t[6] * v[3];
    const double w2 = t[2] * v[0] + t[5] * v[1] + t[7] * v[2] + t[8] * v[3];
    const double w3 = t[3] * v[0] + t[6] * v[1] + t[8] * v[2] + t[9] * v[3];
    const double n = 1.0 / sqrt((w0 * w0 + w1 * w1) + (w2 * w2 + w3 * w3));
    v[0] = w0 * n; v[1] = w1 * n; v[2] = w2 * n; v[3] = w3 * n;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) out[k] = v[k];
}

// ------------------------------------------------------------------------------------------ decode ori
// One 256-thread workgroup per image; the image's logits stay in registers (PER per thread, n <= 256 PER) from one
// global read. Softmax in float32 as SPEUtils.last_activ; the ten fp64 moments of a = sum_i p_i q_i q_i^T are
// reduced through LDS (each of 160 threads sums 16 interleaved partials, each 16-lane row sums those by DPP: a fixed
// order).
// It also writes the image's whole status word (the decode's first kernel: no memset launch) and, in position
// regression mode, copies the 3 raw position outputs (no copy launch): pos_src == nullptr skips the copy.
template <int PER>
__global__ __launch_bounds__(256) void decode_ori_kernel(const float* __restrict__ logits, int n,
                                                         const double* __restrict__ qb, float* __restrict__ soft,
                                                         float* __restrict__ quat, int* __restrict__ status,
                                                         const float* __restrict__ pos_src, float* __restrict__ pos) {
  __shared__ float shf[2][4];
  __shared__ double shd[10][256];
  __shared__ double shp[10][16];
  const int tid = threadIdx.x, b = blockIdx.x;
  SPEF_TRACE(0);   // timeline probes (tools/kbench/head_bench.hip trace): nothing in the library build
  if (pos_src && tid < 3) pos[3 * b + tid] = pos_src[3 * b + tid];
  const float* x = logits + (size_t)b * n;
  float v[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = tid + 256 * j;
    v[j] = i < n ? x[i] : -INFINITY;
  }
  // the bin quaternions are loaded with the logits (PER <= 8: 64 VGPRs), not after the softmax: in the network the
  // forward has evicted them, and that second dependent HBM round trip was 40 % of the kernel (head_bench trace)
  constexpr bool PF = PER <= 8;
  double4 qv[PF ? PER : 1];
  if constexpr (PF) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + 256 * j;
      qv[j] = *reinterpret_cast<const double4*>(qb + 4 * (i < n ? i : 0));
    }
  }
  float m = v[0];
#pragma unroll
  for (int j = 1; j < PER; ++j) m = fmaxf(m, v[j]);
  SPEF_TRACE(1);
  m = block_max256(m, shf[0]);
  SPEF_TRACE(2);
  float s = 0.0f;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    v[j] = tid + 256 * j < n ? expf(v[j] - m) : 0.0f;
    s += v[j];
  }
  s = block_sum256(s, shf[1]);
  SPEF_TRACE(3);
  double mom[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) mom[k] = 0.0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = tid + 256 * j;
    if (i < n) {
      const float p = v[j] / s;
      if (soft) soft[(size_t)b * n + i] = p;
      const double pd = (double)p;
      double4 q;
      if constexpr (PF) q = qv[j];
      else q = *reinterpret_cast<const double4*>(qb + 4 * i);
      mom[0] += (q.x * q.x) * pd; mom[1] += (q.x * q.y) * pd; mom[2] += (q.x * q.z) * pd; mom[3] += (q.x * q.w) * pd;
      mom[4] += (q.y * q.y) * pd; mom[5] += (q.y * q.z) * pd; mom[6] += (q.y * q.w) * pd;
      mom[7] += (q.z * q.z) * pd; mom[8] += (q.z * q.w) * pd; mom[9] += (q.w * q.w) * pd;
    }
  }
  SPEF_TRACE(4);
#pragma unroll
  for (int k = 0; k < 10; ++k) shd[k][tid] = mom[k];
  __syncthreads();
  SPEF_TRACE(5);
  if (tid < 160) {   // 16-lane row k sums moment k: 16 partials per lane, then the row by DPP
    const int k = tid >> 4, j = tid & 15;
    double a = 0.0;
#pragma unroll
    for (int r = 0; r < 16; ++r) a += shd[k][j + 16 * r];
    a = dpp_add_d<0xB1>(a);    // quad_perm [1,0,3,2]
    a = dpp_add_d<0x4E>(a);    // quad_perm [2,3,0,1]
    a = dpp_add_d<0x141>(a);   // row_half_mirror
    a = dpp_add_d<0x140>(a);   // row_mirror
    if (j == 0) shp[k][0] = a;
  }
  __syncthreads();
  SPEF_TRACE(6);
  if (tid != 0) return;
  double t[10];
  bool nan = false;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    t[k] = shp[k][0];
    nan |= isnan(t[k]);
  }
  status[b] = nan ? 1 : 0;
  if (nan) {  // classification_utils.py:134-135
    for (int k = 0; k < 4; ++k) quat[4 * b + k] = NAN;
    return;
  }
  double q[4];
  SPEF_TRACE(7);
  sym4_top_eigvec(t, q);
  for (int k = 0; k < 4; ++k) quat[4 * b + k] = (float)q[k];
  SPEF_TRACE(8);
}

// ------------------------------------------------------------------------------------------ decode pos
__global__ __launch_bounds__(256) void decode_pos_kernel(const float* __restrict__ logits, int n,
                                                         const double* __restrict__ grid, float* __restrict__ soft,
                                                         float* __restrict__ pos, int* __restrict__ status) {
  __shared__ float shf[2][4];
  __shared__ double shd[4][3];
  __shared__ float shp[4];
  const int b = blockIdx.x;
  const float* x = logits + (size_t)b * n;
  float m = -INFINITY;
  for (int i = threadIdx.x; i < n; i += 256) m = fmaxf(m, x[i]);
  m = block_max256(m, shf[0]);
  float s = 0.0f;
  for (int i = threadIdx.x; i < n; i += 256) s += expf(x[i] - m);
  s = block_sum256(s, shf[1]);
  double acc[3] = {0.0, 0.0, 0.0};
  float ps = 0.0f;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float p = expf(x[i] - m) / s;
    if (soft) soft[(size_t)b * n + i] = p;
    ps += p;
    const double pd = (double)p;
    acc[0] += grid[3 * i] * pd;
    acc[1] += grid[3 * i + 1] * pd;
    acc[2] += grid[3 * i + 2] * pd;
  }
  ps = warp_sum(ps);
  for (int k = 0; k < 3; ++k) acc[k] = warp_sum_d(acc[k]);
  if ((threadIdx.x & 63) == 0) {
    shp[threadIdx.x >> 6] = ps;
    for (int k = 0; k < 3; ++k) shd[threadIdx.x >> 6][k] = acc[k];
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const float tot = (shp[0] + shp[1]) + (shp[2] + shp[3]);
  if (tot == 0.0f) status[b] |= 2;  // classification_utils.py:253-254
  for (int k = 0; k < 3; ++k) {
    const double v = ((shd[0][k] + shd[1][k]) + (shd[2][k] + shd[3][k])) / (double)tot;
    if (isnan(v)) status[b] |= 4;  // classification_utils.py:262-263
    pos[3 * b + k] = (float)v;
  }
}

__global__ void normalize_ori_kernel(const float* __restrict__ raw, int B, float* __restrict__ quat,
                                     int* __restrict__ status, const float* __restrict__ pos_src,
                                     float* __restrict__ pos) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  status[b] = 0;   // as decode_ori_kernel: the decode's first kernel owns the status word and the position copy
  if (pos_src)
    for (int k = 0; k < 3; ++k) pos[3 * b + k] = pos_src[3 * b + k];
  const float4 q = *reinterpret_cast<const float4*>(raw + 4 * b);
  const float n = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  *reinterpret_cast<float4*>(quat + 4 * b) = make_float4(q.x / n, q.y / n, q.z / n, q.w / n);
}

// ------------------------------------------------------------------------------------------ launchers
hipError_t launch_fc(const float* x, const float* w, const float* bias, float* out0, int n0, float* out1, int n1, int B,
                     int K, hipStream_t s) {
  if (K % 16) return hipErrorInvalidValue;
  const int Np = (n0 + n1 + 15) & ~15;
  const int64_t nwg = (int64_t)(Np / 16) * ((B + 15) / 16);
  if (nwg > 0x7fffffff) return hipErrorInvalidValue;
  fc_kernel<<<(uint32_t)nwg, 256, 0, s>>>(x, w, bias, out0, n0, out1, n1, B, K, Np);
  return hipGetLastError();
}

hipError_t launch_fc_splitk(const float* x, const float* w, const float* bias, float* out, int n, int B, int K,
                            int splits, float* part, hipStream_t s) {
  if (K % 16) return hipErrorInvalidValue;
  const int Np = (n + 15) & ~15;
  int kslice = (K + splits - 1) / splits;
  kslice = (kslice + 63) / 64 * 64;
  splits = (K + kslice - 1) / kslice;
  const int64_t nwg = (int64_t)(Np / 16) * ((B + 15) / 16) * splits;
  if (nwg > 0x7fffffff) return hipErrorInvalidValue;
  fc_partial_kernel<<<(uint32_t)nwg, 256, 0, s>>>(x, w, part, B, K, Np, kslice);
  fc_reduce_kernel<<<(B * n + 255) / 256, 256, 0, s>>>(part, bias, out, n, B, Np, splits);
  return hipGetLastError();
}

hipError_t launch_decode_ori(const float* logits, int B, int n_bins, const double* q_bins, float* soft, float* quat,
                             int* status, const float* pos_src, float* pos, hipStream_t s) {
  if (n_bins <= 256 * 8)
    decode_ori_kernel<8><<<B, 256, 0, s>>>(logits, n_bins, q_bins, soft, quat, status, pos_src, pos);
  else if (n_bins <= 256 * 32)
    decode_ori_kernel<32><<<B, 256, 0, s>>>(logits, n_bins, q_bins, soft, quat, status, pos_src, pos);
  else
    return hipErrorInvalidValue;   // more than 8192 orientation bins (20^3 = 8000 is the largest cubic grid)
  return hipGetLastError();
}

hipError_t launch_normalize_ori(const float* raw, int B, float* quat, int* status, const float* pos_src, float* pos,
                                hipStream_t s) {
  normalize_ori_kernel<<<(B + 255) / 256, 256, 0, s>>>(raw, B, quat, status, pos_src, pos);
  return hipGetLastError();
}

hipError_t launch_decode_pos(const float* logits, int B, int n_bins, const double* grid, float* soft, float* pos,
                             int* status, hipStream_t s) {
  decode_pos_kernel<<<B, 256, 0, s>>>(logits, n_bins, grid, soft, pos, status);
  return hipGetLastError();
}

}  // namespace spef
