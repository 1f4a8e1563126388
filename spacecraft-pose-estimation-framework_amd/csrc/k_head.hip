// Head and decode kernels on gfx950.
//
//   fc_kernel          URSONetHead Linear layers (src/modeling/head/ursonet.py:17-25), ori and pos weights
//                      concatenated into one fp32 GEMM on the exact f32-input MFMA (v_mfma_f32_16x16x4_f32)
//   decode_ori_kernel  SPEUtils.last_activ softmax (src/spe/spe_utils.py:75-76) fused with
//                      OrientationSoftClassification.decode (src/spe/classification_utils.py:113-146):
//                      a = sum_i p_i q_i q_i^T in fp64, top eigenvector by cyclic Jacobi, normalised
//   decode_pos_kernel  softmax (spe_utils.py:78-79) + PositionSoftClassification.decode
//                      (classification_utils.py:242-267): 3-D soft-argmax over the bin grid
//   normalize_ori      orientation regression L2 normalisation (spe_utils.py:72)
// One 256-thread workgroup decodes one image (the reference loops over images in Python,
// classification_utils.py:163-164).
#include <math.h>

#include "spef_common.hpp"
#include "spef_kernels.hpp"

namespace spef {

// ------------------------------------------------------------------------------------------ fc
// out[b][i] = sum_k X[b][k] W[i][k] + bias[i]. One workgroup per 16x16 output tile; its 4 waves take
// interleaved quarters of K (split-K inside the workgroup, reduced through LDS in a fixed order, so the
// result is deterministic). Lane l loads float4 W[i0+(l&15)][t+4(l>>4)..] and X[j0+(l&15)][t+4(l>>4)..];
// MFMA step e takes element e from both, so A and B see the same k.
__global__ __launch_bounds__(256) void fc_kernel(const float* __restrict__ X, const float* __restrict__ W,
                                                 const float* __restrict__ bias, float* __restrict__ out0, int n0,
                                                 float* __restrict__ out1, int n1, int B, int K, int Np) {
  __shared__ f32x4 part[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i0 = blockIdx.x * 16;
  const int j0 = blockIdx.y * 16;
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
  const int i0 = blockIdx.x * 16, j0 = blockIdx.y * 16, z = blockIdx.z;
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
  float v = bias[i];
  for (int z = 0; z < splits; ++z) v += part[((size_t)z * B + j) * Np + i];
  out[(size_t)j * n + i] = v;
}

// ------------------------------------------------------------------------------------------ reductions
__device__ __forceinline__ float block_max256(float v, float* sh) {
  v = warp_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
}
__device__ __forceinline__ float block_sum256(float v, float* sh) {
  v = warp_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// Cyclic Jacobi on a symmetric 4x4 (fp64): returns the unit eigenvector of the largest eigenvalue.
__device__ void sym4_top_eigvec(double a[4][4], double out[4]) {
  double v[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
  for (int sweep = 0; sweep < 32; ++sweep) {
    double off = 0.0, diag = 0.0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      diag += a[p][p] * a[p][p];
#pragma unroll
      for (int q = p + 1; q < 4; ++q) off += a[p][q] * a[p][q];
    }
    if (off <= 1e-34 * diag || off == 0.0) break;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int q = p + 1; q < 4; ++q) {
        const double apq = a[p][q];
        if (apq == 0.0) continue;
        const double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 4; ++k) {  // A <- A J (columns p, q)
          const double akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - s * akq;
          a[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 4; ++k) {  // A <- J^T A (rows p, q)
          const double apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - s * aqk;
          a[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 4; ++k) {  // V <- V J
          const double vkp = v[k][p], vkq = v[k][q];
          v[k][p] = c * vkp - s * vkq;
          v[k][q] = s * vkp + c * vkq;
        }
      }
  }
  // column of the largest diagonal entry, selected with static indices only (no scratch)
  double bd = a[0][0], col[4] = {v[0][0], v[1][0], v[2][0], v[3][0]};
#pragma unroll
  for (int p = 1; p < 4; ++p)
    if (a[p][p] > bd) {
      bd = a[p][p];
#pragma unroll
      for (int k = 0; k < 4; ++k) col[k] = v[k][p];
    }
  double n = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) n += col[k] * col[k];
  n = sqrt(n);
#pragma unroll
  for (int k = 0; k < 4; ++k) out[k] = col[k] / n;
}

// ------------------------------------------------------------------------------------------ decode ori
__global__ __launch_bounds__(256) void decode_ori_kernel(const float* __restrict__ logits, int n,
                                                         const double* __restrict__ qb, float* __restrict__ soft,
                                                         float* __restrict__ quat, int* __restrict__ status) {
  __shared__ float shf[4];
  __shared__ double shd[4][10];
  const int b = blockIdx.x;
  const float* x = logits + (size_t)b * n;
  float m = -INFINITY;
  for (int i = threadIdx.x; i < n; i += 256) m = fmaxf(m, x[i]);
  m = block_max256(m, shf);
  float s = 0.0f;
  for (int i = threadIdx.x; i < n; i += 256) s += expf(x[i] - m);
  s = block_sum256(s, shf);
  double mom[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) mom[k] = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float p = expf(x[i] - m) / s;
    if (soft) soft[(size_t)b * n + i] = p;
    const double pd = (double)p;
    const double q0 = qb[4 * i], q1 = qb[4 * i + 1], q2 = qb[4 * i + 2], q3 = qb[4 * i + 3];
    mom[0] += (q0 * q0) * pd; mom[1] += (q0 * q1) * pd; mom[2] += (q0 * q2) * pd; mom[3] += (q0 * q3) * pd;
    mom[4] += (q1 * q1) * pd; mom[5] += (q1 * q2) * pd; mom[6] += (q1 * q3) * pd;
    mom[7] += (q2 * q2) * pd; mom[8] += (q2 * q3) * pd; mom[9] += (q3 * q3) * pd;
  }
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    const double w = warp_sum_d(mom[k]);
    if ((threadIdx.x & 63) == 0) shd[threadIdx.x >> 6][k] = w;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  double t[10];
  bool nan = false;
  for (int k = 0; k < 10; ++k) {
    t[k] = (shd[0][k] + shd[1][k]) + (shd[2][k] + shd[3][k]);
    nan |= isnan(t[k]);
  }
  if (nan) {  // classification_utils.py:134-135
    status[b] |= 1;
    for (int k = 0; k < 4; ++k) quat[4 * b + k] = NAN;
    return;
  }
  double a[4][4] = {{t[0], t[1], t[2], t[3]}, {t[1], t[4], t[5], t[6]}, {t[2], t[5], t[7], t[8]}, {t[3], t[6], t[8], t[9]}};
  double q[4];
  sym4_top_eigvec(a, q);
  for (int k = 0; k < 4; ++k) quat[4 * b + k] = (float)q[k];
}

// ------------------------------------------------------------------------------------------ decode pos
__global__ __launch_bounds__(256) void decode_pos_kernel(const float* __restrict__ logits, int n,
                                                         const double* __restrict__ grid, float* __restrict__ soft,
                                                         float* __restrict__ pos, int* __restrict__ status) {
  __shared__ float shf[4];
  __shared__ double shd[4][3];
  __shared__ float shp[4];
  const int b = blockIdx.x;
  const float* x = logits + (size_t)b * n;
  float m = -INFINITY;
  for (int i = threadIdx.x; i < n; i += 256) m = fmaxf(m, x[i]);
  m = block_max256(m, shf);
  float s = 0.0f;
  for (int i = threadIdx.x; i < n; i += 256) s += expf(x[i] - m);
  s = block_sum256(s, shf);
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

__global__ void normalize_ori_kernel(const float* __restrict__ raw, int B, float* __restrict__ quat) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const float4 q = *reinterpret_cast<const float4*>(raw + 4 * b);
  const float n = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  *reinterpret_cast<float4*>(quat + 4 * b) = make_float4(q.x / n, q.y / n, q.z / n, q.w / n);
}

// ------------------------------------------------------------------------------------------ launchers
hipError_t launch_fc(const float* x, const float* w, const float* bias, float* out0, int n0, float* out1, int n1, int B,
                     int K, hipStream_t s) {
  if (K % 16) return hipErrorInvalidValue;
  const int Np = (n0 + n1 + 15) & ~15;
  dim3 g(Np / 16, (B + 15) / 16);
  fc_kernel<<<g, 256, 0, s>>>(x, w, bias, out0, n0, out1, n1, B, K, Np);
  return hipGetLastError();
}

hipError_t launch_fc_splitk(const float* x, const float* w, const float* bias, float* out, int n, int B, int K,
                            int splits, float* part, hipStream_t s) {
  if (K % 16) return hipErrorInvalidValue;
  const int Np = (n + 15) & ~15;
  int kslice = (K + splits - 1) / splits;
  kslice = (kslice + 63) / 64 * 64;
  splits = (K + kslice - 1) / kslice;
  dim3 g(Np / 16, (B + 15) / 16, splits);
  fc_partial_kernel<<<g, 256, 0, s>>>(x, w, part, B, K, Np, kslice);
  fc_reduce_kernel<<<(B * n + 255) / 256, 256, 0, s>>>(part, bias, out, n, B, Np, splits);
  return hipGetLastError();
}

hipError_t launch_decode_ori(const float* logits, int B, int n_bins, const double* q_bins, float* soft, float* quat,
                             int* status, hipStream_t s) {
  decode_ori_kernel<<<B, 256, 0, s>>>(logits, n_bins, q_bins, soft, quat, status);
  return hipGetLastError();
}

hipError_t launch_normalize_ori(const float* raw, int B, float* quat, hipStream_t s) {
  normalize_ori_kernel<<<(B + 255) / 256, 256, 0, s>>>(raw, B, quat);
  return hipGetLastError();
}

hipError_t launch_decode_pos(const float* logits, int B, int n_bins, const double* grid, float* soft, float* pos,
                             int* status, hipStream_t s) {
  decode_pos_kernel<<<B, 256, 0, s>>>(logits, n_bins, grid, soft, pos, status);
  return hipGetLastError();
}

}  // namespace spef
