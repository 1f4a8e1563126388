// Batched keypoint decode: SPEUtils.last_activ sigmoid (src/spe/spe_utils.py:68) + KeyPoints.pnp
// (src/spe/keypoints_utils.py:112-150) = cv2.solvePnP(SOLVEPNP_EPNP) -> Rodrigues -> dcm2quat (spe/utils.py:56-118),
// including solvePnP's undistortPoints for cameras with lens distortion (SPEED+, data/datasets/speed_plus.py:18-40).
//
// One 3-wave workgroup per problem, fp64; the algorithm is OpenCV 4.5.5 epnp.cpp's (the reference's pinned OpenCV):
// PCA control points, barycentric alphas, M (2n x 12), the 4 eigenvectors of M^T M with the smallest
// eigenvalues, L_6x10 / rho, beta approximations 1/2/3 (least squares), 5 Gauss-Newton steps (Householder
// QR), R|t by Procrustes with OpenCV's sign fixes, lowest mean reprojection error wins. Symmetric
// eigenproblems use Jacobi (fp64: the 12x12 one lane-parallel in tournament order, the 3x3 one cyclic) instead of
// LAPACK/cvSVD -- same subspaces, independent of the eigenvector signs. Rodrigues(rvec(R)) == R, so R goes straight
// to the Spurrier quaternion.
#include <math.h>

#include "spef_common.hpp"
#include "spef_kernels.hpp"

namespace spef {

#define EPNP_MAXN 16

// Jacobi rotation (c, s) annihilating a_pq: theta = (a_qq - a_pp) / (2 a_pq), t = sign(theta) / (|theta| +
// sqrt(theta^2 + 1)), c = 1 / sqrt(t^2 + 1), s = t c. The reciprocals and square roots are the hardware fp64
// estimates (v_rcp_f64 / v_rsq_f64) refined by Newton steps instead of the IEEE-correct library sequences (scaling,
// fixup): a rotation only has to be orthogonal to fp64 precision, not correctly rounded, and these four operations are
// the serial latency of every Jacobi round (the rounds are ~55 % of the kernel, tools/epnp_time.py ablations).
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  return fma(r, fma(-x, r, 1.0), r);
}
__device__ __forceinline__ double rsq_nr(double x) {   // x > 0
  double r = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  r = r * fma(-h * r, r, 1.5);
  return r * fma(-h * r, r, 1.5);
}
// Division and square root in the small serial solves (QR least squares, Gauss-Newton, Procrustes): the same
// hardware-estimate + Newton forms (a x (1/b) is within an ulp or two of a / b, against ~15 dependent instructions of
// the IEEE division sequence on one lane's critical path).
__device__ __forceinline__ double ddiv(double a, double b) { return a * rcp_nr(b); }
__device__ __forceinline__ double dsqrt(double x) { return x > 0.0 ? x * rsq_nr(x) : 0.0; }   // x >= 0
// The angle in fp32 (fast rcp / sqrt), the rotation itself orthogonal to fp64 for that angle. Where fp32 cannot
// represent 2 a_pq (|a_pq| below ~1e-38 while the fp64 skip guard let it through) or the fp32 angle is not finite,
// the rotation is the fp64 form below, so no 0 x inf reaches (c, s).
__device__ __forceinline__ void jacobi_rot(double app, double aqq, double apq, double& c, double& s) {
  const float den = (float)(2.0 * apq);
  if (fabsf(den) >= 1.17549435e-38f) {   // FLT_MIN: a normal fp32 divisor
    const float th = (float)(aqq - app) * __builtin_amdgcn_rcpf(den);
    if (__builtin_isfinite(th)) {
      const float tf = (th >= 0 ? 1.0f : -1.0f) * __builtin_amdgcn_rcpf(fabsf(th) + __builtin_sqrtf(th * th + 1.0f));
      const double t = (double)tf;
      c = rsq_nr(t * t + 1.0);
      s = t * c;
      return;
    }
  }
  const double theta = (aqq - app) * rcp_nr(2.0 * apq);
  double t;
  if (fabs(theta) > 1e100) {                             // sqrt(theta^2 + 1) = |theta| to fp64: t = 1 / (2 theta)
    t = 0.5 * rcp_nr(theta);
  } else {
    const double t2 = theta * theta + 1.0;
    const double sq = t2 * rsq_nr(t2);                   // sqrt(theta^2 + 1)
    t = (theta >= 0 ? 1.0 : -1.0) * rcp_nr(fabs(theta) + sq);
  }
  c = rsq_nr(t * t + 1.0);
  s = t * c;
}

// cyclic Jacobi on a symmetric N x N: a is destroyed (diagonal = eigenvalues), v = eigenvectors (columns)
template <int N>
__device__ void jacobi_sym(double (&a)[N][N], double (&v)[N][N]) {
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) v[i][j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 40; ++sweep) {
    double off = 0.0, diag = 0.0;
    for (int p = 0; p < N; ++p) {
      diag += a[p][p] * a[p][p];
      for (int q = p + 1; q < N; ++q) off += a[p][q] * a[p][q];
    }
    if (off <= 1e-32 * diag || off == 0.0) break;
    for (int p = 0; p < N - 1; ++p)
      for (int q = p + 1; q < N; ++q) {
        const double apq = a[p][q];
        if (fabs(apq) < 1e-300) continue;
        double c, s;
        jacobi_rot(a[p][p], a[q][q], apq, c, s);
        for (int k = 0; k < N; ++k) {
          const double akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - s * akq;
          a[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < N; ++k) {
          const double apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - s * aqk;
          a[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < N; ++k) {
          const double vkp = v[k][p], vkq = v[k][q];
          v[k][p] = c * vkp - s * vkq;
          v[k][q] = s * vkp + c * vkq;
        }
      }
  }
}

// least squares min ||A x - b|| for a full-column-rank 6 x NC A by Householder QR (epnp.cpp qr_solve)
template <int NC>
__device__ void qr_lstsq(double (&A)[6][NC], double (&b)[6], double (&x)[NC]) {
  double ia1[NC], ia2[NC];   // reciprocals of epnp.cpp's A1 / A2 (the only form the solve uses)
  for (int k = 0; k < NC; ++k) {
    double eta = 0.0;
    for (int i = k; i < 6; ++i) eta = fmax(eta, fabs(A[i][k]));
    if (eta == 0.0) {
      for (int j = 0; j < NC; ++j) x[j] = 0.0;
      return;
    }
    const double inv = ddiv(1.0, eta);
    double sum2 = 0.0;
    for (int i = k; i < 6; ++i) {
      A[i][k] *= inv;
      sum2 += A[i][k] * A[i][k];
    }
    double sigma = dsqrt(sum2);
    if (A[k][k] < 0) sigma = -sigma;
    A[k][k] += sigma;
    ia1[k] = ddiv(1.0, sigma * A[k][k]);
    ia2[k] = ddiv(1.0, -eta * sigma);
    for (int j = k + 1; j < NC; ++j) {
      double sum = 0.0;
      for (int i = k; i < 6; ++i) sum += A[i][k] * A[i][j];
      const double tau = sum * ia1[k];
      for (int i = k; i < 6; ++i) A[i][j] -= tau * A[i][k];
    }
  }
  for (int j = 0; j < NC; ++j) {
    double tau = 0.0;
    for (int i = j; i < 6; ++i) tau += A[i][j] * b[i];
    tau *= ia1[j];
    for (int i = j; i < 6; ++i) b[i] -= tau * A[i][j];
  }
  x[NC - 1] = b[NC - 1] * ia2[NC - 1];
  for (int i = NC - 2; i >= 0; --i) {
    double sum = 0.0;
    for (int j = i + 1; j < NC; ++j) sum += A[i][j] * x[j];
    x[i] = (b[i] - sum) * ia2[i];
  }
}

__device__ __forceinline__ void epnp_gn(const double (&L)[6][10], const double (&rho)[6], double (&b)[4]) {
  for (int it = 0; it < 5; ++it) {
    double A[6][4], r[6], x[4];
    for (int i = 0; i < 6; ++i) {
      const double* l = L[i];
      A[i][0] = 2 * l[0] * b[0] + l[1] * b[1] + l[3] * b[2] + l[6] * b[3];
      A[i][1] = l[1] * b[0] + 2 * l[2] * b[1] + l[4] * b[2] + l[7] * b[3];
      A[i][2] = l[3] * b[0] + l[4] * b[1] + 2 * l[5] * b[2] + l[8] * b[3];
      A[i][3] = l[6] * b[0] + l[7] * b[1] + l[8] * b[2] + 2 * l[9] * b[3];
      r[i] = rho[i] - (l[0] * b[0] * b[0] + l[1] * b[0] * b[1] + l[2] * b[1] * b[1] + l[3] * b[0] * b[2] +
                       l[4] * b[1] * b[2] + l[5] * b[2] * b[2] + l[6] * b[0] * b[3] + l[7] * b[1] * b[3] +
                       l[8] * b[2] * b[3] + l[9] * b[3] * b[3]);
    }
    qr_lstsq<4>(A, r, x);
    for (int i = 0; i < 4; ++i) b[i] += x[i];
  }
}

// cv::undistortPoints as solvePnP(SOLVEPNP_EPNP) applies it before EPnP (OpenCV 4.5.5 solvepnp.cpp;
// undistort.dispatch.cpp cvUndistortPointsInternal, default criteria COUNT = 5) followed by epnp::init_points'
// re-projection with K: x = (u - cx) * (1/fx); five fixed-point steps x <- (x0 - delta(x)) * icdist(x) (5-coefficient
// model: k1 k2 p1 p2 k3); the normalised point is stored as float32 (the reference's points are float32) and
// re-projected in double, us = x fu + uc. Without distortion only that float32 round trip remains (the reference
// always passes distCoeffs, zeros for SPEED: keypoints_utils.py:136-142).
__device__ __forceinline__ void undistort_point(const EpnpDist& d, double fu, double fv, double uc, double vc,
                                                float uf, float vf, double& u_out, double& v_out) {
  const double ifx = 1.0 / fu, ify = 1.0 / fv;
  const double x0 = ((double)uf - uc) * ifx, y0 = ((double)vf - vc) * ify;
  double x = x0, y = y0;
  if (d.on) {
    for (int it = 0; it < 5; ++it) {
      const double r2 = x * x + y * y;
      const double icdist = 1.0 / (1.0 + ((d.k3 * r2 + d.k2) * r2 + d.k1) * r2);
      if (icdist < 0) {
        x = x0;
        y = y0;
        break;
      }
      const double dx = 2 * d.p1 * x * y + d.p2 * (r2 + 2 * x * x);
      const double dy = d.p1 * (r2 + 2 * y * y) + 2 * d.p2 * x * y;
      x = (x0 - dx) * icdist;
      y = (y0 - dy) * icdist;
    }
  }
  u_out = (double)(float)x * fu + uc;
  v_out = (double)(float)y * fv + vc;
}

// ---- one 3-wave workgroup per problem ----
// Every wave's lane i < n holds point i (its 3-D point, undistorted pixel, barycentric alphas). The 12 x 12 symmetric
// eigenproblem of M^T M runs as a parallel (tournament-ordered) cyclic Jacobi in LDS: each of the 11 rounds of a sweep
// applies 6 disjoint rotations at once (wave 0's lanes 0..11 compute them), thread e < 144 updating entry e of A and of
// V (A' = J^T A J, V' = V J with J the product of the round's rotations), double-buffered. The three beta
// approximations of epnp.cpp compute_pose are independent: wave w runs approximation w + 1 (L_6x10 betas, 5
// Gauss-Newton steps, R|t by Procrustes, mean reprojection error) on its own lanes, and the lowest error wins (ties:
// the lower approximation, as epnp.cpp). The small fixed-size steps run uniformly on every lane of a wave; the per-point
// sums are wave reductions. Latency per problem is what all this buys (a B = 64 batch is 64 concurrent problems):
// one wave per problem took 134 us per launch, the former one-thread-per-problem kernel ~2 ms.

// partner of index i in round r of the 12-player round robin: pairs (r, 11) and (r + k, r - k) mod 11, k = 1..5
__device__ __forceinline__ int rr_partner(int r, int i) {
  if (i == 11) return r;
  if (i == r) return 11;
  return (2 * r - i + 22) % 11;
}

#ifndef SPEF_EPNP_JTOL   // Jacobi stops once off-diagonal^2 <= JTOL x diagonal^2
#define SPEF_EPNP_JTOL 1e-26
#endif
#ifndef SPEF_EPNP_WPE   // waves per SIMD the register allocation targets (0: the compiler's choice: 312 registers, one wave per SIMD; 2: 256 + a 200-B spill, two workgroups per CU -- P = 1800: 365 -> 232 us, B = 64 unchanged)
#define SPEF_EPNP_WPE 2
#endif
#if SPEF_EPNP_WPE
#define SPEF_EPNP_ATTR __attribute__((amdgpu_waves_per_eu(SPEF_EPNP_WPE)))
#else
#define SPEF_EPNP_ATTR
#endif
__global__ __launch_bounds__(192) SPEF_EPNP_ATTR void epnp_kernel(const float* __restrict__ raw, int B, int n,
                                                   const float* __restrict__ kp3d, const double* __restrict__ model,
                                                   double fu, double fv, double uc,
                                                   double vc, float nu, float nv, EpnpDist dist, int apply_sigmoid,
                                                   float* __restrict__ kp_out, float* __restrict__ quat,
                                                   float* __restrict__ pos, int* __restrict__ status) {
  __shared__ double As[2][144], Vs[2][144];
  __shared__ double Cc[12], Cs[12];
  __shared__ double Pal[EPNP_MAXN][4], Pdu[EPNP_MAXN], Pdv[EPNP_MAXN];
  __shared__ double Red[3][2];
  __shared__ double Ls[6][10], Rho[6];
  __shared__ double Res[3][13];   // per approximation: error, R (9), t (3)
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (b >= B) return;   // uniform per workgroup
  const int nk = 2 * (n + 1);

  // ---- points: lane i <= n reads raw point i (origin first); lane j < n then owns keypoint j (every wave)
  double uu = 0.0, vv = 0.0;
  if (lane <= n) {
    float x = raw[(size_t)b * nk + 2 * lane], y = raw[(size_t)b * nk + 2 * lane + 1];
    if (apply_sigmoid) {   // spe_utils.py:68, float32
      x = 1.0f / (1.0f + expf(-x));
      y = 1.0f / (1.0f + expf(-y));
    }
    if (kp_out && wave == 0) {
      kp_out[(size_t)b * nk + 2 * lane] = x;
      kp_out[(size_t)b * nk + 2 * lane + 1] = y;
    }
    // keypoints_utils.py:127-131: pixels (float32 products), origin dropped; then undistortPoints
    undistort_point(dist, fu, fv, uc, vc, x * nu, y * nv, uu, vv);
  }
  const double us0 = __shfl_down(uu, 1, 64), us1 = __shfl_down(vv, 1, 64);   // lane j: keypoint j = raw point j + 1
  const bool pt = lane < n;
  double pw[3] = {0, 0, 0}, al[4] = {0, 0, 0, 0};
  if (pt) {
#pragma unroll
    for (int k = 0; k < 3; ++k) pw[k] = (double)kp3d[3 * lane + k];
#pragma unroll
    for (int k = 0; k < 4; ++k) al[k] = model[12 + 4 * lane + k];
    if (wave == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) Pal[lane][k] = al[k];
      Pdu[lane] = uc - us0;
      Pdv[lane] = vc - us1;
    }
  }
  // control points: model[0..11] (model-only, spef_set_keypoints), read where used
  __syncthreads();

  // ---- M^T M (M never stored): entry e = (p, q) = thread e, accumulated point by point as r1[p] r1[q] + r2[p] r2[q]
  const int e = tid;
  const bool ent = e < 144;
  const int ei = e / 12, ej = e - 12 * (e / 12);
  if (ent) {
    const int cp = ei / 3, dp = ei - 3 * cp, cq = ej / 3, dq = ej - 3 * cq;
    double acc = 0.0;
    for (int i = 0; i < n; ++i) {
      const double ap = Pal[i][cp], aq = Pal[i][cq];
      const double r1p = dp == 0 ? ap * fu : dp == 2 ? ap * Pdu[i] : 0.0;
      const double r1q = dq == 0 ? aq * fu : dq == 2 ? aq * Pdu[i] : 0.0;
      const double r2p = dp == 1 ? ap * fv : dp == 2 ? ap * Pdv[i] : 0.0;
      const double r2q = dq == 1 ? aq * fv : dq == 2 ? aq * Pdv[i] : 0.0;
      acc += r1p * r1q + r2p * r2q;
    }
    As[0][e] = acc;
    Vs[0][e] = ei == ej ? 1.0 : 0.0;
  }
  __syncthreads();

  // ---- parallel cyclic Jacobi (tournament order): sweeps of 11 rounds x 6 disjoint rotations
  int cur = 0;
  for (int sweep = 0; sweep < 40; ++sweep) {
    double off = 0.0, diag = 0.0;
    if (ent) {
      const double a = As[cur][e];
      if (ei == ej) diag = a * a;
      else if (ei < ej) off = a * a;
    }
    off = warp_sum_d(off);
    diag = warp_sum_d(diag);
    if (lane == 0) {
      Red[wave][0] = off;
      Red[wave][1] = diag;
    }
    __syncthreads();
    off = Red[0][0] + Red[1][0] + Red[2][0];
    diag = Red[0][1] + Red[1][1] + Red[2][1];
    if (off <= SPEF_EPNP_JTOL * diag || off == 0.0) break;   // uniform: every thread read the same sums
    for (int r = 0; r < 11; ++r) {
      if (tid < 12) {   // thread i: the rotation of its pair, its own signed coefficient
        const int j = rr_partner(r, tid);
        const int p = tid < j ? tid : j, q = tid < j ? j : tid;
        const double apq = As[cur][12 * p + q];
        double c = 1.0, sn = 0.0;
        if (fabs(apq) >= 1e-300) jacobi_rot(As[cur][13 * p], As[cur][13 * q], apq, c, sn);
        Cc[tid] = c;
        Cs[tid] = tid == p ? -sn : sn;
      }
      __syncthreads();
      if (ent) {
        const int i2 = rr_partner(r, ei), j2 = rr_partner(r, ej);
        const double ci = Cc[ei], si = Cs[ei], cj = Cc[ej], sj = Cs[ej];
        const double* a = As[cur];
        As[cur ^ 1][e] = ci * (cj * a[12 * ei + ej] + sj * a[12 * ei + j2]) + si * (cj * a[12 * i2 + ej] + sj * a[12 * i2 + j2]);
        const double* v = Vs[cur];
        Vs[cur ^ 1][e] = cj * v[12 * ei + ej] + sj * v[12 * ei + j2];
      }
      cur ^= 1;
      __syncthreads();
    }
  }
  // the 4 eigenvectors of smallest eigenvalue, ascending (ties keep the lower index); static loops only (a
  // dynamically indexed private array would live in scratch)
  double ev[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) ev[i] = As[cur][13 * i];
  int idx[4];
  uint32_t used = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double best = INFINITY;
    int bi = 0;
#pragma unroll
    for (int j = 0; j < 12; ++j)
      if (!((used >> j) & 1u) && ev[j] < best) {
        best = ev[j];
        bi = j;
      }
    idx[i] = bi;
    used |= 1u << bi;
  }
  // ut4[i][k] = V[k][idx[i]] stays in LDS (read as broadcasts); L_6x10 rows and rho by threads 0..5 into LDS
  const double* Vf = Vs[cur];
  auto ut4 = [&](int i, int k) { return Vf[12 * k + idx[i]]; };
  if (tid < 6) {
    const int r = tid;
    const int pa = r < 3 ? 0 : r < 5 ? 1 : 2, pb = r < 3 ? r + 1 : r < 5 ? r - 1 : 3;
    double dv[4][3];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int k = 0; k < 3; ++k) dv[i][k] = ut4(i, 3 * pa + k) - ut4(i, 3 * pb + k);
    auto dot = [&](int i, int j) { return dv[i][0] * dv[j][0] + dv[i][1] * dv[j][1] + dv[i][2] * dv[j][2]; };
    Ls[r][0] = dot(0, 0);
    Ls[r][1] = 2 * dot(0, 1);
    Ls[r][2] = dot(1, 1);
    Ls[r][3] = 2 * dot(0, 2);
    Ls[r][4] = 2 * dot(1, 2);
    Ls[r][5] = dot(2, 2);
    Ls[r][6] = 2 * dot(0, 3);
    Ls[r][7] = 2 * dot(1, 3);
    Ls[r][8] = 2 * dot(2, 3);
    Ls[r][9] = dot(3, 3);
    double d2 = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double dk = model[3 * pa + k] - model[3 * pb + k];
      d2 += dk * dk;
    }
    Rho[r] = d2;
  }
  __syncthreads();
  // L_6x10 stays in LDS (read where used, broadcast): as 60 fp64 registers it held the kernel at 256+ VGPRs, one
  // wave per SIMD (one problem per CU at a time)
  const double (&L)[6][10] = Ls;
  double rho[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) rho[r] = Rho[r];
  // pw centroid (uniform): a wave reduction over the point lanes
  double pw0[3];
  const double inv_n = ddiv(1.0, (double)n);
#pragma unroll
  for (int k = 0; k < 3; ++k) pw0[k] = warp_sum_d(pw[k]) * inv_n;

  // ---- approximation ap = wave + 1 (epnp.cpp compute_pose: find_betas_approx_1/2/3 + gauss_newton + compute_R_and_t)
  const int ap = wave + 1;
  {
    double be[4] = {0, 0, 0, 0};
    double rr[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) rr[i] = rho[i];
    if (ap == 1) {
      double A[6][4], x[4];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        A[i][0] = L[i][0]; A[i][1] = L[i][1]; A[i][2] = L[i][3]; A[i][3] = L[i][6];
      }
      qr_lstsq<4>(A, rr, x);
      const double s = x[0] < 0 ? -1.0 : 1.0;
      be[0] = dsqrt(fabs(x[0]));
      const double ib = ddiv(s, be[0]);
      be[1] = x[1] * ib;
      be[2] = x[2] * ib;
      be[3] = x[3] * ib;
    } else if (ap == 2) {
      double A[6][3], x[3];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        A[i][0] = L[i][0]; A[i][1] = L[i][1]; A[i][2] = L[i][2];
      }
      qr_lstsq<3>(A, rr, x);
      if (x[0] < 0) {
        be[0] = dsqrt(-x[0]);
        be[1] = x[2] < 0 ? dsqrt(-x[2]) : 0.0;
      } else {
        be[0] = dsqrt(x[0]);
        be[1] = x[2] > 0 ? dsqrt(x[2]) : 0.0;
      }
      if (x[1] < 0) be[0] = -be[0];
    } else {
      double A[6][5], x[5];
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int k = 0; k < 5; ++k) A[i][k] = L[i][k];
      qr_lstsq<5>(A, rr, x);
      if (x[0] < 0) {
        be[0] = dsqrt(-x[0]);
        be[1] = x[2] < 0 ? dsqrt(-x[2]) : 0.0;
      } else {
        be[0] = dsqrt(x[0]);
        be[1] = x[2] > 0 ? dsqrt(x[2]) : 0.0;
      }
      if (x[1] < 0) be[0] = -be[0];
      be[2] = ddiv(x[3], be[0]);
    }
    epnp_gn(L, rho, be);
    // R|t (epnp.cpp compute_R_and_t): ccs uniform, pcs of point = lane, sums by wave reduction
    double ccs[4][3] = {};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 3; ++k) ccs[j][k] += be[i] * ut4(i, 3 * j + k);
    double pc[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) pc[j] = pt ? al[0] * ccs[0][j] + al[1] * ccs[1][j] + al[2] * ccs[2][j] + al[3] * ccs[3][j] : 0.0;
    if (__shfl(pc[2], 0, 64) < 0.0)   // solve_for_sign
#pragma unroll
      for (int j = 0; j < 3; ++j) pc[j] = -pc[j];
    double pc0[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) pc0[j] = warp_sum_d(pc[j]) * inv_n;
    double abt[3][3];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int k = 0; k < 3; ++k) abt[j][k] = warp_sum_d(pt ? (pc[j] - pc0[j]) * (pw[k] - pw0[k]) : 0.0);
    // R = U V^T of abt = U S V^T: V from eig(abt^T abt), U = abt V S^-1
    double ata[3][3], Vm[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) ata[i][j] = abt[0][i] * abt[0][j] + abt[1][i] * abt[1][j] + abt[2][i] * abt[2][j];
    jacobi_sym<3>(ata, Vm);
    double U[3][3], R[3][3], t[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      double col[3], nrm = 0.0;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        col[r] = abt[r][0] * Vm[0][c] + abt[r][1] * Vm[1][c] + abt[r][2] * Vm[2][c];
        nrm += col[r] * col[r];
      }
      const double inrm = nrm > 0 ? rsq_nr(nrm) : 0.0;
#pragma unroll
      for (int r = 0; r < 3; ++r) U[r][c] = col[r] * inrm;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) R[i][j] = U[i][0] * Vm[j][0] + U[i][1] * Vm[j][1] + U[i][2] * Vm[j][2];
    const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] + R[0][2] * R[1][0] * R[2][1] -
                       R[0][2] * R[1][1] * R[2][0] - R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
    if (det < 0)
#pragma unroll
      for (int j = 0; j < 3; ++j) R[2][j] = -R[2][j];
#pragma unroll
    for (int i = 0; i < 3; ++i) t[i] = pc0[i] - (R[i][0] * pw0[0] + R[i][1] * pw0[1] + R[i][2] * pw0[2]);
    double err = 0.0;
    if (pt) {
      const double xc = R[0][0] * pw[0] + R[0][1] * pw[1] + R[0][2] * pw[2] + t[0];
      const double yc = R[1][0] * pw[0] + R[1][1] * pw[1] + R[1][2] * pw[2] + t[1];
      const double iz = ddiv(1.0, R[2][0] * pw[0] + R[2][1] * pw[1] + R[2][2] * pw[2] + t[2]);
      const double ue = uc + fu * xc * iz, ve = vc + fv * yc * iz;
      err = dsqrt((us0 - ue) * (us0 - ue) + (us1 - ve) * (us1 - ve));
    }
    const double em = warp_sum_d(err) * inv_n;
    if (lane == 0) {
      Res[wave][0] = em;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) Res[wave][1 + 3 * i + j] = R[i][j];
        Res[wave][10 + i] = t[i];
      }
    }
  }
  __syncthreads();
  if (tid != 0) return;
  int bw = 0;   // lowest mean reprojection error; strict, so ties keep the lower approximation (epnp.cpp compute_pose)
  double bestE = Res[0][0];
  for (int w = 1; w < 3; ++w)
    if (Res[w][0] < bestE) {
      bestE = Res[w][0];
      bw = w;
    }
  double bestR[3][3], bestT[3];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) bestR[i][j] = Res[bw][1 + 3 * i + j];
    bestT[i] = Res[bw][10 + i];
  }
  // dcm2quat (spe/utils.py:56-118, Spurrier)
  const double m11 = bestR[0][0], m12 = bestR[0][1], m13 = bestR[0][2];
  const double m21 = bestR[1][0], m22 = bestR[1][1], m23 = bestR[1][2];
  const double m31 = bestR[2][0], m32 = bestR[2][1], m33 = bestR[2][2];
  const double tr = m11 + m22 + m33;
  double q0, q1, q2, q3;
  if (tr > fmax(m11, fmax(m22, m33))) {
    q0 = sqrt(1 + tr) / 2;
    q1 = (m32 - m23) / (4 * q0); q2 = (m13 - m31) / (4 * q0); q3 = (m21 - m12) / (4 * q0);
  } else if (m11 > fmax(tr, fmax(m22, m33))) {
    q1 = sqrt(m11 / 2 + (1 - tr) / 4);
    q0 = (m32 - m23) / (4 * q1); q2 = (m21 + m12) / (4 * q1); q3 = (m31 + m13) / (4 * q1);
  } else if (m22 > fmax(tr, fmax(m11, m33))) {
    q2 = sqrt(m22 / 2 + (1 - tr) / 4);
    q0 = (m13 - m31) / (4 * q2); q3 = (m32 + m23) / (4 * q2); q1 = (m12 + m21) / (4 * q2);
  } else {
    q3 = sqrt(m33 / 2 + (1 - tr) / 4);
    q0 = (m21 - m12) / (4 * q3); q1 = (m13 + m31) / (4 * q3); q2 = (m23 + m32) / (4 * q3);
  }
  const double qn = sqrt(q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3);
  quat[4 * b + 0] = (float)(q0 / qn);
  quat[4 * b + 1] = (float)(q1 / qn);
  quat[4 * b + 2] = (float)(q2 / qn);
  quat[4 * b + 3] = (float)(q3 / qn);
#pragma unroll
  for (int i = 0; i < 3; ++i) pos[3 * b + i] = (float)bestT[i];
  if (!(bestE < INFINITY) || isnan(qn)) status[b] |= 8;
}

hipError_t launch_epnp(const float* raw, int B, int n, const float* kp3d, const double* model, const double* K,
                       float nu, float nv, const EpnpDist& dist, int apply_sigmoid, float* kp_out, float* quat,
                       float* pos, int* status, hipStream_t s) {
  if (n < 4 || n > EPNP_MAXN) return hipErrorInvalidValue;
  epnp_kernel<<<B, 192, 0, s>>>(raw, B, n, kp3d, model, K[0], K[4], K[2], K[5], nu, nv, dist, apply_sigmoid, kp_out,
                                quat, pos, status);
  return hipGetLastError();
}

}  // namespace spef
