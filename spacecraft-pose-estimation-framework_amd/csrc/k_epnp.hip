// Batched keypoint decode: SPEUtils.last_activ sigmoid (src/spe/spe_utils.py:68) + KeyPoints.pnp
// (src/spe/keypoints_utils.py:112-150) = cv2.solvePnP(SOLVEPNP_EPNP) -> Rodrigues -> dcm2quat (spe/utils.py:56-118),
// including solvePnP's undistortPoints for cameras with lens distortion (SPEED+, data/datasets/speed_plus.py:18-40).
//
// One fp64 thread per problem; the algorithm is OpenCV 4.5.5 epnp.cpp's (the reference's pinned OpenCV):
// PCA control points, barycentric alphas, M (2n x 12), the 4 eigenvectors of M^T M with the smallest
// eigenvalues, L_6x10 / rho, beta approximations 1/2/3 (least squares), 5 Gauss-Newton steps (Householder
// QR), R|t by Procrustes with OpenCV's sign fixes, lowest mean reprojection error wins. Symmetric
// eigenproblems use cyclic Jacobi (fp64) instead of LAPACK/cvSVD -- same subspaces, independent of the
// eigenvector signs. Rodrigues(rvec(R)) == R, so R goes straight to the Spurrier quaternion.
#include <math.h>

#include "spef_common.hpp"
#include "spef_kernels.hpp"

namespace spef {

#define EPNP_MAXN 16

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
        const double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
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
  double a1[NC], a2[NC];
  for (int k = 0; k < NC; ++k) {
    double eta = 0.0;
    for (int i = k; i < 6; ++i) eta = fmax(eta, fabs(A[i][k]));
    if (eta == 0.0) {
      for (int j = 0; j < NC; ++j) x[j] = 0.0;
      return;
    }
    const double inv = 1.0 / eta;
    double sum2 = 0.0;
    for (int i = k; i < 6; ++i) {
      A[i][k] *= inv;
      sum2 += A[i][k] * A[i][k];
    }
    double sigma = sqrt(sum2);
    if (A[k][k] < 0) sigma = -sigma;
    A[k][k] += sigma;
    a1[k] = sigma * A[k][k];
    a2[k] = -eta * sigma;
    for (int j = k + 1; j < NC; ++j) {
      double sum = 0.0;
      for (int i = k; i < 6; ++i) sum += A[i][k] * A[i][j];
      const double tau = sum / a1[k];
      for (int i = k; i < 6; ++i) A[i][j] -= tau * A[i][k];
    }
  }
  for (int j = 0; j < NC; ++j) {
    double tau = 0.0;
    for (int i = j; i < 6; ++i) tau += A[i][j] * b[i];
    tau /= a1[j];
    for (int i = j; i < 6; ++i) b[i] -= tau * A[i][j];
  }
  x[NC - 1] = b[NC - 1] / a2[NC - 1];
  for (int i = NC - 2; i >= 0; --i) {
    double sum = 0.0;
    for (int j = i + 1; j < NC; ++j) sum += A[i][j] * x[j];
    x[i] = (b[i] - sum) / a2[i];
  }
}

struct EpnpProblem {
  int n;
  double pw[EPNP_MAXN][3], us[EPNP_MAXN][2], al[EPNP_MAXN][4];
  double cws[4][3];
  double fu, fv, uc, vc;
};

__device__ void epnp_gn(const double (&L)[6][10], const double (&rho)[6], double (&b)[4]) {
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

// R|t from betas (epnp.cpp compute_R_and_t); returns the mean reprojection error
__device__ double epnp_rt(const EpnpProblem& P, const double (&ut4)[4][12], const double (&be)[4], double (&R)[3][3],
                          double (&t)[3]) {
  double ccs[4][3] = {};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 3; ++k) ccs[j][k] += be[i] * ut4[i][3 * j + k];
  double pcs[EPNP_MAXN][3];
  for (int i = 0; i < P.n; ++i)
    for (int j = 0; j < 3; ++j)
      pcs[i][j] = P.al[i][0] * ccs[0][j] + P.al[i][1] * ccs[1][j] + P.al[i][2] * ccs[2][j] + P.al[i][3] * ccs[3][j];
  if (pcs[0][2] < 0.0)   // solve_for_sign
    for (int i = 0; i < P.n; ++i)
      for (int j = 0; j < 3; ++j) pcs[i][j] = -pcs[i][j];
  double pc0[3] = {}, pw0[3] = {};
  for (int i = 0; i < P.n; ++i)
    for (int j = 0; j < 3; ++j) {
      pc0[j] += pcs[i][j];
      pw0[j] += P.pw[i][j];
    }
  for (int j = 0; j < 3; ++j) {
    pc0[j] /= P.n;
    pw0[j] /= P.n;
  }
  double abt[3][3] = {};
  for (int i = 0; i < P.n; ++i)
    for (int j = 0; j < 3; ++j)
      for (int k = 0; k < 3; ++k) abt[j][k] += (pcs[i][j] - pc0[j]) * (P.pw[i][k] - pw0[k]);
  // R = U V^T of abt = U S V^T: V from eig(abt^T abt), U = abt V S^-1
  double ata[3][3], V[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) ata[i][j] = abt[0][i] * abt[0][j] + abt[1][i] * abt[1][j] + abt[2][i] * abt[2][j];
  jacobi_sym<3>(ata, V);
  double U[3][3];
  for (int c = 0; c < 3; ++c) {
    double col[3], nrm = 0.0;
    for (int r = 0; r < 3; ++r) {
      col[r] = abt[r][0] * V[0][c] + abt[r][1] * V[1][c] + abt[r][2] * V[2][c];
      nrm += col[r] * col[r];
    }
    nrm = sqrt(nrm);
    for (int r = 0; r < 3; ++r) U[r][c] = nrm > 0 ? col[r] / nrm : 0.0;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[i][j] = U[i][0] * V[j][0] + U[i][1] * V[j][1] + U[i][2] * V[j][2];
  const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] + R[0][2] * R[1][0] * R[2][1] -
                     R[0][2] * R[1][1] * R[2][0] - R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
  if (det < 0)
    for (int j = 0; j < 3; ++j) R[2][j] = -R[2][j];
  for (int i = 0; i < 3; ++i) t[i] = pc0[i] - (R[i][0] * pw0[0] + R[i][1] * pw0[1] + R[i][2] * pw0[2]);
  double err = 0.0;
  for (int i = 0; i < P.n; ++i) {
    const double* p = P.pw[i];
    const double xc = R[0][0] * p[0] + R[0][1] * p[1] + R[0][2] * p[2] + t[0];
    const double yc = R[1][0] * p[0] + R[1][1] * p[1] + R[1][2] * p[2] + t[1];
    const double iz = 1.0 / (R[2][0] * p[0] + R[2][1] * p[1] + R[2][2] * p[2] + t[2]);
    const double ue = P.uc + P.fu * xc * iz, ve = P.vc + P.fv * yc * iz;
    err += sqrt((P.us[i][0] - ue) * (P.us[i][0] - ue) + (P.us[i][1] - ve) * (P.us[i][1] - ve));
  }
  return err / P.n;
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

__global__ __launch_bounds__(64) void epnp_kernel(const float* __restrict__ raw, int B, int n,
                                                  const float* __restrict__ kp3d, const double* __restrict__ model,
                                                  double fu, double fv, double uc,
                                                  double vc, float nu, float nv, EpnpDist dist, int apply_sigmoid,
                                                  float* __restrict__ kp_out, float* __restrict__ quat,
                                                  float* __restrict__ pos, int* __restrict__ status) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= B) return;
  const int nk = 2 * (n + 1);
  EpnpProblem P;
  P.n = n;
  P.fu = fu; P.fv = fv; P.uc = uc; P.vc = vc;
  for (int i = 0; i <= n; ++i) {
    float x = raw[(size_t)b * nk + 2 * i], y = raw[(size_t)b * nk + 2 * i + 1];
    if (apply_sigmoid) {   // spe_utils.py:68, float32
      x = 1.0f / (1.0f + expf(-x));
      y = 1.0f / (1.0f + expf(-y));
    }
    if (kp_out) {
      kp_out[(size_t)b * nk + 2 * i] = x;
      kp_out[(size_t)b * nk + 2 * i + 1] = y;
    }
    if (i > 0)   // keypoints_utils.py:127-131: pixels (float32 products), origin dropped; then undistortPoints
      undistort_point(dist, fu, fv, uc, vc, x * nu, y * nv, P.us[i - 1][0], P.us[i - 1][1]);
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 3; ++j) P.pw[i][j] = (double)kp3d[3 * i + j];

  // control points and barycentric coordinates: model-only, precomputed on the host (spef_set_keypoints)
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 3; ++j) P.cws[i][j] = model[3 * i + j];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 4; ++j) P.al[i][j] = model[12 + 4 * i + j];
  // M^T M accumulated row pair by row pair (M is never stored)
  double mtm[12][12] = {};
  for (int i = 0; i < n; ++i) {
    double r1[12], r2[12];
    for (int j = 0; j < 4; ++j) {
      r1[3 * j] = P.al[i][j] * fu;
      r1[3 * j + 1] = 0.0;
      r1[3 * j + 2] = P.al[i][j] * (uc - P.us[i][0]);
      r2[3 * j] = 0.0;
      r2[3 * j + 1] = P.al[i][j] * fv;
      r2[3 * j + 2] = P.al[i][j] * (vc - P.us[i][1]);
    }
    for (int p = 0; p < 12; ++p)
      for (int q = p; q < 12; ++q) mtm[p][q] += r1[p] * r1[q] + r2[p] * r2[q];
  }
  for (int p = 0; p < 12; ++p)
    for (int q = 0; q < p; ++q) mtm[p][q] = mtm[q][p];
  double ev[12][12];
  jacobi_sym<12>(mtm, ev);
  // the 4 eigenvectors of smallest eigenvalue, ascending: ut4[0] = ut row 11 (smallest), ..., ut4[3] = row 8
  int idx[12];
  for (int i = 0; i < 12; ++i) idx[i] = i;
  for (int i = 0; i < 4; ++i)
    for (int j = i + 1; j < 12; ++j)
      if (mtm[idx[j]][idx[j]] < mtm[idx[i]][idx[i]]) {
        const int tmp = idx[i];
        idx[i] = idx[j];
        idx[j] = tmp;
      }
  double ut4[4][12];
  for (int i = 0; i < 4; ++i)
    for (int k = 0; k < 12; ++k) ut4[i][k] = ev[k][idx[i]];
  // L_6x10 and rho
  const int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
  double L[6][10], rho[6];
  for (int r = 0; r < 6; ++r) {
    double dv[4][3];
    for (int i = 0; i < 4; ++i)
      for (int k = 0; k < 3; ++k) dv[i][k] = ut4[i][3 * pa[r] + k] - ut4[i][3 * pb[r] + k];
    auto dot = [&](int i, int j) { return dv[i][0] * dv[j][0] + dv[i][1] * dv[j][1] + dv[i][2] * dv[j][2]; };
    L[r][0] = dot(0, 0);
    L[r][1] = 2 * dot(0, 1);
    L[r][2] = dot(1, 1);
    L[r][3] = 2 * dot(0, 2);
    L[r][4] = 2 * dot(1, 2);
    L[r][5] = dot(2, 2);
    L[r][6] = 2 * dot(0, 3);
    L[r][7] = 2 * dot(1, 3);
    L[r][8] = 2 * dot(2, 3);
    L[r][9] = dot(3, 3);
    double d2 = 0.0;
    for (int k = 0; k < 3; ++k) d2 += (P.cws[pa[r]][k] - P.cws[pb[r]][k]) * (P.cws[pa[r]][k] - P.cws[pb[r]][k]);
    rho[r] = d2;
  }
  double bestR[3][3], bestT[3], bestE = INFINITY;
  for (int ap = 1; ap <= 3; ++ap) {
    double be[4] = {0, 0, 0, 0};
    double rr[6];
    for (int i = 0; i < 6; ++i) rr[i] = rho[i];
    if (ap == 1) {
      double A[6][4], x[4];
      for (int i = 0; i < 6; ++i) {
        A[i][0] = L[i][0]; A[i][1] = L[i][1]; A[i][2] = L[i][3]; A[i][3] = L[i][6];
      }
      qr_lstsq<4>(A, rr, x);
      const double s = x[0] < 0 ? -1.0 : 1.0;
      be[0] = sqrt(fabs(x[0]));
      be[1] = s * x[1] / be[0];
      be[2] = s * x[2] / be[0];
      be[3] = s * x[3] / be[0];
    } else if (ap == 2) {
      double A[6][3], x[3];
      for (int i = 0; i < 6; ++i) {
        A[i][0] = L[i][0]; A[i][1] = L[i][1]; A[i][2] = L[i][2];
      }
      qr_lstsq<3>(A, rr, x);
      if (x[0] < 0) {
        be[0] = sqrt(-x[0]);
        be[1] = x[2] < 0 ? sqrt(-x[2]) : 0.0;
      } else {
        be[0] = sqrt(x[0]);
        be[1] = x[2] > 0 ? sqrt(x[2]) : 0.0;
      }
      if (x[1] < 0) be[0] = -be[0];
    } else {
      double A[6][5], x[5];
      for (int i = 0; i < 6; ++i)
        for (int k = 0; k < 5; ++k) A[i][k] = L[i][k];
      qr_lstsq<5>(A, rr, x);
      if (x[0] < 0) {
        be[0] = sqrt(-x[0]);
        be[1] = x[2] < 0 ? sqrt(-x[2]) : 0.0;
      } else {
        be[0] = sqrt(x[0]);
        be[1] = x[2] > 0 ? sqrt(x[2]) : 0.0;
      }
      if (x[1] < 0) be[0] = -be[0];
      be[2] = x[3] / be[0];
    }
    epnp_gn(L, rho, be);
    double R[3][3], t[3];
    const double e = epnp_rt(P, ut4, be, R, t);
    if (e < bestE) {   // strict: ties keep the lower approximation index (epnp.cpp compute_pose)
      bestE = e;
      for (int i = 0; i < 3; ++i) {
        bestT[i] = t[i];
        for (int j = 0; j < 3; ++j) bestR[i][j] = R[i][j];
      }
    }
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
  for (int i = 0; i < 3; ++i) pos[3 * b + i] = (float)bestT[i];
  if (!(bestE < INFINITY) || isnan(qn)) status[b] |= 8;
}

hipError_t launch_epnp(const float* raw, int B, int n, const float* kp3d, const double* model, const double* K,
                       float nu, float nv, const EpnpDist& dist, int apply_sigmoid, float* kp_out, float* quat,
                       float* pos, int* status, hipStream_t s) {
  if (n < 4 || n > EPNP_MAXN) return hipErrorInvalidValue;
  epnp_kernel<<<(B + 63) / 64, 64, 0, s>>>(raw, B, n, kp3d, model, K[0], K[4], K[2], K[5], nu, nv, dist,
                                           apply_sigmoid, kp_out, quat, pos, status);
  return hipGetLastError();
}

}  // namespace spef
