"""EPnP restatement in float64 NumPy (ORACLE -- test infrastructure only).

The reference decodes keypoint-mode poses with ``cv2.solvePnP(..., flags=cv2.SOLVEPNP_EPNP)`` followed by
``cv2.Rodrigues`` and ``dcm2quat`` (src/spe/keypoints_utils.py:112-150, loop :169-172). OpenCV is not installed
here and no reference test pins its output, so this module restates the published EPnP algorithm as OpenCV
4.5.5 implements it (modules/calib3d/src/epnp.cpp; pinned version from setup/finn/Dockerfile:142
``opencv-python==4.5.5.64``):

  choose_control_points   centroid + PCA of the 3-D points (SVD of PW0^T PW0), c_i = c0 + sqrt(s_i / n) v_i
  barycentric coords      alphas from the inverse of [c1-c0 | c2-c0 | c3-c0]
  fill_M                  2n x 12: [a_i fu, 0, a_i (uc - u)], [0, a_i fv, a_i (vc - v)]
  eigenvectors            of M^T M (SVD), the 4 of smallest eigenvalue (ut rows 11, 10, 9, 8)
  L_6x10, rho             pairwise control-point distance constraints
  betas approx 1/2/3      least squares on column subsets of L (cvSolve SVD)
  gauss_newton            5 iterations, Householder QR (qr_solve)
  compute_R_and_t         ccs, pcs, solve_for_sign (pcs[2] < 0 -> flip), Procrustes by SVD of sum (pc-pc0)(pw-pw0)^T,
                          det < 0 -> negate R's third row, t = pc0 - R pw0; reprojection error (mean pixel distance)
  pick                    N = argmin of rep_errors[1..3] with ties keeping the lower index

  undistort_points        solvePnP's cv::undistortPoints (5 fixed-point iterations) + epnp::init_points re-projection

Parity status: UNPINNED against OpenCV itself (absent); pinned by the noise-free known-answer tests on the
reference's own projections (tests/golden/keypoints.npz: 1,800 valid.json poses, SPEED camera;
tests/golden/keypoints_speedplus.npz: the same poses through the SPEED+ camera's lens distortion) -- see tests.
"""
from __future__ import annotations

import numpy as np

from .decode_ref import SPEED_K, SPEED_NU, SPEED_NV, dcm2quat


def _control_points(pw):
    n = pw.shape[0]
    c0 = pw.mean(axis=0)
    p0 = pw - c0
    u, s, vt = np.linalg.svd(p0.T @ p0)          # cvSVD(PW0tPW0): descending singular values, rows of U^T
    cws = np.zeros((4, 3))
    cws[0] = c0
    for i in range(1, 4):
        axis = u[:, i - 1]
        # The axis sign is arbitrary (LAPACK / cvSVD / Jacobi differ) and, with noisy keypoints, changes the EPnP
        # estimate at the noise level; fix it canonically (largest-|component| positive), as the HIP path does.
        axis = axis * (1.0 if axis[np.argmax(np.abs(axis))] >= 0 else -1.0)
        cws[i] = c0 + np.sqrt(s[i - 1] / n) * axis
    return cws


def _alphas(pw, cws):
    cc = (cws[1:] - cws[0]).T                     # cc[i][j-1] = cws[j][i] - cws[0][i]
    ci = np.linalg.inv(cc)
    a = (ci @ (pw - cws[0]).T).T                  # a[1..3]
    return np.concatenate([1.0 - a.sum(axis=1, keepdims=True), a], axis=1)


def _fill_m(alphas, us, fu, fv, uc, vc):
    n = alphas.shape[0]
    m = np.zeros((2 * n, 12))
    for i in range(n):
        u, v = us[i]
        for j in range(4):
            m[2 * i, 3 * j] = alphas[i, j] * fu
            m[2 * i, 3 * j + 2] = alphas[i, j] * (uc - u)
            m[2 * i + 1, 3 * j + 1] = alphas[i, j] * fv
            m[2 * i + 1, 3 * j + 2] = alphas[i, j] * (vc - v)
    return m


def _l6x10(ut):
    v = [ut[11], ut[10], ut[9], ut[8]]
    pairs = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]
    dv = np.array([[v[i][3 * a:3 * a + 3] - v[i][3 * b:3 * b + 3] for (a, b) in pairs] for i in range(4)])
    l = np.zeros((6, 10))
    for i in range(6):
        d = dv[:, i]
        l[i] = [d[0] @ d[0], 2 * d[0] @ d[1], d[1] @ d[1], 2 * d[0] @ d[2], 2 * d[1] @ d[2], d[2] @ d[2],
                2 * d[0] @ d[3], 2 * d[1] @ d[3], 2 * d[2] @ d[3], d[3] @ d[3]]
    return l


def _rho(cws):
    pairs = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]
    return np.array([np.sum((cws[a] - cws[b]) ** 2) for a, b in pairs])


def _lstsq(a, b):
    return np.linalg.lstsq(a, b, rcond=None)[0]


def _betas1(l, rho):
    b4 = _lstsq(l[:, [0, 1, 3, 6]], rho)
    if b4[0] < 0:
        b0 = np.sqrt(-b4[0])
        return np.array([b0, -b4[1] / b0, -b4[2] / b0, -b4[3] / b0])
    b0 = np.sqrt(b4[0])
    return np.array([b0, b4[1] / b0, b4[2] / b0, b4[3] / b0])


def _betas2(l, rho):
    b3 = _lstsq(l[:, [0, 1, 2]], rho)
    if b3[0] < 0:
        b0, b1 = np.sqrt(-b3[0]), (np.sqrt(-b3[2]) if b3[2] < 0 else 0.0)
    else:
        b0, b1 = np.sqrt(b3[0]), (np.sqrt(b3[2]) if b3[2] > 0 else 0.0)
    if b3[1] < 0:
        b0 = -b0
    return np.array([b0, b1, 0.0, 0.0])


def _betas3(l, rho):
    b5 = _lstsq(l[:, [0, 1, 2, 3, 4]], rho)
    if b5[0] < 0:
        b0, b1 = np.sqrt(-b5[0]), (np.sqrt(-b5[2]) if b5[2] < 0 else 0.0)
    else:
        b0, b1 = np.sqrt(b5[0]), (np.sqrt(b5[2]) if b5[2] > 0 else 0.0)
    if b5[1] < 0:
        b0 = -b0
    return np.array([b0, b1, b5[3] / b0, 0.0])


def _gauss_newton(l, rho, betas, iters=5):
    betas = betas.copy()
    for _ in range(iters):
        b = betas
        a = np.stack([
            2 * l[:, 0] * b[0] + l[:, 1] * b[1] + l[:, 3] * b[2] + l[:, 6] * b[3],
            l[:, 1] * b[0] + 2 * l[:, 2] * b[1] + l[:, 4] * b[2] + l[:, 7] * b[3],
            l[:, 3] * b[0] + l[:, 4] * b[1] + 2 * l[:, 5] * b[2] + l[:, 8] * b[3],
            l[:, 6] * b[0] + l[:, 7] * b[1] + l[:, 8] * b[2] + 2 * l[:, 9] * b[3]], axis=1)
        bb = np.array([b[0] * b[0], b[0] * b[1], b[1] * b[1], b[0] * b[2], b[1] * b[2], b[2] * b[2],
                       b[0] * b[3], b[1] * b[3], b[2] * b[3], b[3] * b[3]])
        r = rho - l @ bb
        q, rr = np.linalg.qr(a)                       # qr_solve: Householder least squares
        betas = betas + np.linalg.solve(rr, q.T @ r)
    return betas


def _r_and_t(ut, betas, alphas, pw, us, fu, fv, uc, vc):
    ccs = np.zeros((4, 3))
    for i in range(4):
        ccs += betas[i] * ut[11 - i].reshape(4, 3)
    pcs = alphas @ ccs
    if pcs[0, 2] < 0:                                 # solve_for_sign
        ccs, pcs = -ccs, -pcs
    pc0, pw0 = pcs.mean(axis=0), pw.mean(axis=0)
    abt = (pcs - pc0).T @ (pw - pw0)
    u, s, vt = np.linalg.svd(abt)
    r = u @ vt
    if np.linalg.det(r) < 0:
        r[2] = -r[2]
    t = pc0 - r @ pw0
    xc = pw @ r.T + t
    ue = uc + fu * xc[:, 0] / xc[:, 2]
    ve = vc + fv * xc[:, 1] / xc[:, 2]
    err = np.mean(np.sqrt((us[:, 0] - ue) ** 2 + (us[:, 1] - ve) ** 2))
    return r, t, err


def control_points_and_alphas(pw):
    """Model-only part of EPnP (choose_control_points + compute_barycentric_coordinates)."""
    pw = np.asarray(pw, np.float64)
    cws = _control_points(pw)
    return cws, _alphas(pw, cws)


def epnp(pw, us, k=SPEED_K):
    """-> (R 3x3, t 3): pose of the 3-D points pw (n x 3) seen at pixels us (n x 2)."""
    pw = np.asarray(pw, np.float64)
    us = np.asarray(us, np.float64)
    fu, fv, uc, vc = k[0, 0], k[1, 1], k[0, 2], k[1, 2]
    cws = _control_points(pw)
    alphas = _alphas(pw, cws)
    m = _fill_m(alphas, us, fu, fv, uc, vc)
    _, _, ut = np.linalg.svd(m.T @ m)                 # rows sorted by descending singular value
    l, rho = _l6x10(ut), _rho(cws)
    best = None
    for fn in (_betas1, _betas2, _betas3):
        b = _gauss_newton(l, rho, fn(l, rho))
        r, t, err = _r_and_t(ut, b, alphas, pw, us, fu, fv, uc, vc)
        if best is None or err < best[2]:
            best = (r, t, err)
    return best[0], best[1]


def undistort_points(us32, k, dist=None, iters=5):
    """cv::undistortPoints(src, dst, K, D) as solvePnP(SOLVEPNP_EPNP) calls it before EPnP (OpenCV 4.5.5
    calib3d/src/solvepnp.cpp, undistort.dispatch.cpp cvUndistortPointsInternal; default criteria COUNT = 5):
    x = (u - cx) / fx (as a product with 1/fx), then x <- (x0 - delta(x)) * icdist(x) five times (k4..k6 and the thin
    prism / tilt terms are 0 for a 5-coefficient model; icdist < 0 falls back to the distorted point), output
    rounded to the input's float32; epnp::init_points then re-projects with K (us = x * fu + uc, in double).
    With ``dist`` None or all zeros only the float32 round trip of the normalised coordinate remains (the reference
    passes zeros for SPEED, keypoints_utils.py:136)."""
    fu, fv, uc, vc = k[0, 0], k[1, 1], k[0, 2], k[1, 2]
    ifx, ify = 1.0 / fu, 1.0 / fv
    d = np.zeros(5) if dist is None else np.asarray(dist, np.float64).reshape(-1)
    k1, k2, p1, p2, k3 = d[:5]
    out = np.zeros((us32.shape[0], 2))
    for i in range(us32.shape[0]):
        u, v = float(us32[i, 0]), float(us32[i, 1])
        x = x0 = (u - uc) * ifx
        y = y0 = (v - vc) * ify
        for _ in range(iters):
            r2 = x * x + y * y
            icdist = 1.0 / (1 + ((k3 * r2 + k2) * r2 + k1) * r2)
            if icdist < 0:
                x, y = (u - uc) * ifx, (v - vc) * ify
                break
            dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
            dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
            x = (x0 - dx) * icdist
            y = (y0 - dy) * icdist
        out[i, 0] = float(np.float32(x)) * fu + uc
        out[i, 1] = float(np.float32(y)) * fv + vc
    return out


def pnp(kp2d_norm, kp3d, k=SPEED_K, nu=SPEED_NU, nv=SPEED_NV, dist=None):
    """KeyPoints.pnp (keypoints_utils.py:112-150): normalised (x0,y0,x1,y1,...) incl. origin -> (q f32, t f32)."""
    x = kp2d_norm[0::2] * nu
    y = kp2d_norm[1::2] * nv
    us32 = np.stack([x, y], axis=1)[1:].astype(np.float32)         # float32 pixels (keypoints_utils.py:127-131)
    us = undistort_points(us32, k, dist)
    r, t = epnp(np.asarray(kp3d, np.float32).astype(np.float64), us, k)
    return dcm2quat(r).astype(np.float32), np.asarray(t, np.float32)


def decode_batch(kp2d_norm, kp3d, k=SPEED_K, nu=SPEED_NU, nv=SPEED_NV, dist=None):
    """KeyPoints.decode_batch (keypoints_utils.py:152-174)."""
    q = np.zeros((kp2d_norm.shape[0], 4), np.float32)
    t = np.zeros((kp2d_norm.shape[0], 3), np.float32)
    for i in range(kp2d_norm.shape[0]):
        q[i], t[i] = pnp(kp2d_norm[i], kp3d, k, nu, nv, dist)
    return q, t
