"""NumPy restatement of the reference pose decode (ORACLE -- test infrastructure only).

Every function cites the reference lines it follows. Arithmetic types follow the reference:
softmax in float32 (``pose[...]`` arrays are float32 NumPy, spe_utils.py:75-79), quaternion moment
sums / eig in float64 (classification_utils.py:131-142), outputs cast to float32 (:144-145).
"""
from __future__ import annotations

import numpy as np

# --------------------------------------------------------------------------- quaternion helpers


def euler2quat(yaw, pitch, roll):
    """src/spe/utils.py:167-232 (ZYX, scalar-first, Hamilton, active), gymbal_check off, no north."""
    cy, sy = np.cos(np.deg2rad(yaw) / 2), np.sin(np.deg2rad(yaw) / 2)
    cp, sp = np.cos(np.deg2rad(pitch) / 2), np.sin(np.deg2rad(pitch) / 2)
    cr, sr = np.cos(np.deg2rad(roll) / 2), np.sin(np.deg2rad(roll) / 2)
    q = np.array([cy * cp * cr + sy * sp * sr,
                  cy * cp * sr - sy * sp * cr,
                  cy * sp * cr + sy * cp * sr,
                  sy * cp * cr - cy * sp * sr])
    return q / np.linalg.norm(q)


def quat2dcm(q):
    """src/spe/utils.py:10-53."""
    q0, q1, q2, q3 = q
    d = np.zeros((3, 3))
    d[0, 0] = 2 * q0 ** 2 - 1 + 2 * q1 ** 2
    d[1, 1] = 2 * q0 ** 2 - 1 + 2 * q2 ** 2
    d[2, 2] = 2 * q0 ** 2 - 1 + 2 * q3 ** 2
    d[0, 1] = 2 * q1 * q2 - 2 * q0 * q3
    d[0, 2] = 2 * q1 * q3 + 2 * q0 * q2
    d[1, 0] = 2 * q1 * q2 + 2 * q0 * q3
    d[1, 2] = 2 * q2 * q3 - 2 * q0 * q1
    d[2, 0] = 2 * q1 * q3 - 2 * q0 * q2
    d[2, 1] = 2 * q2 * q3 + 2 * q0 * q1
    return d


def dcm2quat(dcm):
    """src/spe/utils.py:56-118 (Spurrier branch selection, then normalise)."""
    m11, m12, m13 = dcm[0]
    m21, m22, m23 = dcm[1]
    m31, m32, m33 = dcm[2]
    tr = m11 + m22 + m33
    if tr > max(m11, m22, m33):
        q0 = np.sqrt(1 + tr) / 2
        q1, q2, q3 = (m32 - m23) / (4 * q0), (m13 - m31) / (4 * q0), (m21 - m12) / (4 * q0)
    elif m11 > max(tr, m22, m33):
        q1 = np.sqrt(m11 / 2 + (1 - tr) / 4)
        q0, q2, q3 = (m32 - m23) / (4 * q1), (m21 + m12) / (4 * q1), (m31 + m13) / (4 * q1)
    elif m22 > max(tr, m11, m33):
        q2 = np.sqrt(m22 / 2 + (1 - tr) / 4)
        q0, q3, q1 = (m13 - m31) / (4 * q2), (m32 + m23) / (4 * q2), (m12 + m21) / (4 * q2)
    else:
        q3 = np.sqrt(m33 / 2 + (1 - tr) / 4)
        q0, q1, q2 = (m21 - m12) / (4 * q3), (m13 + m31) / (4 * q3), (m23 + m32) / (4 * q3)
    q = np.array([q0, q1, q2, q3])
    return q / np.linalg.norm(q)


# --------------------------------------------------------------------------- histograms


def orientation_histogram(n_bins_per_dim=12, delete_unused_bins=False):
    """OrientationSoftClassification.build_histogram, classification_utils.py:39-83.
    Returns (quats float64 [n,4], redundant_flags bool [n_bins_per_dim**3])."""
    lo, hi = np.array([-180, -90, -180]), np.array([180, 90, 180])
    b = np.linspace(0.0, 1.0, n_bins_per_dim)
    g = np.stack(np.meshgrid(b, b, b, indexing='ij'), axis=-1).reshape(-1, 3)
    e = g * (hi - lo) + lo
    q = np.stack([euler2quat(*e[i]) for i in range(e.shape[0])])
    boundary = np.logical_or(e[:, 0] == hi[0], e[:, 2] == hi[2])
    gimbal = np.logical_and(np.abs(e[:, 1]) == hi[1], e[:, 0] != lo[0])
    red = np.logical_or(boundary, gimbal)
    if delete_unused_bins:
        q = q[~red]
    return q, red


def position_histogram(n_bins_per_dim=10, lo=(-16, -12, -2), hi=(16, 12, 40)):
    """PositionSoftClassification.build_histogram, classification_utils.py:201-215;
    limits from SPEUtils.__init__, spe_utils.py:50-53."""
    lo, hi = np.array(lo), np.array(hi)
    b = np.linspace(0.0, 1.0, n_bins_per_dim)
    g = np.stack(np.meshgrid(b, b, b, indexing='ij'), axis=-1).reshape(-1, 3)
    return g * (hi - lo) + lo


def encode_orientation(q, hist, redundant, n_bins_per_dim=12, smooth=3, delete_unused_bins=False):
    """classification_utils.py:85-111."""
    var = (smooth / n_bins_per_dim) ** 2 / 12
    k = np.exp(-((2 * np.arccos(np.minimum(1.0, np.abs(np.sum(q * hist, axis=1)))) / np.pi) ** 2) / (2 * var))
    if not delete_unused_bins:
        k[redundant] = 0
    return (k / np.sum(k)).astype(np.float32)


def encode_position(p, grid, n_bins_per_dim=10, smooth=100):
    """classification_utils.py:217-240."""
    var = (smooth / n_bins_per_dim) ** 2 / 12
    k = np.exp(-np.sum((p - grid) ** 2, axis=1) / (2 * var))
    return (k / np.sum(k)).astype(np.float32)


# --------------------------------------------------------------------------- last_activ / decode


def softmax_f32(x):
    """SPEUtils.last_activ softmax, spe_utils.py:75-79 (float32 NumPy)."""
    x = np.asarray(x, dtype=np.float32)
    e = np.exp(x - np.max(x, axis=1, keepdims=True))
    return e / np.sum(e, axis=1, keepdims=True)


def sigmoid_f32(x):
    """spe_utils.py:68."""
    x = np.asarray(x, dtype=np.float32)
    return 1 / (1 + np.exp(-x))


def l2_normalise_f32(x):
    """spe_utils.py:72 (orientation regression)."""
    x = np.asarray(x, dtype=np.float32)
    return x / np.linalg.norm(x, ord=2, axis=1, keepdims=True)


def decode_orientation(p, hist):
    """OrientationSoftClassification.decode, classification_utils.py:113-146: a = sum_i p_i q_i q_i^T
    (float64), top eigenvector of a, normalised, cast float32. Raises ValueError on NaN (:134-135)."""
    b = hist[:, :, None] * hist[:, None, :]
    a = np.sum(b * np.reshape(p, (-1, 1, 1)), axis=0)
    if np.any(np.isnan(a)):
        raise ValueError('Error during orientation decoding')
    s, v = np.linalg.eig(a)
    q = v[:, np.argsort(s)[-1]]
    q = q / np.linalg.norm(q)
    return np.real(q).astype(np.float32)


def decode_orientation_batch(p, hist):
    """classification_utils.py:148-166 (per-image loop)."""
    return np.stack([decode_orientation(p[i], hist) for i in range(p.shape[0])]).astype(np.float32)


def decode_position_batch(p, grid):
    """PositionSoftClassification.decode/decode_batch, classification_utils.py:242-285."""
    out = np.zeros((p.shape[0], 3), np.float32)
    for i in range(p.shape[0]):
        if np.sum(p[i]) == 0:
            raise ValueError('Encoded position vector sum is zero, cannot decode.')
        pa = np.sum(grid * np.reshape(p[i], (-1, 1)), axis=0) / np.sum(p[i])
        if np.any(np.isnan(pa)):
            raise ValueError('Error during position decoding, NaN found in decoded position.')
        out[i] = pa.astype(np.float32)
    return out


# --------------------------------------------------------------------------- keypoints


SPEED_K = np.array([[0.0176 / 5.86e-6, 0, 960.0], [0, 0.0176 / 5.86e-6, 600.0], [0, 0, 1]])
SPEED_NU, SPEED_NV = 1920, 1200          # src/data/datasets/speed.py:18-32


def project_keypoints(q, t, kp3d, K=SPEED_K, dist=None):
    """KeyPoints.project, keypoints_utils.py:47-92: origin + N keypoints -> 2 x (N+1) px; with ``dist`` =
    (k1, k2, p1, p2, k3) the radial + tangential distortion of :74-80 (the SPEED+ camera, speed_plus.py:18-40)."""
    pts = np.concatenate((np.zeros((3, 1)), np.asarray(kp3d, np.float32).T.astype(np.float64)), axis=1)
    pts = np.vstack((pts, np.ones((1, pts.shape[1]))))
    xyz = np.hstack((quat2dcm(q), np.expand_dims(t, 1))) @ pts
    x0, y0 = xyz[0] / xyz[2], xyz[1] / xyz[2]
    if dist is not None:
        d = dist
        r2 = x0 * x0 + y0 * y0
        cdist = 1 + d[0] * r2 + d[1] * r2 * r2 + d[4] * r2 * r2 * r2
        x = x0 * cdist + d[2] * 2 * x0 * y0 + d[3] * (r2 + 2 * x0 * x0)
        y = y0 * cdist + d[2] * (r2 + 2 * y0 * y0) + d[3] * 2 * x0 * y0
    else:
        x, y = x0, y0
    return np.vstack((K[0, 0] * x + K[0, 2], K[1, 1] * y + K[1, 2]))


def create_keypoints2d(q, t, kp3d, K=SPEED_K, nu=SPEED_NU, nv=SPEED_NV, dist=None):
    """KeyPoints.create_keypoints2d, keypoints_utils.py:94-110 -> 2(N+1) float32, normalised (x,y)."""
    k2 = project_keypoints(q, t, kp3d, K, dist)
    k2[0] /= nu
    k2[1] /= nv
    return np.reshape(k2.T, (-1,)).astype(np.float32)


def create_bbox_from_keypoints(kp2d, nu=SPEED_NU, nv=SPEED_NV):
    """KeyPoints.create_bbox_from_keypoints, keypoints_utils.py:176-198 -> [x_min, y_min, x_max, y_max]."""
    x = kp2d[::2] * nu
    y = kp2d[1::2] * nv
    return np.array([np.min(x) / nu, np.min(y) / nv, np.max(x) / nu, np.max(y) / nv])


# --------------------------------------------------------------------------- metrics


def get_score(true_ori, true_pos, pred_ori, pred_pos):
    """SPEUtils.get_score, spe_utils.py:103-159 (ESA score)."""
    pos_err = np.linalg.norm(true_pos - pred_pos, axis=1)
    norm_pos = pos_err / np.linalg.norm(true_pos, axis=1)
    s = np.abs(np.sum(pred_ori * true_ori, axis=1, keepdims=True))
    if np.any(s > 1.01):
        raise ValueError('Intermediate sum issue due to error in model prediction (orientation)')
    s[s > 1] = 1
    ori = np.mean(2 * np.arccos(s))
    return {'esa_score': ori + np.mean(norm_pos), 'ori_score': ori, 'pos_score': np.mean(norm_pos),
            'ori_error': ori * 180 / np.pi, 'pos_error': np.mean(pos_err)}


def angle_deg_stable(q1, q2):
    """Sign-insensitive rotation angle in float64: 2*atan2(|q1 - s q2|, |q1 + s q2|), s = sign(q1.q2).
    Used for parity (the reference's 2*acos on float32 resolves only ~0.04 deg)."""
    q1 = np.asarray(q1, np.float64)
    q2 = np.asarray(q2, np.float64)
    q1 = q1 / np.linalg.norm(q1, axis=-1, keepdims=True)
    q2 = q2 / np.linalg.norm(q2, axis=-1, keepdims=True)
    s = np.sign(np.sum(q1 * q2, axis=-1, keepdims=True))
    s[s == 0] = 1
    return np.rad2deg(2 * np.arctan2(np.linalg.norm(q1 - s * q2, axis=-1), np.linalg.norm(q1 + s * q2, axis=-1)))
