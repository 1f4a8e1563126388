"""Quaternion / rotation helpers (scalar-first, Hamilton, active) -- src/spe/utils.py conventions.

Used host-side for decode-table construction (orientation bins), synthetic poses and metrics; never on
the per-frame hot path.
"""
from __future__ import annotations

import numpy as np


def euler2quat(yaw: float, pitch: float, roll: float) -> np.ndarray:
    """src/spe/utils.py:167-232 (ZYX sequence, degrees), no gimbal warning, no north enforcement."""
    cy, sy = np.cos(np.deg2rad(yaw) / 2), np.sin(np.deg2rad(yaw) / 2)
    cp, sp = np.cos(np.deg2rad(pitch) / 2), np.sin(np.deg2rad(pitch) / 2)
    cr, sr = np.cos(np.deg2rad(roll) / 2), np.sin(np.deg2rad(roll) / 2)
    q = np.array([cy * cp * cr + sy * sp * sr,
                  cy * cp * sr - sy * sp * cr,
                  cy * sp * cr + sy * cp * sr,
                  sy * cp * cr - cy * sp * sr])
    return q / np.linalg.norm(q)


def quat2dcm(q) -> np.ndarray:
    """src/spe/utils.py:10-53."""
    q0, q1, q2, q3 = q
    return np.array([
        [2 * q0 ** 2 - 1 + 2 * q1 ** 2, 2 * q1 * q2 - 2 * q0 * q3, 2 * q1 * q3 + 2 * q0 * q2],
        [2 * q1 * q2 + 2 * q0 * q3, 2 * q0 ** 2 - 1 + 2 * q2 ** 2, 2 * q2 * q3 - 2 * q0 * q1],
        [2 * q1 * q3 - 2 * q0 * q2, 2 * q2 * q3 + 2 * q0 * q1, 2 * q0 ** 2 - 1 + 2 * q3 ** 2]], dtype=np.float64)


def random_orientations(n: int, rng: np.random.Generator) -> np.ndarray:
    """Uniform random unit quaternions (Shoemake), scalar-first, float32."""
    u1, u2, u3 = rng.random(n), rng.random(n), rng.random(n)
    q = np.stack([np.sqrt(u1) * np.cos(2 * np.pi * u3), np.sqrt(1 - u1) * np.sin(2 * np.pi * u2),
                  np.sqrt(1 - u1) * np.cos(2 * np.pi * u2), np.sqrt(u1) * np.sin(2 * np.pi * u3)], axis=1)
    return q.astype(np.float32)


def angle_deg(q1, q2) -> np.ndarray:
    """Sign-insensitive rotation angle (fp64 atan2 form) between two quaternion arrays."""
    q1 = np.asarray(q1, np.float64)
    q2 = np.asarray(q2, np.float64)
    q1 = q1 / np.linalg.norm(q1, axis=-1, keepdims=True)
    q2 = q2 / np.linalg.norm(q2, axis=-1, keepdims=True)
    s = np.where(np.sum(q1 * q2, axis=-1, keepdims=True) < 0, -1.0, 1.0)
    return np.rad2deg(2 * np.arctan2(np.linalg.norm(q1 - s * q2, axis=-1), np.linalg.norm(q1 + s * q2, axis=-1)))
