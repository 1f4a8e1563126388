"""Host-side mirror of the reference ``SPEUtils`` surface the MI355X target needs.

Reference: ``src/spe/spe_utils.py:10-159`` (``SPEUtils``), ``src/spe/classification_utils.py:10-83,179-215``
(histogram construction). The MI355X target reads the same attributes the reference targets read --
``ori_mode``, ``pos_mode``, ``orientation.histogram`` / ``n_bins``, ``position.histogram`` / ``n_bins``,
``keypoints`` -- so a reference ``SPEUtils`` instance can be passed to ``SPEMi355x`` unchanged; this class
provides the same attributes for standalone use (bench, deploy) without importing the reference.

The decode itself (``last_activ`` + ``decode``) runs on the GPU (csrc/k_head.hip); there is deliberately no
CPU decode here. ``get_score`` is the evaluation metric (not on the hot path).
"""
from __future__ import annotations

import numpy as np

from .. import quaternion as Q


class OrientationHistogram:
    """Bins of ``OrientationSoftClassification`` (classification_utils.py:20-83)."""

    def __init__(self, n_bins_per_dim: int = 12, smooth_factor: int = 3, delete_unused_bins: bool = False):
        self.n_bins_per_dim = n_bins_per_dim
        self.smooth_factor = smooth_factor
        self.delete_unused_bins = delete_unused_bins
        lo, hi = np.array([-180, -90, -180]), np.array([180, 90, 180])
        b = np.linspace(0.0, 1.0, n_bins_per_dim)
        g = np.stack(np.meshgrid(b, b, b, indexing='ij'), axis=-1).reshape(-1, 3)
        e = g * (hi - lo) + lo
        q = np.stack([Q.euler2quat(*e[i]) for i in range(e.shape[0])])
        boundary = np.logical_or(e[:, 0] == hi[0], e[:, 2] == hi[2])
        gimbal = np.logical_and(np.abs(e[:, 1]) == hi[1], e[:, 0] != lo[0])
        self.redundant_flags = np.logical_or(boundary, gimbal)
        self.histogram = q[~self.redundant_flags] if delete_unused_bins else q
        self.n_bins = self.histogram.shape[0]

    def encode(self, ori: np.ndarray) -> np.ndarray:
        """Soft-classification target (classification_utils.py:85-111); used to plant logits in tests/bench."""
        var = (self.smooth_factor / self.n_bins_per_dim) ** 2 / 12
        k = np.exp(-((2 * np.arccos(np.minimum(1.0, np.abs(np.sum(ori * self.histogram, axis=1))))
                      / np.pi) ** 2) / (2 * var))
        if not self.delete_unused_bins:
            k[self.redundant_flags] = 0
        return (k / np.sum(k)).astype(np.float32)


class PositionHistogram:
    """Bins of ``PositionSoftClassification`` (classification_utils.py:184-215)."""

    def __init__(self, n_bins_per_dim: int = 10, smooth_factor: int = 100,
                 min_lim=(-16, -12, -2), max_lim=(16, 12, 40)):
        self.n_bins_per_dim = n_bins_per_dim
        self.smooth_factor = smooth_factor
        lo, hi = np.array(min_lim), np.array(max_lim)
        b = np.linspace(0.0, 1.0, n_bins_per_dim)
        g = np.stack(np.meshgrid(b, b, b, indexing='ij'), axis=-1).reshape(-1, 3)
        self.histogram = g * (hi - lo) + lo
        self.n_bins = self.histogram.shape[0]


class SPEUtils:
    """Same constructor signature as the reference (spe_utils.py:15-54)."""

    def __init__(self, camera=None, ori_mode: str = 'regression', n_ori_bins_per_dim: int = 12,
                 ori_smooth_factor: int = 3, ori_delete_unused_bins: bool = True, pos_mode: str = 'regression',
                 n_pos_bins_per_dim: int = 10, pos_smooth_factor: int = 100, keypoints_path: str = None):
        assert ori_mode in ['regression', 'classification', 'keypoints']
        assert pos_mode in ['regression', 'classification', 'keypoints']
        if pos_mode == 'keypoints' or ori_mode == 'keypoints':
            assert keypoints_path is not None
        self.ori_mode, self.pos_mode, self.camera = ori_mode, pos_mode, camera
        self.orientation = OrientationHistogram(n_ori_bins_per_dim, ori_smooth_factor, ori_delete_unused_bins)
        self.position = PositionHistogram(n_pos_bins_per_dim, pos_smooth_factor)
        # KeyPoints(camera, path) like the reference (spe_utils.py:54); a ready KeyPoints object is accepted too
        if keypoints_path is None or hasattr(keypoints_path, 'keypoints3d'):
            self.keypoints = keypoints_path
        else:
            from .keypoints import KeyPoints
            self.keypoints = KeyPoints(camera, keypoints_path)

    @staticmethod
    def get_score(true_pose: dict, pred_pose: dict) -> dict:
        """ESA score, spe_utils.py:103-159 (same definitions and error behaviour)."""
        pos_err = np.linalg.norm(true_pose['pos'] - pred_pose['pos'], axis=1)
        norm_pos = pos_err / np.linalg.norm(true_pose['pos'], axis=1)
        s = np.abs(np.sum(pred_pose['ori'] * true_pose['ori'], axis=1, keepdims=True))
        if np.any(s > 1.01):
            raise ValueError('Intermediate sum issue due to error in model prediction (orientation)')
        s[s > 1] = 1
        ori = np.mean(2 * np.arccos(s))
        return {'esa_score': ori + np.mean(norm_pos), 'ori_score': ori, 'pos_score': np.mean(norm_pos),
                'ori_error': ori * 180 / np.pi, 'pos_error': np.mean(pos_err)}
