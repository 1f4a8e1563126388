"""Adaptive temporal PDF filter of the reference's ``Inference`` engine (src/temporal/pdf_compare.py:9-134).

Host NumPy, per frame: it blends the current soft-classification histogram (``pose['ori_soft']`` /
``pose['pos_soft']``, produced on the GPU by ``SPEMi355x``) with the previous filtered one, weighted by
``exp(-alpha * distance)``. Pinned to the reference by tests/golden/temporal_pdf.npz (every distance metric).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

METRICS = ('l2', 'kl', 'js', 'hellinger', 'tv', 'wasserstein')


class TemporalPDF:
    """Same constructor, attributes and methods as the reference ``TemporalPDF`` (pdf_compare.py:10-22)."""

    def __init__(self, n: float = 1.0, alpha: float = 1.0, distance_metric: str = 'l2'):
        self.n = n
        self.alpha = alpha
        self.distance_metric = distance_metric.lower()
        self.previous_pdf = None

    def reset(self) -> None:
        self.previous_pdf = None

    def compute_distance(self, pdf1: np.ndarray, pdf2: np.ndarray) -> float:
        """pdf_compare.py:32-78: both PDFs renormalised, then the configured distance."""
        p = pdf1 / np.sum(pdf1)
        q = pdf2 / np.sum(pdf2)
        m = self.distance_metric
        if m == 'l2':
            return np.linalg.norm(p - q)
        if m == 'kl':
            eps = 1e-12                                   # log(0) guard, :55
            ps, qs = p + eps, q + eps
            return np.sum(ps * np.log(ps / qs))
        if m == 'js':
            mid = 0.5 * (p + q)
            return np.sqrt(0.5 * (np.sum(p * np.log(p / mid)) + np.sum(q * np.log(q / mid))))
        if m == 'hellinger':
            return np.sqrt(0.5 * np.sum((np.sqrt(p) - np.sqrt(q)) ** 2))
        if m == 'tv':
            return 0.5 * np.sum(np.abs(p - q))
        if m == 'wasserstein':                            # 1-D: L1 of the CDFs over the bin count
            return np.sum(np.abs(np.cumsum(p) - np.cumsum(q))) / len(p)
        raise ValueError(f'Unsupported distance metric: {self.distance_metric}')

    def compute_weight(self, distance: float) -> float:
        """pdf_compare.py:80-92: exp(-alpha d) clipped to [0, 1]."""
        return np.clip(np.exp(-self.alpha * distance), 0.0, 1.0)

    def update_pdf(self, current_pdf: np.ndarray) -> Tuple[np.ndarray, float]:
        """pdf_compare.py:94-134: -> (filtered PDF, distance to the previous one); the first frame passes through."""
        current_pdf = current_pdf / np.sum(current_pdf)
        if self.previous_pdf is None:
            self.previous_pdf = current_pdf
            return current_pdf, 0.0
        distance = self.compute_distance(current_pdf, self.previous_pdf)
        weight = self.compute_weight(distance)
        updated = weight * self.n * current_pdf + (1 - weight) * self.previous_pdf
        updated = updated / np.sum(updated)
        self.previous_pdf = updated
        return updated, distance
