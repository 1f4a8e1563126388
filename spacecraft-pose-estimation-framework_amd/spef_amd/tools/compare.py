"""Backbone-output comparison statistics of the reference's accelerator check (``SPEFinn.predict_and_compare``,
src/finn/spe_finn.py:116-149), used for the C2 feature check and the per-precision host evaluation
(build_mi355x): share of non-zero elements of each map (:116-119), MSE (:121), zero-pattern similarity
(:128-130) and ``torch.isclose(atol=rtol=1e-6)`` similarity (:147-149), plus max |delta| and relative RMS."""
from __future__ import annotations

import numpy as np


def feature_stats(got, ref) -> dict:
    """``got``: the variant's features, ``ref``: the reference's (same shape, any layout; float arrays)."""
    a = np.asarray(got, np.float64)
    b = np.asarray(ref, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    d = a - b
    close = np.abs(d) <= 1e-6 + 1e-6 * np.abs(b)          # torch.isclose(a, b, atol=1e-6, rtol=1e-6)
    return {'elements': int(a.size),
            'nonzero_variant': float(np.count_nonzero(a) / a.size),
            'nonzero_reference': float(np.count_nonzero(b) / b.size),
            'mse': float(np.mean(d * d)),
            'max_abs': float(np.abs(d).max()),
            'rel_rms': float(np.sqrt(np.mean(d * d) / max(np.mean(b * b), 1e-30))),
            'zero_pattern': float(np.mean((a == 0) == (b == 0))),
            'isclose_1e-6': float(np.mean(close))}
