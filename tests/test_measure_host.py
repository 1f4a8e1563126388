"""Host logic of the measurement and comparison helpers (no GPU): the spe_finn.py:116-149 statistics and the
clock-stamp arithmetic of bench.py's timed-region shader clock."""
import numpy as np
import torch

from spef_amd.measure import ClockProbe
from spef_amd.tools.compare import feature_stats


def test_feature_stats_match_reference_definitions():
    rng = np.random.default_rng(0)
    ref = np.maximum(rng.normal(size=(4, 8, 8, 16)), 0).astype(np.float32)       # a ReLU map
    got = ref + np.where(ref > 0, rng.normal(scale=1e-3, size=ref.shape), 0).astype(np.float32)
    got[0, 0, 0, :4] = 0.0
    st = feature_stats(got, ref)
    d = got.astype(np.float64) - ref
    assert np.isclose(st['mse'], np.mean(d * d))                                   # spe_finn.py:121
    assert np.isclose(st['nonzero_reference'], np.count_nonzero(ref) / ref.size)  # :116-119
    assert np.isclose(st['zero_pattern'], np.mean((got == 0) == (ref == 0)))       # :128-130
    close = torch.isclose(torch.from_numpy(got), torch.from_numpy(ref), atol=1e-6, rtol=1e-6)
    assert np.isclose(st['isclose_1e-6'], close.float().mean().item())             # :147-149
    assert st['max_abs'] == float(np.abs(d).max())
    assert feature_stats(ref, ref)['mse'] == 0.0 and feature_stats(ref, ref)['isclose_1e-6'] == 1.0


def test_clock_probe_per_cu_arithmetic():
    """Two stamps per CU: MHz = delta shader cycles / delta 100 MHz ticks x 100, from the first wave each stamp put on
    that CU; CUs stamped only once are ignored; the median over CUs is reported."""
    p = ClockProbe.__new__(ClockProbe)
    key = lambda xcd, cu: (xcd << 8) | cu   # noqa: E731
    a = np.array([[key(0, 1), 1000, 50], [key(0, 1), 900, 10], [key(1, 2), 5000, 100], [key(2, 3), 7, 7]], np.int64)
    b = np.array([[key(0, 1), 2_000_900, 1010], [key(1, 2), 2_005_000, 1100], [key(3, 4), 1, 1]], np.int64)
    p.buf = [torch.from_numpy(a), torch.from_numpy(b)]
    r = p.mhz()
    # CU (0,1): first wave of stamp a = realtime 10 (cycles 900) -> 2,000,000 cycles / 1000 ticks x 100 = 200,000 MHz
    # CU (1,2): 2,000,000 / 1000 x 100 = 200,000 MHz as well
    assert r['cus'] == 2 and r['sclk_mhz'] == 200000.0
    assert set(r['per_xcd_median']) == {'0', '1'}
