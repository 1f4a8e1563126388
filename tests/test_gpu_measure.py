"""The bench line's measurement legs on the GPU (csrc/k_ubench.hip through spef_measure_peaks / spef_clock_stamp):
plausible MI355X figures, and a clock probe that brackets real work. Ranges are wide on purpose -- they catch a
broken kernel or unit (a factor of 2 or 1000), not box-to-box variation."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_measured_peaks_are_plausible():
    from spef_amd.measure import measure_peaks
    p = measure_peaks(0, reps=1)
    # dense fp16 MFMA: 2.5 PFLOP/s nominal at 2.4 GHz; measured 1.8 PFLOP/s at the 1.83 GHz the loop holds
    assert 800.0 < p['fp16_mfma_tflops'] < 2700.0, p
    # int8 MFMA runs at twice the fp16 rate per clock
    assert 1.5 < p['int8_mfma_tops'] / p['fp16_mfma_tflops'] < 2.6, p
    # HBM3E: 8 TB/s nominal; the copy / read streams measured 4.3-4.7 TB/s
    assert 2000.0 < p['hbm_read_gbs'] < 8500.0 and 2000.0 < p['hbm_copy_gbs'] < 8500.0, p
    for k in ('sclk_mhz_fp16_loop', 'sclk_mhz_int8_loop'):
        assert 800.0 < p[k] < 2600.0, p


def test_clock_probe_brackets_a_busy_region():
    from spef_amd.measure import ClockProbe
    dev = torch.device('cuda:0')
    probe = ClockProbe(dev)
    a = torch.randn(4096, 4096, device=dev, dtype=torch.float16)
    (a @ a).clamp_(-1, 1)              # library initialisation outside the probed region: the shader-cycle counter
    torch.cuda.synchronize(dev)        # does not advance while the GPU idles, so idle time reads as a low clock
    probe.start()
    for _ in range(200):
        a = (a @ a).clamp_(-1, 1)
    probe.stop()
    r = probe.mhz()
    assert r is not None and r['cus'] >= 128, r          # most of the 256 CUs stamped twice
    assert 500.0 < r['sclk_mhz'] < 2600.0, r
    assert set(r['per_xcd_median']) <= {str(i) for i in range(8)} and len(r['per_xcd_median']) >= 4, r
    lo, hi = r['spread_mhz']
    assert lo <= r['sclk_mhz'] <= hi, r
