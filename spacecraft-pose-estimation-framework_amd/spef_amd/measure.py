"""On-box measurement helpers for bench.py (C ABI spef_measure_peaks / spef_clock_stamp, csrc/k_ubench.hip).

``measure_peaks`` re-measures the roofline peaks on the box the bench runs on; ``ClockProbe``
brackets a timed region with two in-kernel clock stamps and returns the shader clock held during it (per CU stamped
in both: delta s_memtime -- shader cycles -- over delta s_memrealtime at 100 MHz; median over CUs, and per XCD)."""
from __future__ import annotations

import ctypes as C
import statistics

import torch

from . import _lib as L


def measure_peaks(device: int = 0, reps: int = 2) -> dict:
    out = (C.c_double * 8)()
    L.check(L.load().spef_measure_peaks(int(device), int(reps), out))

    def cfg(v):
        v = int(v)
        return {'workgroups_per_cu': (v // 100) or 'one per 16-32 KiB block (no grid stride)',
                'loads_in_flight_per_thread': (v // 10) % 10, 'nontemporal': bool(v % 10)}
    return {'fp16_mfma_tflops': round(out[0], 1), 'int8_mfma_tops': round(out[1], 1),
            'hbm_copy_gbs': round(out[2], 1), 'hbm_read_gbs': round(out[3], 1),
            'sclk_mhz_fp16_loop': round(out[4], 1), 'sclk_mhz_int8_loop': round(out[5], 1),
            'hbm_copy_config': cfg(out[6]), 'hbm_read_config': cfg(out[7]),
            'method': 'csrc/k_ubench.hip: best of %d timed launches after a warm-up; MFMA loops on random operands, '
                      '8 chains per wave, 4 waves per SIMD; HBM: 4 GiB buffers (copy counts read + write bytes), '
                      'contiguous 16-32 KiB blocks per workgroup iteration, best of %d launches of each of 4/8/16 '
                      'workgroups per CU or one workgroup per block x 4/8 16-B loads in flight per thread x '
                      'plain/nontemporal' % (reps, reps + 2)}


class ClockProbe:
    """``start()`` / ``stop()`` around a timed region (each enqueues one stamp kernel on the current stream and
    synchronises); ``mhz()`` -> {'sclk_mhz': median over XCDs, 'per_xcd': [...]} or None when no XCD was stamped
    in both."""

    def __init__(self, device: torch.device, n_wg: int = 4096):
        self.dev = torch.device(device)
        self.n = n_wg
        self.buf = [torch.zeros((n_wg, 3), dtype=torch.int64, device=self.dev) for _ in range(2)]

    def _stamp(self, i: int) -> None:
        s = torch.cuda.current_stream(self.dev).cuda_stream
        L.check(L.load().spef_clock_stamp(C.c_void_p(self.buf[i].data_ptr()), self.n, C.c_void_p(s)))
        torch.cuda.synchronize(self.dev)

    def start(self) -> None:
        self._stamp(0)

    def stop(self) -> None:
        self._stamp(1)

    def mhz(self):
        a, b = (t.cpu().numpy() for t in self.buf)
        per_cu = {}
        for key in sorted(set(int(v) for v in a[:, 0]) & set(int(v) for v in b[:, 0])):
            ra, rb = a[a[:, 0] == key], b[b[:, 0] == key]
            # the first wave each stamp put on this CU (smallest realtime), and its own shader-cycle count
            ia, ib = int(ra[:, 2].argmin()), int(rb[:, 2].argmin())
            dt = int(rb[ib, 1]) - int(ra[ia, 1])
            dr = int(rb[ib, 2]) - int(ra[ia, 2])
            if dr > 0 and dt > 0:
                per_cu[key] = dt / dr * 100.0
        if not per_cu:
            return None
        per_xcd = {}
        for key, v in per_cu.items():
            per_xcd.setdefault(key >> 8, []).append(v)
        return {'sclk_mhz': round(statistics.median(per_cu.values()), 1), 'cus': len(per_cu),
                'per_xcd_median': {str(k): round(statistics.median(v), 1) for k, v in sorted(per_xcd.items())},
                'spread_mhz': [round(min(per_cu.values()), 1), round(max(per_cu.values()), 1)]}
