"""Per-kernel timing of the forward under different executor options (GPU box). Prints ms/step per kernel."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd')]

import numpy as np
import torch

from spef_amd import _lib as L
from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.engine import Engine
from spef_amd.weights import synthetic_state_dict


def run(eng, fr, ori, pos, opts, steps=10, label=''):
    for k, v in opts.items():
        eng.set_option(k, v)
    for _ in range(3):
        eng.forward(fr, ori, pos)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.forward(fr, ori, pos)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    eng.profile_begin()
    for _ in range(steps):
        eng.forward(fr, ori, pos)
    prof = eng.profile_end()
    tot = sum(v[1] for v in prof.values()) / steps
    print(f'== {label}: wall {wall:.3f} ms/step, kernel sum {tot:.3f} ms/step, {fr.shape[0] / wall * 1e3:.0f} img/s')
    for k, v in sorted(prof.items(), key=lambda kv: -kv[1][1]):
        print(f'   {v[1] / steps * 1e3:8.1f} us  x{v[0] / steps:4.1f}  {v[2] / (v[1] / 1e3) / 1e9 if v[1] else 0:7.0f} GB/s'
              f'  {v[3] / (v[1] / 1e3) / 1e12 if v[1] else 0:6.1f} TF/s  {k}')
    return ori.clone(), pos.clone()


def main():
    B, S = int(os.environ.get('B', 64)), int(os.environ.get('S', 512))
    sd = synthetic_state_dict(mobilenet_v2(), seed=1001)
    if os.environ.get('DT') == 'int8':   # the C5 path: calibrated int8 blob (bench.py run_int8)
        from spef_amd.blob_q8 import pack_int8
        from spef_amd.data.synthetic import synth_frames
        from spef_amd.quant import calibrate
        eng = Engine(pack_int8(sd, calibrate(sd, synth_frames(4, 128, 128, 900))), 'cuda:0')
    else:
        eng = Engine(Bl.pack(sd, dtype='fp16'), 'cuda:0')
    rng = np.random.Generator(np.random.PCG64(0))
    fr = torch.from_numpy(rng.integers(0, 256, (B, S, S, 3), dtype=np.uint8)).cuda()
    ori = torch.empty((B, 1728), device='cuda')
    pos = torch.empty((B, 3), device='cuda')
    if os.environ.get("SWEEP"):
        # OPTS="7:1,6:0" -> extra spef_set_option(option, value) pairs for every sweep point
        extra = {int(k): int(v) for k, v in (kv.split(':') for kv in os.environ.get('OPTS', '').split(',') if kv)}
        for v in [int(x) for x in os.environ.get("SWEEP", "0,1,2").split(",")]:
            run(eng, fr, ori, pos, {L.OPT_FUSE_BLOCKS: 1, L.OPT_IRB_VARIANT: v, **extra},
                label=f'fused variant {v} {extra}')
        return
    ref = run(eng, fr, ori, pos, {L.OPT_FUSE_BLOCKS: 0, L.OPT_PW_GEMM: 0}, label='unfused, direct pw')
    g = run(eng, fr, ori, pos, {L.OPT_FUSE_BLOCKS: 0, L.OPT_PW_GEMM: 1}, label='unfused, LDS GEMM')
    print('gemm == direct:', torch.equal(ref[0], g[0]))
    for mhw in (0, 64 * 64, 128 * 128):
        f = run(eng, fr, ori, pos, {L.OPT_FUSE_BLOCKS: 1, L.OPT_PW_GEMM: 1, L.OPT_FUSE_MIN_HW: mhw},
                label=f'fused if HW >= {mhw}, LDS GEMM')
        print('fused == direct:', torch.equal(ref[0], f[0]))


if __name__ == '__main__':
    main()
