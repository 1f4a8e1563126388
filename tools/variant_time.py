"""Per-kernel timing of one precision variant (GPU box): python tools/variant_time.py [dtype] [head] [B].
dtype fp16 | bf16 | fp32 | fp16x2 | int8 (URSONet only); head ursonet (512x512) | keypoints (240x384, forward + sigmoid + EPnP)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd')]

import numpy as np
import torch

from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.engine import Engine
from spef_amd.weights import synthetic_state_dict


def main():
    dt = sys.argv[1] if len(sys.argv) > 1 else 'fp16x2'
    head = sys.argv[2] if len(sys.argv) > 2 else 'ursonet'
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    steps = 10
    if head == 'keypoints':
        arch, (H, W) = mobilenet_v2('keypoints'), (240, 384)
        sd = synthetic_state_dict(arch, seed=1001, head_std=0.002)
    else:
        arch, (H, W) = mobilenet_v2('ursonet', 1728, 3), (512, 512)
        sd = synthetic_state_dict(arch, seed=1001)
    if dt == 'int8':   # the C5 path, scales calibrated on random frames (timing only)
        from spef_amd.blob_q8 import pack_int8
        from spef_amd.quant import calibrate
        cal = np.random.Generator(np.random.PCG64(9)).integers(0, 256, (4, 128, 128, 3), dtype=np.uint8)
        blob = pack_int8(sd, calibrate(sd, cal))
    else:
        blob = Bl.pack(sd, arch, dtype=dt)
    eng = Engine(blob, 'cuda:0')
    if head == 'keypoints':
        g = np.load(os.path.join(ROOT, 'tests', 'golden', 'keypoints.npz'))
        eng.set_keypoints(g['kp3d'], g['K'], float(g['nu']), float(g['nv']))
    eng.reserve(B, H, W)
    rng = np.random.Generator(np.random.PCG64(0))
    fr = torch.from_numpy(rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8)).cuda()

    def step():
        o, p = eng.forward(fr)
        if head == 'keypoints':
            eng.decode_keypoints(o)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    eng.profile_begin()
    for _ in range(steps):
        step()
    prof = eng.profile_end()
    tot = sum(v[1] for v in prof.values()) / steps
    print(f'== {dt} {head} B={B} {H}x{W}: wall {wall:.3f} ms/step ({B / wall * 1e3:.0f} img/s), kernel sum {tot:.3f} ms')
    for k, v in sorted(prof.items(), key=lambda kv: -kv[1][1]):
        print(f'   {v[1] / steps * 1e3:8.1f} us  x{v[0] / steps:4.1f}  {v[2] / (v[1] / 1e3) / 1e9 if v[1] else 0:7.0f} GB/s'
              f'  {v[3] / (v[1] / 1e3) / 1e12 if v[1] else 0:6.1f} TF/s  {k}', flush=True)
    eng.close()


if __name__ == '__main__':
    main()
