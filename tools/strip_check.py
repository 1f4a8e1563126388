"""Strip-streaming (k_irs.hip) vs LDS-slab (k_irb.hip) fused blocks: per-block max |diff| and timings (GPU box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd')]
import numpy as np
import torch

from spef_amd import _lib as L
from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.engine import Engine
from spef_amd.weights import synthetic_state_dict

sd = synthetic_state_dict(mobilenet_v2(), seed=1001)
for dt in ('fp16', 'bf16'):
    eng = Engine(Bl.pack(sd, dtype=dt), 'cuda:0')
    for (b, h, w) in [(2, 512, 512), (3, 240, 384), (2, 100, 136)]:
        fr = torch.from_numpy(np.random.Generator(np.random.PCG64(h)).integers(0, 256, (b, h, w, 3), dtype=np.uint8)).cuda()
        worst = []
        for op in range(2, 18):
            eng.set_option(L.OPT_STRIP, 0)
            u = eng.probe(fr, op).float()
            eng.set_option(L.OPT_STRIP, 1)
            f = eng.probe(fr, op).float()
            d = (u - f).abs().max().item()
            worst.append((op, d, u.abs().max().item()))
        print(dt, (b, h, w), ' '.join(f'{op}:{d:.2e}/{m:.1f}' for op, d, m in worst), flush=True)
    eng.close()
