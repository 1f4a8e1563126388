"""Per-kernel timings and logit differences of the executor modes (GPU box):
python tools/modes.py  -> baseline (VALU depthwise, slab kernels), MFMA depthwise, + strip kernels."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd'), os.path.join(ROOT, 'tools')]
import numpy as np
import torch

from explore import run
from spef_amd import _lib as L
from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.engine import Engine
from spef_amd.weights import synthetic_state_dict

B, S = int(os.environ.get('B', 64)), int(os.environ.get('S', 512))
eng = Engine(Bl.pack(synthetic_state_dict(mobilenet_v2(), seed=1001), dtype='fp16'), 'cuda:0')
fr = torch.from_numpy(np.random.Generator(np.random.PCG64(0)).integers(0, 256, (B, S, S, 3), dtype=np.uint8)).cuda()
ori = torch.empty((B, 1728), device='cuda')
pos = torch.empty((B, 3), device='cuda')
modes = {"slab": {L.OPT_STRIP: 0, L.OPT_WAVESPEC: 0}, "wavespec": {L.OPT_STRIP: 0, L.OPT_WAVESPEC: 1}}
sel = os.environ.get('MODES')
ref = None
for name, opts in modes.items():
    if sel and name not in sel.split(','):
        continue
    o, p = run(eng, fr, ori, pos, opts, label=name)
    if ref is None:
        ref = (o, p)
    else:
        print(f'   max|d ori logit| vs first mode {(o - ref[0]).abs().max().item():.3e}, '
              f'pos {(p - ref[1]).abs().max().item():.3e}')
