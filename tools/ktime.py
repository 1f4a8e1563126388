"""Per-kernel forward time of one library build (SPEF_LIB) on the fp16mx headline workload (GPU box, development
tool; no decode, so timing-ablation builds with wrong outputs run too): python tools/ktime.py [dtype] -> one JSON line
{kernel: us per step}. tools/ktime.sh alternates builds."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd')]

import numpy as np
import torch

from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.engine import Engine
from spef_amd.weights import synthetic_state_dict

dt = sys.argv[1] if len(sys.argv) > 1 else 'fp16mx'
B, S, steps = int(os.environ.get('B', 64)), int(os.environ.get('S', 512)), int(os.environ.get('STEPS', 20))
eng = Engine(Bl.pack(synthetic_state_dict(mobilenet_v2(), seed=1001), dtype=dt), 'cuda:0')
fr = torch.from_numpy(np.random.Generator(np.random.PCG64(0)).integers(0, 256, (B, S, S, 3), dtype=np.uint8)).cuda()
for _ in range(10):
    eng.forward(fr)
torch.cuda.synchronize()
eng.profile_begin()
for _ in range(steps):
    eng.forward(fr)
prof = eng.profile_end()
print(json.dumps({k: round(v[1] / steps * 1e3, 2) for k, v in prof.items()}))
