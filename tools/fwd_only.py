"""Minimal forward loop for counter collection: python tools/fwd_only.py [iters] (B=64, 512x512; DT=fp16|bf16|int8)."""
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

it = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B, S = int(os.environ.get('B', 64)), int(os.environ.get('S', 512))
sd = synthetic_state_dict(mobilenet_v2(), seed=1001)
if os.environ.get('DT') == 'int8':   # the C5 path, calibrated like bench.py --dtype int8
    from bench import synth_frames
    from spef_amd.blob_q8 import pack_int8
    from spef_amd.quant import calibrate
    eng = Engine(pack_int8(sd, calibrate(sd, synth_frames(4, 128, 128, 900))), 'cuda:0')
else:
    eng = Engine(Bl.pack(sd, dtype=os.environ.get('DT', 'fp16')), 'cuda:0')
fr = torch.from_numpy(np.random.Generator(np.random.PCG64(0)).integers(0, 256, (B, S, S, 3), dtype=np.uint8)).cuda()
for _ in range(it):
    eng.forward(fr)
torch.cuda.synchronize()
print('ok')
