"""GPU box: logits of a schedule on the parity tests' sharp-head frames -> gpurun_out/<dtype>_logits.npz, for a CPU
comparison against tools/precision_budget.py's restatement of the same schedule (development tool)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd'), os.path.join(ROOT, 'tools')]
import numpy as np
import torch

from precision_budget import test_frames
from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.engine import Engine
from spef_amd.weights import synthetic_state_dict

dt = sys.argv[1] if len(sys.argv) > 1 else 'fp16mx'
sd = synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=1001, head_std=0.3, pos_std=0.01,
                          pos_bias=(0.3, -0.2, 12.0))
fr = test_frames(4, 512, 512, 77)
e = Engine(Bl.pack(sd, dtype=dt), 'cuda:0')
tag = dt
if os.environ.get('MXK') is not None:   # SPEF_OPT_MX_KERNELS (8): 0 = fp16x2 slab kernels for blocks 1-7
    from spef_amd import _lib as L
    e.set_option(L.OPT_MX_KERNELS, int(os.environ['MXK']))
    tag += '_mxk' + os.environ['MXK']
probe = [int(v) for v in os.environ.get('PROBE', '').split(',') if v]
o, p = e.forward(torch.from_numpy(fr).cuda())
acts = {f'act{k}': e.probe(torch.from_numpy(fr).cuda(), k).cpu().numpy() for k in probe}
os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
np.savez(os.path.join(ROOT, 'gpurun_out', f'{tag}_logits.npz'), ori=o.cpu().numpy(), pos=p.cpu().numpy(), **acts)
print('saved', o.shape)
