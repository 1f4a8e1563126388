"""Batch-level pipelining over HIP streams (GPU box): consecutive batches of B=64 alternate between K streams
(one engine context each), so one batch's low-occupancy tail kernels overlap the next batch's front kernels.
python tools/streams2.py"""
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
from oracle import decode_ref as D

blob = Bl.pack(synthetic_state_dict(mobilenet_v2(), seed=1001), dtype=os.environ.get('DT', 'fp16'))
B = 64
fr = torch.from_numpy(np.random.Generator(np.random.PCG64(0)).integers(0, 256, (B, 512, 512, 3), dtype=np.uint8)).cuda()
h, _ = D.orientation_histogram(12, False)
for K in (1, 2, 3, 4):
    engs = [Engine(blob, 'cuda:0') for _ in range(K)]
    for e in engs:
        e.set_decode_tables(h, None)
    sts = [torch.cuda.Stream() for _ in range(K)]
    outs = [(torch.empty((B, 1728), device='cuda'), torch.empty((B, 3), device='cuda')) for _ in range(K)]
    for it in range(2):
        steps = 6 if it == 0 else 60
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for st in range(steps):
            i = st % K
            with torch.cuda.stream(sts[i]):
                o, p = engs[i].forward(fr, *outs[i])
                engs[i].decode(1, 0, o, p)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
    print(f'K={K} streams, batches of {B} alternating: {dt * 1e3:.3f} ms/batch, {B / dt:.0f} img/s', flush=True)
    for e in engs:
        e.close()
