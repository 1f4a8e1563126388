"""Throughput of one B=64 forward vs K concurrent streams of B=64/K each (GPU box): does splitting the batch over
HIP streams fill the kernels' tails?  python tools/streams.py"""
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

blob = Bl.pack(synthetic_state_dict(mobilenet_v2(), seed=1001), dtype=os.environ.get('DT', 'fp16'))
B = 64
fr = torch.from_numpy(np.random.Generator(np.random.PCG64(0)).integers(0, 256, (B, 512, 512, 3), dtype=np.uint8)).cuda()
for K in (1, 2, 4):
    engs = [Engine(blob, 'cuda:0') for _ in range(K)]
    sts = [torch.cuda.Stream() for _ in range(K)]
    parts = [fr[i * B // K:(i + 1) * B // K].contiguous() for i in range(K)]
    for it in range(2):
        torch.cuda.synchronize()
        steps = 5 if it == 0 else 30
        t0 = time.perf_counter()
        for _ in range(steps):
            for e, s, p in zip(engs, sts, parts):
                with torch.cuda.stream(s):
                    e.forward(p)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
    print(f'K={K} streams x B={B // K}: {dt * 1e3:.3f} ms/step, {B / dt:.0f} img/s', flush=True)
    for e in engs:
        e.close()
