"""Per-chunk timeline of the role-split kernels (GPU box, timing build): SPEF_LIB=abx2/stamp.so (tools/build_variant.py
stamp -DSPEF_X2_STAMP=1). The kernel's tile-0 workgroup records s_memtime (shader cycles) per hidden chunk in LDS and
writes them over its output; Engine.probe returns that output. Slots per chunk: expand wave 0 -- 0 loop start,
2 after the stage stores (register staging only), 1 before the barrier; depthwise wave 4 -- 4 loop start, 5 after the
depthwise (before the project MFMAs), 6 before the barrier; slot 3 of chunks 0 / 1: expand wave 0 at kernel entry /
after the input fragments; slot 7 of chunks 1 / 0: depthwise wave 4 at kernel entry / after the epilogue stores.
Outputs are wrong by construction."""
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

eng = Engine(Bl.pack(synthetic_state_dict(mobilenet_v2(), seed=1001), dtype='fp16mx'), 'cuda:0')
fr = torch.from_numpy(np.random.Generator(np.random.PCG64(0)).integers(0, 256, (64, 512, 512, 3), dtype=np.uint8)).cuda()
for _ in range(3):
    eng.forward(fr)
torch.cuda.synchronize()
PT = int(os.environ.get('KSTAMP_TILES', '2'))   # tiles per workgroup of the persistent blocks (8-14) at B = 64
for op, nch1 in ((8, 12), (12, 18), (15, 30), (17, 30)):
    nch = nch1 * (PT if op < 15 else 1)
    eng.probe(fr, op)
    y = eng.probe(fr, op)
    torch.cuda.synchronize()
    st = y.flatten()[:8 * nch].cpu().numpy().view(np.uint32).astype(np.int64).reshape(nch, 8)
    t0 = st[0, 0]
    per = np.diff(st[:, 0])
    e_busy = (st[:, 1] - st[:, 0])
    d_dw = (st[:, 5] - st[:, 4])
    d_busy = (st[:, 6] - st[:, 4])
    print(f'block {op}: {nch} chunks, total {st[-1, 1] - t0} cycles; per chunk (median): period {int(np.median(per))}, '
          f'expand start->barrier {int(np.median(e_busy))}, stage stores {int(np.median(st[:, 2] - st[:, 0])) if st[0, 2] else "-"}, '
          f'dw start->depthwise done {int(np.median(d_dw))}, dw start->barrier {int(np.median(d_busy))}')
    e0 = st[0, 3]
    print(f'   entry->fragments {st[1, 3] - e0}, entry->loop start {t0 - e0}, last prebar->epilogue done '
          f'{st[0, 7] - st[-1, 6]}, entry->end {st[0, 7] - e0} cycles (dw entry {st[1, 7] - e0:+d})')
    print('   chunks (expand start, prebar | dw start, mid, prebar) rel. to t0:')
    for c in list(range(min(3, nch))) + (list(range(nch1 - 2, nch1 + 3)) if nch > nch1 else []):
        print('   ', c, st[c, 0] - t0, st[c, 1] - t0, '|', st[c, 4] - t0, st[c, 5] - t0, st[c, 6] - t0)
