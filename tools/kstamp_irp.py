"""Per-chunk timeline of the three-stage kernel (GPU box, timing build: tools/build_variant.py stamp3 -DSPEF_X2_STAMP=1
-DSPEF_X2_K1516=5; SPEF_LIB=abx2/stamp3.so). Slots: MFMA wave 0 -- 0 loop start, 1 after P(c-1) issue, 2 after E(c+1)
issue (before the barrier); VALU wave 4 -- 4 loop start, 5 depthwise done, 6 before the barrier; slot 3 of chunks 0 / 1:
MFMA wave 0 at entry / after its fragments; slot 7 of chunks 0 / 1: MFMA epilogue done / VALU entry."""
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
OPS = [tuple(int(v) for v in a.split(':')) for a in (sys.argv[1:] or ['15:30'])]   # op:chunks (PT: x tiles)
for op, nch in OPS:
    eng.probe(fr, op)
    y = eng.probe(fr, op)
    torch.cuda.synchronize()
    st = y.flatten()[:8 * nch].cpu().numpy().view(np.uint32).astype(np.int64).reshape(nch, 8)
    t0 = st[0, 0]
    per = np.diff(st[:, 0])
    med = lambda v: int(np.median(v))  # noqa: E731
    print(f'block {op}: {nch} chunks, loop {st[-1, 2] - t0} cycles; per chunk (median): period {med(per)}, '
          f'MFMA start->P issued {med(st[:, 1] - st[:, 0])}, ->E issued {med(st[:, 2] - st[:, 0])}, '
          f'barrier wait {med(st[1:, 0] - st[:-1, 2])}; VALU start->DMA issued {med(st[:, 5] - st[:, 4])}, '
          f'->prebar {med(st[:, 6] - st[:, 4])}, barrier wait {med(st[1:, 4] - st[:-1, 6])}')
    print(f'   entry->fragments {st[1, 3] - st[0, 3]}, entry->loop {t0 - st[0, 3]}, loop end->epilogue {st[0, 7] - st[-1, 2]}')
    for c in sorted(set([0, 1, 2, nch // 2 - 1, nch // 2, nch // 2 + 1, nch - 2, nch - 1])):
        print('   ', c, st[c, 0] - t0, st[c, 1] - t0, st[c, 2] - t0, '|', st[c, 4] - t0, st[c, 5] - t0, st[c, 6] - t0)
