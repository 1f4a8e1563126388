"""Orientation-decode timing on the GPU box: the bench's logits (random-weight net, 1728-bin URSONet head) and
sharpened / flattened versions of them, decode_ori alone (HIP events, 200 launches), plus the number of
repeated-squaring steps sym4_top_eigvec needs per image (numpy restatement of k_head.hip's loop)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd')]

import numpy as np
import torch

from spef_amd import _lib as L
from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.data.synthetic import synth_frames
from spef_amd.engine import Engine
from spef_amd.spe.spe_utils import SPEUtils
from spef_amd.weights import synthetic_state_dict


def squarings(p, qb):
    a = np.einsum('bi,ij,ik->bjk', p.astype(np.float64), qb, qb)
    out = []
    for m in a:
        m = m / np.trace(m)
        for it in range(40):
            trm = np.trace(m)
            q = m @ m
            tr = np.trace(q)
            m = q / tr
            if tr >= (1 - 1e-15) * trm * trm:
                break
        out.append(it + 1)
    return np.array(out)


def main():
    B = int(os.environ.get('B', 64))
    sd = synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=1001)
    eng = Engine(Bl.pack(sd, dtype='fp16'), 'cuda:0')
    su = SPEUtils(None, 'classification', 12, 3, False, 'regression')
    qb = np.asarray(su.orientation.histogram, np.float64)
    eng.set_decode_tables(qb, None)
    fr = torch.from_numpy(synth_frames(B, 512, 512, 0)).cuda()
    o, p = eng.forward(fr)
    torch.cuda.synchronize()
    base = o.clone()
    for scale in (1.0, 0.1, 10.0, 100.0):
        x = (base * scale).contiguous()
        pr = torch.softmax(x, 1).cpu().numpy()
        it = squarings(pr, qb)
        for _ in range(10):
            eng.decode(1, 0, x, p, want_soft=True)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        n = 200
        ev[0].record()
        for _ in range(n):
            eng.decode(1, 0, x, p, want_soft=True)
        ev[1].record()
        torch.cuda.synchronize()
        eng.profile_begin()
        for _ in range(n):
            eng.decode(1, 0, x, p, want_soft=True)
        prof = eng.profile_end()
        ks = {k: v[1] / v[0] * 1e3 for k, v in prof.items()}
        print(f'scale {scale:6.1f}: logit std {x.std().item():.3f}  squarings mean {it.mean():.1f} max {it.max()}  '
              f'decode call {ev[0].elapsed_time(ev[1]) / n * 1e3:.1f} us  per kernel (us): '
              + ', '.join(f'{k} {v:.1f}' for k, v in sorted(ks.items())), flush=True)
    time.sleep(0)


if __name__ == '__main__':
    main()
