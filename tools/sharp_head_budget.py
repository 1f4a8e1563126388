"""URSONet logit error budget at a sharp head (CPU experiment, not product code; VERDICT r3 "weak" 1).

The north star bounds the orientation logits at an absolute 1e-3 against float32. Their error is W . d(pooled
features), linear in the head's weight scale, so the reference init (Linear std 0.01) flatters any storage
precision. This restates the fp16 schedule in float64 (every rounding point of the HIP kernels, DESIGN.md section
5) and applies one rounding class at a time, at the fixtures' sharp head (head_std 0.3, tests/golden/cases.py):
  W1  1x1 weights (expand, project, last conv) fp16        WD  depthwise weights fp16
  S   stem output fp16         H  expand output fp16        D  depthwise output fp16
  O   block outputs fp16       A  depthwise accumulated in fp16 (blocks 2-7, the packed kernels)
and prints max |d logit| against the unrounded float64 run.
Usage: python tools/sharp_head_budget.py [frames] [size] [head_std]"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd'))
from spef_amd.arch import mobilenet_v2  # noqa: E402
from spef_amd.blob import fold_bn  # noqa: E402
from spef_amd.weights import synthetic_state_dict  # noqa: E402


def r16(t):
    return t.to(torch.float16).to(torch.float64)


def hilo(t):
    hi = r16(t)
    return hi + r16(t - hi)


def dw_f16acc(t, w, b, stride):
    n, c, h, wd = t.shape
    oh, ow = (h - 1) // stride + 1, (wd - 1) // stride + 1
    tp = F.pad(t, (1, 1, 1, 1))
    acc = r16(b.view(1, c, 1, 1).expand(n, c, oh, ow).clone())
    for kx in range(3):
        for ky in range(3):
            win = tp[:, :, ky:ky + stride * (oh - 1) + 1:stride, kx:kx + stride * (ow - 1) + 1:stride]
            acc = r16(acc + win * w[:, 0, ky, kx].view(1, c, 1, 1))
    return acc


def forward(x, sd, arch, cls, hl=()):
    def rnd(t, c):
        if c in hl:
            return hilo(t)
        return r16(t) if c in cls else t

    def conv(t, spec, stride, groups, act, wc):
        w, b = fold_bn(sd, spec)
        w = torch.from_numpy(w)
        if wc:
            w = rnd(w, wc)
        y = F.conv2d(t, w, torch.from_numpy(b), stride, (w.shape[-1] - 1) // 2, 1, groups)
        return F.relu(y) if act else y
    y = rnd(conv(x, arch.stem, 2, 1, True, None), 'S')
    for blk in arch.blocks:
        cv = list(blk.convs)
        h = y
        if blk.expand != 1:
            h = rnd(conv(h, cv.pop(0), 1, 1, True, 'W1'), 'H')
        if 'A' in cls and 2 <= blk.index <= 7:
            w, b = fold_bn(sd, cv[0])
            w = torch.from_numpy(w)
            h = F.relu(dw_f16acc(h, rnd(w, 'WD'), torch.from_numpy(b), blk.stride))
        else:
            h = rnd(conv(h, cv[0], blk.stride, blk.hidden, True, 'WD'), 'D')
        o = conv(h, cv[1], 1, 1, False, 'W1')
        if blk.residual:
            o = o + y
        y = rnd(o, 'O')
    f = conv(y, arch.last, 1, 1, True, 'W1').mean((2, 3))
    w = torch.from_numpy(sd['head.ori.1.weight'].astype(np.float64))
    return F.linear(f, w, torch.from_numpy(sd['head.ori.1.bias'].astype(np.float64))), f


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    s = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    hs = float(sys.argv[3]) if len(sys.argv) > 3 else 0.3
    torch.set_num_threads(8)
    arch = mobilenet_v2('ursonet', 1728, 3)
    sd = synthetic_state_dict(arch, seed=1001, head_std=hs)
    rng = np.random.Generator(np.random.PCG64(5))
    fr = rng.integers(0, 256, (n, s, s, 3), dtype=np.uint8)
    x = torch.from_numpy(fr).permute(0, 3, 1, 2).to(torch.float64) / 255.0
    allc = {'W1', 'WD', 'S', 'H', 'D', 'O', 'A'}
    with torch.no_grad():
        ref, fref = forward(x, sd, arch, set())
        print(f'head_std {hs}: logit max {ref.abs().max():.3f}; pooled feature mean {fref.mean():.3f}, '
              f'max {fref.max():.3f}', flush=True)

        def run(name, cls, hl=()):
            o, f = forward(x, sd, arch, cls, hl)
            print(f'{name:44s} logits max|d| {(o - ref).abs().max().item():.3e}   '
                  f'pooled rms|d| {(f - fref).pow(2).mean().sqrt().item():.3e}', flush=True)
        for c in ('W1', 'WD', 'S', 'H', 'D', 'O', 'A'):
            run(f'{c} alone', {c})
        run('all (the fp16 schedule)', allc)
        run('all but A (fp32 dw accumulation)', allc - {'A'})
        run('all, hi+lo W1', allc, ('W1',))
        run('all, hi+lo W1+WD', allc, ('W1', 'WD'))
        run('all but A, hi+lo W1+WD', allc - {'A'}, ('W1', 'WD'))
        run('all but A, hi+lo W1+WD+O', allc - {'A'}, ('W1', 'WD', 'O'))
        run('all but A, hi+lo W1+WD+O+S', allc - {'A'}, ('W1', 'WD', 'O', 'S'))
        run('all but A, hi+lo everything', allc - {'A'}, ('W1', 'WD', 'O', 'S', 'H', 'D'))


if __name__ == '__main__':
    main()
