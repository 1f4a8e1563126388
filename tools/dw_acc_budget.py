"""Depthwise accumulation-precision budget (CPU experiment, not product code): what does accumulating the 3x3
depthwise in fp16 (v_pk_fma_f16, two channels per op) instead of fp32 (v_fma_mix_f32 / v_dot2_f32_f16) cost on the
URSONet outputs against float32 (BASELINE.json north star: logits within 1e-3)?

A float64 BN-folded restatement of the fp16 schedule (every rounding point of the HIP kernels)
is run with the depthwise of a chosen set of blocks accumulated tap by tap with an fp16 rounding after every fused
multiply-add (kx outer, ky inner, the bias as the initial value, as a packed-fp16 kernel would), and the max |delta|
of the 1728 orientation logits and 3 position outputs against the unrounded float64 run is printed.
Usage: python tools/dw_acc_budget.py [frames] [size]"""
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


def dw_f16acc(t, w, b, stride):
    """Depthwise 3x3 (pad 1) with every partial sum rounded to fp16 (fused multiply-add, bias first)."""
    n, c, h, wd = t.shape
    oh, ow = (h - 1) // stride + 1, (wd - 1) // stride + 1
    tp = F.pad(t, (1, 1, 1, 1))
    acc = r16(b.view(1, c, 1, 1).expand(n, c, oh, ow).clone())
    for kx in range(3):
        for ky in range(3):
            win = tp[:, :, ky:ky + stride * (oh - 1) + 1:stride, kx:kx + stride * (ow - 1) + 1:stride]
            acc = r16(acc + win * w[:, 0, ky, kx].view(1, c, 1, 1))
    return acc


def forward(x, sd, arch, rounding, f16acc_blocks=()):
    def rnd(t):
        return r16(t) if rounding else t

    def conv(t, spec, stride, groups, act, wround=True):
        w, b = fold_bn(sd, spec)
        w = torch.from_numpy(w)
        if wround and rounding:
            w = r16(w)
        y = F.conv2d(t, w, torch.from_numpy(b), stride, (w.shape[-1] - 1) // 2, 1, groups)
        return F.relu(y) if act else y
    y = rnd(conv(x, arch.stem, 2, 1, True, wround=False))
    for blk in arch.blocks:
        cv = list(blk.convs)
        h = y
        if blk.expand != 1:
            h = rnd(conv(h, cv.pop(0), 1, 1, True))
        if blk.index in f16acc_blocks:
            w, b = fold_bn(sd, cv[0])
            h = F.relu(dw_f16acc(h, r16(torch.from_numpy(w)), torch.from_numpy(b), blk.stride))
        else:
            h = rnd(conv(h, cv[0], blk.stride, blk.hidden, True))
        o = conv(h, cv[1], 1, 1, False)
        if blk.residual:
            o = o + y
        y = rnd(o)
    f = conv(y, arch.last, 1, 1, True).mean((2, 3))
    outs = []
    for k in ('head.ori.1', 'head.pos.0'):
        w = torch.from_numpy(sd[k + '.weight'].astype(np.float64))
        outs.append(F.linear(f, w, torch.from_numpy(sd[k + '.bias'].astype(np.float64))))
    return outs


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    s = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    arch = mobilenet_v2('ursonet', 1728, 3)
    sd = synthetic_state_dict(arch, seed=1001)
    rng = np.random.Generator(np.random.PCG64(5))
    fr = rng.integers(0, 256, (n, s, s, 3), dtype=np.uint8)
    x = torch.from_numpy(fr).permute(0, 3, 1, 2).to(torch.float64) / 255.0
    idx = [b.index for b in arch.blocks]
    s2 = [b.index for b in arch.blocks if b.stride == 2]
    with torch.no_grad():
        ref = forward(x, sd, arch, False)
        print(f'logit magnitude: max {ref[0].abs().max():.3f}, pos max {ref[1].abs().max():.3f}')
        for name, blocks in (('fp16 schedule, fp32 dw accumulation', ()), ('fp16 acc, stride-2 blocks', s2),
                             ('fp16 acc, block 2 only', (2,)), ('fp16 acc, blocks 1-7', tuple(i for i in idx if i <= 7)),
                             ('fp16 acc, every block', tuple(idx))):
            o = forward(x, sd, arch, True, blocks)
            print(f'{name:40s} ori logits max|d| {(o[0] - ref[0]).abs().max().item():.3e}   '
                  f'pos max|d| {(o[1] - ref[1]).abs().max().item():.3e}')


if __name__ == '__main__':
    main()
