"""Per-block URSONet logit error attribution at a sharp head (CPU experiment, not product code).

tools/sharp_head_budget.py applies one fp16 rounding class at a time to the whole network. This tool splits the
same classes per block, so a mixed schedule (fp16 where the budget allows, hi + lo where it does not) can be chosen
from measurements rather than guessed. Everything is restated in float64 at the bench's sharp head (orientation
Linear std 0.3, seed 1001, tests/golden/cases.py scale) on the bench's own SPEED-style frames (synth_frames(.., 10_000),
the frames bench.py's sharp-head leg uses).

Rounding classes of a block (the fp16 schedule's rounding points):
  W1  its 1x1 weights fp16 (expand + project; 'last': the last conv)     WD  depthwise weights fp16
  H   expand output fp16      D  depthwise output fp16      O  block output fp16 (stem: 'S', the stem output)
  A   depthwise accumulated in packed fp16 (blocks 2-7 of the fp16 schedule)
Blocks: 0 = stem (+ block 1 is block 1), 1..17, 18 = last conv.

Modes:
  attrib   one (block, class) rounded, everything else exact: max |d logit| and rms |d pooled| per entry; errors of
           independent rounding points add roughly in quadrature, so the table ranks where precision is needed.
  schedule a named mixed schedule (SCHEDULES below) with every rounding point it has, against the exact run.
Usage: python tools/precision_budget.py attrib|schedule [frames] [size] [schedule names...]"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd'))
from spef_amd.arch import mobilenet_v2  # noqa: E402
from spef_amd.blob import fold_bn  # noqa: E402
from spef_amd.data.synthetic import synth_frames  # noqa: E402
from spef_amd.weights import synthetic_state_dict  # noqa: E402


def r16(t):
    return t.to(torch.float16).to(torch.float64)


def r32(t):
    return t.to(torch.float32).to(torch.float64)


def hilo(t):
    hi = r16(t)
    return hi + r16(r32(t) - hi)


ROUND = {'x': lambda t: t, 'r': r16, 'h': hilo, 'f': r32}


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


class Net:
    def __init__(self, sd, arch):
        self.arch = arch
        self.sd = sd
        self.w = {}
        for c in arch.all_convs():
            w, b = fold_bn(sd, c)
            self.w[c.prefix] = (torch.from_numpy(w), torch.from_numpy(b))
        self.hw = torch.from_numpy(sd['head.ori.1.weight'].astype(np.float64))
        self.hb = torch.from_numpy(sd['head.ori.1.bias'].astype(np.float64))

    def conv(self, t, spec, stride, groups, act, wmode='x'):
        w, b = self.w[spec.prefix]
        w = ROUND[wmode](w)
        y = F.conv2d(t, w, b, stride, (w.shape[-1] - 1) // 2, 1, groups)
        return F.relu(y) if act else y

    def stem(self, x, rule):
        return ROUND[rule(0, 'S')](self.conv(x, self.arch.stem, 2, 1, True))

    def block(self, y, blk, rule):
        i = blk.index
        cv = list(blk.convs)
        h = y
        if blk.expand != 1:
            h = ROUND[rule(i, 'H')](self.conv(h, cv.pop(0), 1, 1, True, rule(i, 'W1')))
        if rule(i, 'A') == 'r':
            w, b = self.w[cv[0].prefix]
            h = F.relu(dw_f16acc(h, ROUND[rule(i, 'WD')](w), b, blk.stride))
        else:
            h = ROUND[rule(i, 'D')](self.conv(h, cv[0], blk.stride, blk.hidden, True, rule(i, 'WD')))
        o = self.conv(h, cv[1], 1, 1, False, rule(i, 'W1'))
        if blk.residual:
            o = o + y
        return ROUND[rule(i, 'O')](o)

    def tail(self, y, rule):
        f = self.conv(y, self.arch.last, 1, 1, True, rule(18, 'W1')).mean((2, 3))
        return F.linear(f, self.hw, self.hb), f

    def forward(self, x, rule, start=0, y=None):
        """Whole net (start 0) or from block ``start`` (1..18) given that block's input ``y``."""
        if start == 0:
            y = self.stem(x, rule)
            start = 1
        for blk in self.arch.blocks[start - 1:]:
            y = self.block(y, blk, rule)
        return self.tail(y, rule)


# mixed schedules: rule(block, class) -> 'x' exact | 'r' fp16 | 'h' hi+lo fp16 pair | 'f' fp32
def sched_fp16(i, c):
    if c == 'A':
        return 'r' if 2 <= i <= 7 else 'x'
    return 'r'


def mixed(rounded):
    """Exact (hi + lo) weights, fp32 depthwise accumulation and fp32 activations everywhere except the rounding
    points in ``rounded``: a set of (block range, class) pairs stored as fp16 (e.g. ((0, 6), 'O'))."""
    def rule(i, c):
        if c in ('W1', 'WD'):
            return 'h'
        if c == 'A':
            return 'x'
        for (a, b), cl in rounded:
            if a <= i <= b and cl == c:
                return 'r'
        return 'f'
    return rule


EARLY = (0, 6)
SCHEDULES = {
    'fp16': sched_fp16,
    'fp16x2': mixed(()),
    'exactw': mixed([((0, 18), c) for c in 'SHDO']),
    'S1 early HOS': mixed([(EARLY, 'H'), (EARLY, 'O'), (EARLY, 'S')]),
    'S1b early HOS, late H': mixed([(EARLY, 'H'), (EARLY, 'O'), (EARLY, 'S'), ((7, 17), 'H')]),
    'S2 early HDOS': mixed([(EARLY, 'H'), (EARLY, 'O'), (EARLY, 'S'), (EARLY, 'D')]),
    'S3 all H, early OS': mixed([((0, 17), 'H'), (EARLY, 'O'), (EARLY, 'S')]),
    'S4 early HOS to 3': mixed([((0, 3), 'H'), ((0, 3), 'O'), ((0, 3), 'S')]),
    'S5 all HO': mixed([((0, 17), 'H'), ((0, 17), 'O'), ((0, 17), 'S')]),
    'S6 early OS': mixed([(EARLY, 'O'), (EARLY, 'S')]),
    'S7 early HS, all O': mixed([(EARLY, 'H'), (EARLY, 'S'), ((0, 17), 'O')]),
    'mx O1-6': mixed([((1, 6), 'O')]),
    'mx O1-7': mixed([((1, 7), 'O')]),
    'mx O1-6 H2-4': mixed([((1, 6), 'O'), ((2, 4), 'H')]),
    'mx O1-6 S': mixed([((1, 6), 'O'), ((0, 0), 'S')]),
    'mx O1-6 H2-7': mixed([((1, 6), 'O'), ((2, 7), 'H')]),
    'mx O1-6 H2-7 S': mixed([((1, 6), 'O'), ((2, 7), 'H'), ((0, 0), 'S')]),
    'mx O1-7 H2-7 S': mixed([((1, 7), 'O'), ((2, 7), 'H'), ((0, 0), 'S')]),
    'mx O1-6 H247': mixed([((1, 6), 'O'), ((2, 2), 'H'), ((4, 4), 'H'), ((7, 7), 'H')]),
    'mx O1-6 H247 S': mixed([((1, 6), 'O'), ((2, 2), 'H'), ((4, 4), 'H'), ((7, 7), 'H'), ((0, 0), 'S')]),
    'mx O1-3 H2-7 S': mixed([((1, 3), 'O'), ((2, 7), 'H'), ((0, 0), 'S')]),
    'mx O1-4 H2-7 S': mixed([((1, 4), 'O'), ((2, 7), 'H'), ((0, 0), 'S')]),
    'mx O1-2 H2-7 S': mixed([((1, 2), 'O'), ((2, 7), 'H'), ((0, 0), 'S')]),
    'mx O1-3 H2-4 S': mixed([((1, 3), 'O'), ((2, 4), 'H'), ((0, 0), 'S')]),
    'mx O1-3 H2-3 S': mixed([((1, 3), 'O'), ((2, 3), 'H'), ((0, 0), 'S')]),
    'mx O1-3 H2-7': mixed([((1, 3), 'O'), ((2, 7), 'H')]),
    'mx O1-2 H2-4 S': mixed([((1, 2), 'O'), ((2, 4), 'H'), ((0, 0), 'S')]),
    'mx O1-3 H247 S': mixed([((1, 3), 'O'), ((2, 2), 'H'), ((4, 4), 'H'), ((7, 7), 'H'), ((0, 0), 'S')]),
}


def test_frames(b, h, w, seed):
    """tests/test_gpu_mx.py's blocky random frames (FRAMES=test)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    base = rng.integers(0, 40, (b, h, w, 1), dtype=np.uint8)
    blob = rng.integers(0, 215, (b, h // 4, w // 4, 1), dtype=np.uint8).repeat(4, 1).repeat(4, 2)
    return np.repeat(np.clip(base.astype(np.int32) + blob, 0, 255).astype(np.uint8), 3, axis=3)


def setup(n, s, hs=0.3):
    torch.set_num_threads(8)
    arch = mobilenet_v2('ursonet', 1728, 3)
    sd = synthetic_state_dict(arch, seed=1001, head_std=hs, pos_std=0.01, pos_bias=(0.3, -0.2, 12.0))
    fr = test_frames(n, s, s, 77) if os.environ.get('FRAMES') == 'test' else synth_frames(n, s, s, 10_000)
    x = torch.from_numpy(fr).permute(0, 3, 1, 2).to(torch.float64) / 255.0
    return Net(sd, arch), x


def exact(i, c):
    return 'x'


def attrib(net, x):
    with torch.no_grad():
        # exact block inputs, so a perturbation at block b restarts from b
        ins = {}
        y = net.stem(x, exact)
        for blk in net.arch.blocks:
            ins[blk.index] = y
            y = net.block(y, blk, exact)
        ins[18] = y
        ref, fref = net.tail(y, exact)
        print(f'logit max {ref.abs().max():.3f}; pooled mean {fref.mean():.3f} max {fref.max():.3f}', flush=True)
        rows = []
        for i in range(0, 19):
            classes = ['S'] if i == 0 else (['W1'] if i == 18 else ['W1', 'WD', 'H', 'D', 'O', 'A'])
            for c in classes:
                if c == 'H' and net.arch.blocks[i - 1].expand == 1:
                    continue
                rule = (lambda i0, c0: (lambda j, k: 'r' if (j, k) == (i0, c0) else 'x'))(i, c)
                if i == 0:
                    o, f = net.forward(x, rule)
                elif i == 18:
                    o, f = net.tail(ins[18], rule)
                else:
                    o, f = net.forward(None, rule, start=i, y=ins[i])
                d = (o - ref).abs().max().item()
                rows.append((i, c, d, (f - fref).pow(2).mean().sqrt().item()))
                print(f'block {i:2d} {c:3s} max|d logit| {d:.3e}  rms|d pooled| {rows[-1][3]:.3e}', flush=True)
        return rows


def schedule(net, x, names):
    with torch.no_grad():
        ref, fref = net.forward(x, exact)
        for nm in names:
            o, f = net.forward(x, SCHEDULES[nm])
            print(f'{nm:20s} max|d logit| {(o - ref).abs().max().item():.3e}  '
                  f'rms|d logit| {(o - ref).pow(2).mean().sqrt().item():.3e}  '
                  f'rms|d pooled| {(f - fref).pow(2).mean().sqrt().item():.3e}', flush=True)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else 'attrib'
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    s = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    net, x = setup(n, s)
    if mode == 'attrib':
        rows = attrib(net, x)
        print('\nper block, quadrature sum over classes (max |d logit|):')
        for i in range(19):
            v = [r[2] for r in rows if r[0] == i]
            print(f'  block {i:2d}: {np.sqrt(np.sum(np.square(v))):.3e}')
        for c in ('W1', 'WD', 'H', 'D', 'O', 'A', 'S'):
            v = [r[2] for r in rows if r[1] == c]
            print(f'  class {c:3s}: {np.sqrt(np.sum(np.square(v))):.3e}')
    else:
        schedule(net, x, sys.argv[4:] or list(SCHEDULES))


if __name__ == '__main__':
    main()
