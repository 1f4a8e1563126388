"""INT8 restatement of the reference's Brevitas-quantized MobileNet-V2 + URSONet head (ORACLE -- test
infrastructure only).

Reference graph (all bit widths 8, ``src/config/train/exp_1/bit_width.json``):
  * input       ``QuantIdentity(InputQuant, bit_width=8, signed=True)``          mobilenet_v2.py:177-178
  * stem        ``QConvBnAct``: QuantConv2d (int8 per-output-channel weights, ``IntWeightQuant``,
                quantizers.py:16-20) -> BatchNorm2d -> QuantReLU (unsigned 8-bit, ``UintActQuant``)
                brevitas_layers.py:10-54
  * blocks      ``QInvertedResidual`` brevitas_layers.py:57-136: [expand QConvBnAct] -> dw QConvBnAct ->
                project conv+BN (no activation, no quant); a shared signed quantizer ``self.quant``
                (``IntActQuant``) quantizes the block input when ``input_quant or use_residual`` and, for
                residual blocks, the projection output before ``x + residual`` (:126-136); ``input_quant``
                per mobilenet_v2.py:189-197 (every block but the first, with residual connections)
  * final       signed ``QuantIdentity`` on the last block's output                 mobilenet_v2.py:208-211
  * last conv   ``QConvBnAct`` 320 -> 1280, unsigned 8-bit ReLU quant               mobilenet_v2.py:213-217
  * head        ``QURSONetHead`` ursonet.py:36-93: ``QuantAvgPool2d`` with ``TruncTo8bit`` over the whole
                map, then ``QuantLinear`` (int8 per-channel weights, ``Int8Bias`` 8-bit bias) for pos / ori.
                The reference's pooling table (model.py:242-247) has no 512x512 entry; the kernel is the whole
                feature map here (16x16 at 512x512), the natural extension.

Brevitas itself (``brevitas==0.7.1``) is absent, and no reference file pins its numerics: **parity is
unpinned against Brevitas**. This module fixes the integer semantics the MI355X kernels implement and that
the GPU is held to BIT-EXACTLY (``int8_forward``), and restates the Brevitas float fake-quant graph
(``fake_quant_forward``) to measure how far the integer semantics sit from it (rare 1-LSB rounding flips).

Integer semantics (every scale a float64 on the host):
  weights       s_w[c] = max|W[c]| / 127 (>= 2e-16); q_w = clip(rint(W / s_w), -127, 127)
  conv+BN+quant acc = sum q_x q_w (exact int); y / s_out = acc * m[c] + b[c] with
                g = gamma / sqrt(var + 1e-5), h = beta - mean * g, m = (s_in * s_w * g) / s_out, b = h / s_out;
                evaluated in fixed point: q = (acc * M + B) >> sh  (int64, arithmetic shift), see ``fixed``;
                clip to [0, 255] after ReLU, to [-128, 127] for the signed shared quantizers
  residual      q_sum = q_proj + q_in (both at the block's shared scale s_q), then requantised to the next
                consumer's scale: clip_s8(fixed(q_sum, s_q / s_next, 0))
  input         u8 frame -> q = clip(rint(f32(f32(u) / 255) / f32(s_img)), -128, 127) (float32 ops)
  pool          sum over the H*W map, shifted right by tb = ceil(log2(H*W)) (TruncTo8bit floor):
                pooled u8 at scale s_pool = s_l * 2**tb / (H*W)
  FC            q_b[c] = clip(rint(b[c] / (s_pool * s_w[c])), -128, 127); out = f32(acc) * f32(s_pool * s_w[c])
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn.functional as F

_IR = ((1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2), (6, 320, 1, 1))
FP = 'features.features'


def _np(v):
    return v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)


def blocks_topology(residual: bool = True) -> List[Tuple[int, int, int, int, int, bool]]:
    """-> [(idx, cin, cout, stride, t, use_residual)] for the 17 inverted residuals (mobilenet_v2.py:186-203)."""
    out, cin, idx = [], 32, 1
    for t, c, n, s in _IR:
        for i in range(n):
            stride = s if i == 0 else 1
            out.append((idx, cin, c, stride, t, stride == 1 and cin == c and residual))
            cin, idx = c, idx + 1
    return out


def weight_q(w):
    """IntWeightQuant, 8 bit, per output channel (quantizers.py:16-20): -> (q int64, s float64 [cout])."""
    w = _np(w).astype(np.float64)
    s = np.maximum(np.abs(w.reshape(w.shape[0], -1)).max(axis=1) / 127.0, 2e-16)
    q = np.clip(np.rint(w / s.reshape((-1,) + (1,) * (w.ndim - 1))), -127, 127).astype(np.int64)
    return q, s


def bn(sd, prefix):
    g = _np(sd[f'{prefix}.1.weight']).astype(np.float64) / np.sqrt(_np(sd[f'{prefix}.1.running_var']).astype(np.float64) + 1e-5)
    h = _np(sd[f'{prefix}.1.bias']).astype(np.float64) - _np(sd[f'{prefix}.1.running_mean']).astype(np.float64) * g
    return g, h


def fixed(m, b):
    """Per-channel fixed-point form of ``x * m + b``: -> (M int64, B int64 incl. the rounding half, sh int64)
    with q = (x * M + B) >> sh. sh = 32 exactly when 2**-12 <= |m| < 0.5 (every realistic conv scale: the fused
    kernel's requant is the high word of one 64-bit multiply-add), otherwise |m| * 2**sh in [2**29, 2**30); sh
    capped so |b| * 2**sh < 2**61."""
    m = np.atleast_1d(np.asarray(m, np.float64))
    b = np.broadcast_to(np.atleast_1d(np.asarray(b, np.float64)), m.shape)
    M = np.zeros(m.shape, np.int64)
    B = np.zeros(m.shape, np.int64)
    S = np.zeros(m.shape, np.int64)
    for i in range(m.size):
        em = math.frexp(abs(m[i]))[1] if m[i] != 0 else -30
        eb = math.frexp(abs(b[i]))[1] if b[i] != 0 else -200
        sh0 = 30 - em
        if 2.0 ** -12 <= abs(m[i]) < 0.5:
            # sh = 32 exactly: M = rint(m 2**32) in [2**20, 2**31) keeps the requant error below 2**-13 LSB for
            # outputs in the 8-bit range, and the fused kernels take the high word of acc * M + B with no shift
            sh0 = 32
        sh = int(min(sh0, 61 - eb, 62))
        assert sh >= 1, (m[i], b[i])
        M[i] = int(np.rint(math.ldexp(m[i], sh)))
        B[i] = int(np.rint(math.ldexp(b[i], sh))) + (1 << (sh - 1))
        S[i] = sh
    return M, B, S


def requant(acc, M, B, S, lo, hi, axis=1):
    """clip((acc * M + B) >> sh, lo, hi) with per-channel (M, B, sh) along ``axis`` of int64 ``acc``."""
    shp = [1] * acc.ndim
    shp[axis] = -1
    v = (acc * M.reshape(shp) + B.reshape(shp)) >> S.reshape(shp)
    return np.clip(v, lo, hi)


def conv_requant_params(sd, prefix, s_in, s_out):
    """QConvBnAct weights + fixed-point requant (shared by the stem, expand, dw, project, last conv)."""
    q, s_w = weight_q(sd[f'{prefix}.0.weight'])
    g, h = bn(sd, prefix)
    m = (s_in * s_w * g) / s_out
    b = h / s_out
    return q, fixed(m, b)


def input_lut(s_img: float) -> np.ndarray:
    """uint8 frame value -> quantized input (ToTensor /255 in float32, then round(x / s_img) in float32)."""
    x = np.arange(256, dtype=np.float32) / np.float32(255.0)
    return np.clip(np.rint(x / np.float32(s_img)), -128, 127).astype(np.int64)


def _conv_int(x, q, stride, groups):
    """Exact integer convolution through float64 (every partial sum < 2**53)."""
    k = q.shape[-1]
    y = F.conv2d(torch.from_numpy(x.astype(np.float64)), torch.from_numpy(q.astype(np.float64)), None, stride,
                 (k - 1) // 2, 1, groups)
    return np.rint(y.numpy()).astype(np.int64)


def pool_shift(hw: int) -> int:
    """ceil(log2(hw)): the accumulator growth TruncTo8bit removes."""
    return (hw - 1).bit_length()


def head_params(sd, qp: Dict, hw: int):
    """Per-launch FC constants for a feature map of ``hw`` pixels: -> dict of (q_w, q_b, sc) per branch."""
    tb = pool_shift(hw)
    s_pool = qp['last'] * 2.0 ** tb / hw
    out = {}
    for name, key in (('ori', 'head.ori.1'), ('pos', 'head.pos.0')):
        q, s_w = weight_q(sd[f'{key}.weight'])
        b = _np(sd[f'{key}.bias']).astype(np.float64)
        qb = np.clip(np.rint(b / (s_pool * s_w)), -128, 127).astype(np.int64)
        out[name] = (q, qb, (s_pool * s_w).astype(np.float32))
    return tb, out


def int8_forward(frames_u8: np.ndarray, sd: Dict, qp: Dict, residual: bool = True, upto: int | None = None):
    """uint8 NHWC frames -> (ori logits f32, pos f32), or the integer activation after block ``upto``
    (NCHW int64; 0 = stem output) / ``upto='last'`` (last conv output) / ``upto='pool'``."""
    x = input_lut(qp['image'])[frames_u8.astype(np.int64)].transpose(0, 3, 1, 2)       # NCHW int
    q, (M, B, S) = conv_requant_params(sd, f'{FP}.0', qp['image'], qp['stem'])
    x = requant(_conv_int(x, q, 2, 1), M, B, S, 0, 255)
    if upto == 0:
        return x
    s_x = qp['stem']
    topo = blocks_topology(residual)
    for n, (idx, cin, cout, stride, t, res) in enumerate(topo):
        bq = qp['blocks'][n]
        s_q = bq['quant']
        s_next = qp['blocks'][n + 1]['quant'] if n + 1 < len(topo) else qp['final']
        # the block input arrives already at s_q (the previous project requantised to it) or, for block 1,
        # as the stem's unsigned output
        s_in = s_q if s_q is not None else s_x
        y, j = x, 0
        if t != 1:
            q, (M, B, S) = conv_requant_params(sd, f'{FP}.{idx}.conv.0', s_in, bq['expand'])
            y = requant(_conv_int(y, q, 1, 1), M, B, S, 0, 255)
            s_y, j = bq['expand'], 1
        else:
            s_y = s_in
        q, (M, B, S) = conv_requant_params(sd, f'{FP}.{idx}.conv.{j}', s_y, bq['dw'])
        y = requant(_conv_int(y, q, stride, q.shape[0]), M, B, S, 0, 255)
        if res:
            q, (M, B, S) = conv_requant_params(sd, f'{FP}.{idx}.conv.{j + 1}', bq['dw'], s_q)
            p = requant(_conv_int(y, q, 1, 1), M, B, S, -128, 127)
            R, RB, RS = fixed(s_q / s_next, 0.0)
            x = np.clip(((p + x) * R[0] + RB[0]) >> RS[0], -128, 127)
        else:
            q, (M, B, S) = conv_requant_params(sd, f'{FP}.{idx}.conv.{j + 1}', bq['dw'], s_next)
            x = requant(_conv_int(y, q, 1, 1), M, B, S, -128, 127)
        if upto == idx:
            return x
    q, (M, B, S) = conv_requant_params(sd, f'{FP}.18', qp['final'], qp['last'])
    x = requant(_conv_int(x, q, 1, 1), M, B, S, 0, 255)
    if upto == 'last':
        return x
    hw = x.shape[2] * x.shape[3]
    tb, hp = head_params(sd, qp, hw)
    pooled = x.reshape(x.shape[0], x.shape[1], -1).sum(axis=2) >> tb
    if upto == 'pool':
        return pooled
    outs = []
    for name in ('ori', 'pos'):
        qw, qb, sc = hp[name]
        acc = pooled.astype(np.float64) @ qw.astype(np.float64).T            # exact (< 2**53)
        acc = np.rint(acc).astype(np.int64) + qb
        outs.append(acc.astype(np.float32) * sc)
    return outs[0], outs[1]


# --------------------------------------------------------------------------- Brevitas float fake-quant graph


def _fq(x, s, lo, hi):
    return torch.clamp(torch.round(x / s), lo, hi) * s


@torch.no_grad()
def fake_quant_forward(frames_u8: np.ndarray, sd: Dict, qp: Dict, residual: bool = True):
    """The same network as Brevitas evaluates it: float32 tensors holding quantized values, dequantized
    weights, float BatchNorm, round-half-even quantizers (for measuring the integer semantics' distance)."""
    f32 = torch.float32

    def wq(key):
        q, s = weight_q(sd[key])
        return torch.from_numpy((q * s.reshape((-1,) + (1,) * (q.ndim - 1))).astype(np.float32))

    def cbn(x, prefix, stride, groups):
        w = wq(f'{prefix}.0.weight')
        k = w.shape[-1]
        x = F.conv2d(x, w, None, stride, (k - 1) // 2, 1, groups)
        t = lambda n: torch.as_tensor(_np(sd[f'{prefix}.1.{n}']), dtype=f32)
        return F.batch_norm(x, t('running_mean'), t('running_var'), t('weight'), t('bias'), False, 0.1, 1e-5)

    x = torch.from_numpy(frames_u8).permute(0, 3, 1, 2).to(f32) / 255.0
    x = _fq(x, float(np.float32(qp['image'])), -128, 127)
    x = _fq(F.relu(cbn(x, f'{FP}.0', 2, 1)), float(np.float32(qp['stem'])), 0, 255)
    for n, (idx, cin, cout, stride, t, res) in enumerate(blocks_topology(residual)):
        bq = qp['blocks'][n]
        if bq['quant'] is not None:
            x = _fq(x, float(np.float32(bq['quant'])), -128, 127)
        y, j = x, 0
        if t != 1:
            y = _fq(F.relu(cbn(y, f'{FP}.{idx}.conv.0', 1, 1)), float(np.float32(bq['expand'])), 0, 255)
            j = 1
        y = _fq(F.relu(cbn(y, f'{FP}.{idx}.conv.{j}', stride, y.shape[1])), float(np.float32(bq['dw'])), 0, 255)
        y = cbn(y, f'{FP}.{idx}.conv.{j + 1}', 1, 1)
        x = _fq(y, float(np.float32(bq['quant'])), -128, 127) + x if res else y
    x = _fq(x, float(np.float32(qp['final'])), -128, 127)
    x = _fq(F.relu(cbn(x, f'{FP}.18', 1, 1)), float(np.float32(qp['last'])), 0, 255)
    hw = x.shape[2] * x.shape[3]
    tb = pool_shift(hw)
    s_l = float(np.float32(qp['last']))
    pooled = torch.floor(torch.round(x / s_l).sum(dim=(2, 3)) / 2 ** tb) * (s_l * 2 ** tb / hw)
    outs = []
    for key in ('head.ori.1', 'head.pos.0'):
        w = wq(f'{key}.weight')
        q, s_w = weight_q(sd[f'{key}.weight'])
        s_b = torch.from_numpy((s_l * 2.0 ** tb / hw * s_w).astype(np.float32))
        b = torch.clamp(torch.round(torch.as_tensor(_np(sd[f'{key}.bias']), dtype=f32) / s_b), -128, 127) * s_b
        outs.append(F.linear(pooled, w, b))
    return outs[0], outs[1]
