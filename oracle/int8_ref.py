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

Bit widths (``qp['bits']``, the reference's bit_width.json as spef_amd.quant.BitWidths; None = all 8): every
quantizer below keeps its own width b in 3..8 -- weights L = 2^(b-1) - 1, unsigned ReLU quantizers [0, 2^b - 1],
signed input / shared quantizers [-2^(b-1), 2^(b-1) - 1] (the 8-bit values are written out below).

Integer semantics (every scale a float64 on the host):
  weights       s_w[c] = max|W[c]| / 127 (>= 2e-16); q_w = clip(rint(W / s_w), -127, 127)
  conv+BN+quant acc = sum q_x q_w (exact int); y / s_out = acc * m[c] + b[c] with
                g = gamma / sqrt(var + 1e-5), h = beta - mean * g, m = (s_in * s_w * g) / s_out, b = h / s_out;
                evaluated in fixed point: q = (acc * M + B) >> sh  (int64, arithmetic shift), see ``fixed``;
                clip to [0, 255] after ReLU, to [-128, 127] for the signed shared quantizers
  residual      q_sum = q_proj + q_in (both at the block's shared scale s_q), then requantised to the next
                consumer's scale: clip_s8(fixed(q_sum, s_q / s_next, 0))
  input         u8 frame -> q = clip(rint(f32(f32(u) / 255) / f32(s_img)), -128, 127) (float32 ops)
  pool          sum over the H*W map, shifted right by tb = b_last + ceil(log2(H*W)) - b_pool (TruncTo8bit
                floor; ceil(log2(H*W)) at 8 bits): pooled u8 at scale s_pool = s_l * 2**tb / (H*W)
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


class _Bits:
    """Quantizer widths of ``qp['bits']`` (duck-typed spef_amd.quant.BitWidths; None = every width 8)."""

    def __init__(self, bw):
        self.bw = bw

    def __getattr__(self, k):
        if self.bw is None:
            return (8, 8) if k in ('first_conv', 'last_conv', 'fully_connected') else 8
        return getattr(self.bw, k)

    def block(self, i):
        return (8, 8, 8, 8, 8) if self.bw is None else tuple(8 if v is None else v for v in self.bw.block(i))


def weight_q(w, bits: int = 8):
    """IntWeightQuant, per output channel, narrow range (quantizers.py:16-20): -> (q int64, s float64 [cout])."""
    w = _np(w).astype(np.float64)
    L = (1 << (bits - 1)) - 1
    s = np.maximum(np.abs(w.reshape(w.shape[0], -1)).max(axis=1) / L, 2e-16)
    q = np.clip(np.rint(w / s.reshape((-1,) + (1,) * (w.ndim - 1))), -L, L).astype(np.int64)
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


def conv_requant_params(sd, prefix, s_in, s_out, wbits: int = 8):
    """QConvBnAct weights + fixed-point requant (shared by the stem, expand, dw, project, last conv)."""
    q, s_w = weight_q(sd[f'{prefix}.0.weight'], wbits)
    g, h = bn(sd, prefix)
    m = (s_in * s_w * g) / s_out
    b = h / s_out
    return q, fixed(m, b)


def input_lut(s_img: float, bits: int = 8) -> np.ndarray:
    """uint8 frame value -> quantized input (ToTensor /255 in float32, then round(x / s_img) in float32), clipped to
    the signed input quantizer (QuantIdentity(signed=True), mobilenet_v2.py:177-178)."""
    x = np.arange(256, dtype=np.float32) / np.float32(255.0)
    return np.clip(np.rint(x / np.float32(s_img)), -(1 << (bits - 1)), (1 << (bits - 1)) - 1).astype(np.int64)


def _conv_int(x, q, stride, groups):
    """Exact integer convolution through float64 (every partial sum < 2**53)."""
    k = q.shape[-1]
    y = F.conv2d(torch.from_numpy(x.astype(np.float64)), torch.from_numpy(q.astype(np.float64)), None, stride,
                 (k - 1) // 2, 1, groups)
    return np.rint(y.numpy()).astype(np.int64)


def pool_shift(hw: int, last_bits: int = 8, pool_bits: int = 8) -> int:
    """The TruncTo8bit shift: the sum of hw b_last-bit codes has b_last + ceil(log2(hw)) bits, truncated to the
    pooling width (ceil(log2(hw)) when both are 8)."""
    return max(last_bits + (hw - 1).bit_length() - pool_bits, 0)


def head_params(sd, qp: Dict, hw: int):
    """Per-launch FC constants for a feature map of ``hw`` pixels: -> dict of (q_w, q_b, sc) per branch."""
    bits = _Bits(qp.get('bits'))
    tb = pool_shift(hw, bits.last_conv[1], bits.pooling)
    s_pool = qp['last'] * 2.0 ** tb / hw
    wb, bb = bits.fully_connected
    out = {}
    for name, key in (('ori', 'head.ori.1'), ('pos', 'head.pos.0')):
        q, s_w = weight_q(sd[f'{key}.weight'], wb)
        b = _np(sd[f'{key}.bias']).astype(np.float64)
        qb = np.clip(np.rint(b / (s_pool * s_w)), -(1 << (bb - 1)), (1 << (bb - 1)) - 1).astype(np.int64)
        out[name] = (q, qb, (s_pool * s_w).astype(np.float32))
    return tb, out


def int8_forward(frames_u8: np.ndarray, sd: Dict, qp: Dict, residual: bool = True, upto: int | None = None):
    """uint8 NHWC frames -> (ori logits f32, pos f32), or the integer activation after block ``upto``
    (NCHW int64; 0 = stem output) / ``upto='last'`` (last conv output) / ``upto='pool'``."""
    bits = _Bits(qp.get('bits'))
    slo, shi = -(1 << (bits.shared_act - 1)), (1 << (bits.shared_act - 1)) - 1
    x = input_lut(qp['image'], bits.image)[frames_u8.astype(np.int64)].transpose(0, 3, 1, 2)       # NCHW int
    q, (M, B, S) = conv_requant_params(sd, f'{FP}.0', qp['image'], qp['stem'], bits.first_conv[0])
    x = requant(_conv_int(x, q, 2, 1), M, B, S, 0, (1 << bits.first_conv[1]) - 1)
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
        ew, ea, dwb, da, pw = bits.block(n)
        y, j = x, 0
        if t != 1:
            q, (M, B, S) = conv_requant_params(sd, f'{FP}.{idx}.conv.0', s_in, bq['expand'], ew)
            y = requant(_conv_int(y, q, 1, 1), M, B, S, 0, (1 << ea) - 1)
            s_y, j = bq['expand'], 1
        else:
            s_y = s_in
        q, (M, B, S) = conv_requant_params(sd, f'{FP}.{idx}.conv.{j}', s_y, bq['dw'], dwb)
        y = requant(_conv_int(y, q, stride, q.shape[0]), M, B, S, 0, (1 << da) - 1)
        if res:
            q, (M, B, S) = conv_requant_params(sd, f'{FP}.{idx}.conv.{j + 1}', bq['dw'], s_q, pw)
            p = requant(_conv_int(y, q, 1, 1), M, B, S, slo, shi)
            R, RB, RS = fixed(s_q / s_next, 0.0)
            x = np.clip(((p + x) * R[0] + RB[0]) >> RS[0], slo, shi)
        else:
            q, (M, B, S) = conv_requant_params(sd, f'{FP}.{idx}.conv.{j + 1}', bq['dw'], s_next, pw)
            x = requant(_conv_int(y, q, 1, 1), M, B, S, slo, shi)
        if upto == idx:
            return x
    q, (M, B, S) = conv_requant_params(sd, f'{FP}.18', qp['final'], qp['last'], bits.last_conv[0])
    x = requant(_conv_int(x, q, 1, 1), M, B, S, 0, (1 << bits.last_conv[1]) - 1)
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
    bits = _Bits(qp.get('bits'))
    slo, shi = -(1 << (bits.shared_act - 1)), (1 << (bits.shared_act - 1)) - 1

    def wq(key, wb):
        q, s = weight_q(sd[key], wb)
        return torch.from_numpy((q * s.reshape((-1,) + (1,) * (q.ndim - 1))).astype(np.float32))

    def cbn(x, prefix, stride, groups, wb):
        w = wq(f'{prefix}.0.weight', wb)
        k = w.shape[-1]
        x = F.conv2d(x, w, None, stride, (k - 1) // 2, 1, groups)
        t = lambda n: torch.as_tensor(_np(sd[f'{prefix}.1.{n}']), dtype=f32)
        return F.batch_norm(x, t('running_mean'), t('running_var'), t('weight'), t('bias'), False, 0.1, 1e-5)

    x = torch.from_numpy(frames_u8).permute(0, 3, 1, 2).to(f32) / 255.0
    ib = bits.image
    x = _fq(x, float(np.float32(qp['image'])), -(1 << (ib - 1)), (1 << (ib - 1)) - 1)
    x = _fq(F.relu(cbn(x, f'{FP}.0', 2, 1, bits.first_conv[0])), float(np.float32(qp['stem'])), 0,
            (1 << bits.first_conv[1]) - 1)
    for n, (idx, cin, cout, stride, t, res) in enumerate(blocks_topology(residual)):
        bq = qp['blocks'][n]
        ew, ea, dwb, da, pw = bits.block(n)
        if bq['quant'] is not None:
            x = _fq(x, float(np.float32(bq['quant'])), slo, shi)
        y, j = x, 0
        if t != 1:
            y = _fq(F.relu(cbn(y, f'{FP}.{idx}.conv.0', 1, 1, ew)), float(np.float32(bq['expand'])), 0, (1 << ea) - 1)
            j = 1
        y = _fq(F.relu(cbn(y, f'{FP}.{idx}.conv.{j}', stride, y.shape[1], dwb)), float(np.float32(bq['dw'])), 0,
                (1 << da) - 1)
        y = cbn(y, f'{FP}.{idx}.conv.{j + 1}', 1, 1, pw)
        x = _fq(y, float(np.float32(bq['quant'])), slo, shi) + x if res else y
    x = _fq(x, float(np.float32(qp['final'])), slo, shi)
    x = _fq(F.relu(cbn(x, f'{FP}.18', 1, 1, bits.last_conv[0])), float(np.float32(qp['last'])), 0,
            (1 << bits.last_conv[1]) - 1)
    hw = x.shape[2] * x.shape[3]
    tb = pool_shift(hw, bits.last_conv[1], bits.pooling)
    s_l = float(np.float32(qp['last']))
    pooled = torch.floor(torch.round(x / s_l).sum(dim=(2, 3)) / 2 ** tb) * (s_l * 2 ** tb / hw)
    outs = []
    wb, bb = bits.fully_connected
    for key in ('head.ori.1', 'head.pos.0'):
        w = wq(f'{key}.weight', wb)
        q, s_w = weight_q(sd[f'{key}.weight'], wb)
        s_b = torch.from_numpy((s_l * 2.0 ** tb / hw * s_w).astype(np.float32))
        b = torch.clamp(torch.round(torch.as_tensor(_np(sd[f'{key}.bias']), dtype=f32) / s_b), -(1 << (bb - 1)),
                        (1 << (bb - 1)) - 1) * s_b
        outs.append(F.linear(pooled, w, b))
    return outs[0], outs[1]
