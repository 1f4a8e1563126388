"""INT8 quantisation parameters of the Brevitas-mirroring path.

The reference's quantized model (``QMobileNetV2`` + ``QURSONetHead``; src/modeling/backbone/mobilenet_v2.py:
119-229, common/brevitas_layers.py:10-136, head/ursonet.py:36-93) carries one learned scale per activation
quantizer; weight scales are statistics of the weights (per output channel, quantizers.py:16-20) and are
recomputed at pack time. ``QParams`` holds the activation scales in the reference graph's order:

    image              input QuantIdentity (signed 8-bit)                     mobilenet_v2.py:177-178
    stem               stem QuantReLU (unsigned)                                               :179-182
    blocks[i].quant    shared signed quantizer of block i (None for block 1)   brevitas_layers.py:126-136
    blocks[i].expand   expand QuantReLU (None when t == 1)                                      :103-111
    blocks[i].dw       depthwise QuantReLU                                                      :113-119
    final              signed QuantIdentity after the last block               mobilenet_v2.py:208-211
    last               last conv QuantReLU                                                      :213-217

There is no QAT checkpoint in this environment (the reference's trained models are remote downloads), so
``calibrate`` sets the scales from activation statistics of the float model on calibration frames --
Brevitas' own initialisation of ``ParameterFromRuntimeStats`` scales (a high percentile of |x|) -- which
stands in for QAT.

Bit widths (``BitWidths``, parsed from the reference's ``bit_width.json``, model.py:16-45): every quantizer
keeps its own width from 3 to 8 bits, held in int8 containers -- weights per output channel in
[-(2^(b-1) - 1), 2^(b-1) - 1] (narrow range), unsigned ReLU quantizers in [0, 2^b - 1], the signed shared /
input quantizers in [-2^(b-1), 2^(b-1) - 1]. The reference's ``QMobileNetV2`` default is 3-bit weights and
activations with a 4-bit shared quantizer (mobilenet_v2.py:140-167, ``BitWidths.qmobilenet_default()``);
``config/train/exp_1/bit_width.json`` is all 8 (``BitWidths()``). Widths 1 and 2 select Brevitas' binary /
ternary quantizers (quantizers.py:78-96), a different arithmetic, and are rejected.
"""
from __future__ import annotations

import ast
import json
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from .arch import IR_SETTINGS, mobilenet_v2

FP = 'features.features'


N_BLOCKS = 17


@dataclass(frozen=True)
class BitWidths:
    """Quantizer bit widths of the reference's quantized model, in ``bit_width.json`` terms (model.py:16-45):
    ``inverted_residual[i] = ((expand_w, expand_act), (dw_w, dw_act), (project_w,))``, ``(None, None)`` for the
    expand of t == 1 blocks. Defaults: all 8 (``config/train/exp_1/bit_width.json``)."""
    image: int = 8
    first_conv: Tuple[int, int] = (8, 8)
    last_conv: Tuple[int, int] = (8, 8)
    fully_connected: Tuple[int, int] = (8, 8)
    shared_act: int = 8
    pooling: int = 8
    inverted_residual: Tuple = tuple(((8, 8), (8, 8), (8,)) for _ in range(N_BLOCKS))

    @staticmethod
    def qmobilenet_default() -> 'BitWidths':
        """QMobileNetV2's built-in default (mobilenet_v2.py:140-167) + QURSONetHead's 8-bit head."""
        ir = (((None, None), (3, 3), (3,)),) + tuple(((3, 3), (3, 3), (3,)) for _ in range(N_BLOCKS - 1))
        return BitWidths(8, (3, 3), (3, 3), (8, 8), 4, 8, ir)

    def block(self, i: int):
        """-> (expand_w, expand_act, dw_w, dw_act, project_w) of inverted residual i (0-based)."""
        (ew, ea), (dw, da), (pw,) = self.inverted_residual[i]
        return ew, ea, dw, da, pw

    def all_widths(self) -> List[int]:
        v = [self.image, *self.first_conv, *self.last_conv, *self.fully_connected, self.shared_act, self.pooling]
        for b in self.inverted_residual:
            v += [x for t in b for x in t if x is not None]
        return v


def parse_bit_width(path_or_dict) -> BitWidths:
    """A reference ``bit_width.json`` (path, or the dict ``load_bit_width`` returns; string values are parsed with
    ``ast.literal_eval`` like model.py:33-38) -> ``BitWidths``. Missing keys keep their 8-bit default."""
    d = path_or_dict
    if not isinstance(d, dict):
        with open(d) as f:
            d = json.load(f)
    lit = lambda x: ast.literal_eval(x) if isinstance(x, str) else x   # noqa: E731
    kw = {}
    for k in ('image', 'shared_act', 'pooling'):
        if k in d:
            kw[k] = int(lit(d[k]))
    for k in ('first_conv', 'last_conv', 'fully_connected'):
        if k in d:
            kw[k] = tuple(int(x) for x in lit(d[k]))
    if 'inverted_residual' in d:
        ir = [tuple(tuple(t) for t in lit(b)) for b in d['inverted_residual']]
        if len(ir) != N_BLOCKS:
            raise ValueError(f'inverted_residual needs {N_BLOCKS} entries, got {len(ir)}')
        kw['inverted_residual'] = tuple(ir)
    bw = BitWidths(**kw)
    check_bit_width(bw)
    return bw


def check_bit_width(path_or_dict_or_widths) -> BitWidths:
    """Validate a bit-width configuration for the int8 path: every width 3..8 (-> the parsed ``BitWidths``)."""
    bw = path_or_dict_or_widths
    if not isinstance(bw, BitWidths):
        return parse_bit_width(bw)
    bad = sorted({v for v in bw.all_widths() if not (3 <= int(v) <= 8)})
    if bad:
        raise NotImplementedError(f'bit widths {bad}: the int8 MFMA path holds 3..8-bit quantizers (1 and 2 bits '
                                  f'are Brevitas binary / ternary quantizers, quantizers.py:78-96)')
    return bw


def uint_levels(bits: int) -> int:
    """Top code of an unsigned b-bit quantizer."""
    return (1 << bits) - 1


def int_levels(bits: int) -> int:
    """Top code of a signed b-bit quantizer (the scale unit of the signed activation quantizers)."""
    return (1 << (bits - 1)) - 1


def _bn(sd, p, x):
    t = lambda n: torch.as_tensor(np.asarray(sd[f'{p}.1.{n}']), dtype=torch.float32)
    return F.batch_norm(x, t('running_mean'), t('running_var'), t('weight'), t('bias'), False, 0.1, 1e-5)


def _cbn(sd, p, x, stride, groups):
    w = torch.as_tensor(np.asarray(sd[f'{p}.0.weight']), dtype=torch.float32)
    k = w.shape[-1]
    return _bn(sd, p, F.conv2d(x, w, None, stride, (k - 1) // 2, 1, groups))


def _mse_clip(v: np.ndarray, levels: int, signed: bool) -> float:
    """The clip value c minimising the mean squared quantisation error of the values ``v`` for a quantizer with
    ``levels`` top code (scale c / levels; signed: codes down to -levels - 1), searched over c = f max|v|."""
    a = np.abs(v).max()
    if a <= 0:
        return 1e-8
    lo = -levels - 1 if signed else 0
    best, best_c = np.inf, a
    for f in np.linspace(0.05, 1.0, 96):
        sc = f * a / levels
        e = np.mean((np.clip(np.rint(v / sc), lo, levels) * sc - v) ** 2)
        if e < best:
            best, best_c = e, f * a
    return float(best_c)


@torch.no_grad()
def calibrate(sd: Dict, frames_u8: np.ndarray, percentile: float = 99.999, residual: bool = True,
              bw: Optional[BitWidths] = None, method: str = 'percentile') -> Dict:
    """Activation scales from the float model's statistics on ``frames_u8`` (B x H x W x 3 uint8), one per
    quantizer (per tensor, as Brevitas), over the top code of its bit width (``bw``, default all 8):
    ``method='percentile'`` clips at the ``percentile`` of |x|; ``'mse'`` picks the clip that minimises the
    quantisation MSE of the observed values (a common PTQ initialisation; QAT refines the scales further)."""
    bw = bw or BitWidths()
    assert method in ('percentile', 'mse')
    rng = np.random.default_rng(0)

    def amax(*ts, levels=255, signed=False):
        v = torch.cat([t.flatten() for t in ts]).numpy().astype(np.float64)
        if method == 'mse':
            if v.size > 1 << 20:
                v = rng.choice(v, 1 << 20, replace=False)
            return _mse_clip(v, levels, signed)
        return float(max(np.percentile(np.abs(v), percentile), 1e-8))

    x = torch.from_numpy(frames_u8).permute(0, 3, 1, 2).float() / 255.0
    qp: Dict = {'image': amax(x, levels=int_levels(bw.image), signed=True) / int_levels(bw.image), 'blocks': []}
    x = F.relu(_cbn(sd, f'{FP}.0', x, 2, 1))
    qp['stem'] = amax(x, levels=uint_levels(bw.first_conv[1])) / uint_levels(bw.first_conv[1])
    cin, idx = 32, 1
    for t, c, n, s in IR_SETTINGS:
        for i in range(n):
            stride = s if i == 0 else 1
            res = stride == 1 and cin == c and residual
            b: Dict[str, Optional[float]] = {'quant': None, 'expand': None}
            y, j = x, 0
            if t != 1:
                y = F.relu(_cbn(sd, f'{FP}.{idx}.conv.0', y, 1, 1))
                lv = uint_levels(bw.block(idx - 1)[1])
                b['expand'] = amax(y, levels=lv) / lv
                j = 1
            y = F.relu(_cbn(sd, f'{FP}.{idx}.conv.{j}', y, stride, y.shape[1]))
            lv = uint_levels(bw.block(idx - 1)[3])
            b['dw'] = amax(y, levels=lv) / lv
            y = _cbn(sd, f'{FP}.{idx}.conv.{j + 1}', y, 1, 1)
            if idx > 1:
                lv = int_levels(bw.shared_act)
                b['quant'] = (amax(x, y, levels=lv, signed=True) if res else amax(x, levels=lv, signed=True)) / lv
            x = x + y if res else y
            qp['blocks'].append(b)
            cin, idx = c, idx + 1
    qp['final'] = amax(x, levels=int_levels(bw.shared_act), signed=True) / int_levels(bw.shared_act)
    x = F.relu(_cbn(sd, f'{FP}.{idx}', x, 1, 1))
    qp['last'] = amax(x, levels=uint_levels(bw.last_conv[1])) / uint_levels(bw.last_conv[1])
    qp['bits'] = bw
    return qp


def validate(qp: Dict, residual: bool = True) -> None:
    arch = mobilenet_v2(residual=residual)
    assert len(qp['blocks']) == len(arch.blocks), 'one entry per inverted residual'
    for i, (b, blk) in enumerate(zip(qp['blocks'], arch.blocks)):
        assert (b['quant'] is None) == (i == 0), 'block 1 has no shared quantizer (mobilenet_v2.py:189-197)'
        assert (b['expand'] is None) == (blk.expand == 1)
    for k in ('image', 'stem', 'final', 'last'):
        assert qp[k] > 0
    if qp.get('bits') is not None:
        check_bit_width(qp['bits'])
