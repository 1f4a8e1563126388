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
stands in for QAT. All bit widths are 8 (``config/train/exp_1/bit_width.json``); ``check_bit_width``
rejects other widths.
"""
from __future__ import annotations

import ast
import json
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from .arch import IR_SETTINGS, mobilenet_v2

FP = 'features.features'


def check_bit_width(path_or_dict) -> None:
    """Accept a reference ``bit_width.json`` (model.py:16-45 format) only if every width is 8."""
    d = path_or_dict
    if not isinstance(d, dict):
        with open(d) as f:
            d = json.load(f)
    vals: List[int] = []
    for k, v in d.items():
        items = v if k == 'inverted_residual' else [v]
        for it in items:
            x = ast.literal_eval(it) if isinstance(it, str) else it
            flat = [x] if isinstance(x, int) else [z for t in (x if isinstance(x, (list, tuple)) else [x])
                                                      for z in (t if isinstance(t, tuple) else (t,))]
            vals += [int(z) for z in flat if z is not None]
    if any(v != 8 for v in vals):
        raise NotImplementedError(f'only 8-bit Brevitas configs map to the int8 MFMA path (got {sorted(set(vals))})')


def _bn(sd, p, x):
    t = lambda n: torch.as_tensor(np.asarray(sd[f'{p}.1.{n}']), dtype=torch.float32)
    return F.batch_norm(x, t('running_mean'), t('running_var'), t('weight'), t('bias'), False, 0.1, 1e-5)


def _cbn(sd, p, x, stride, groups):
    w = torch.as_tensor(np.asarray(sd[f'{p}.0.weight']), dtype=torch.float32)
    k = w.shape[-1]
    return _bn(sd, p, F.conv2d(x, w, None, stride, (k - 1) // 2, 1, groups))


@torch.no_grad()
def calibrate(sd: Dict, frames_u8: np.ndarray, percentile: float = 99.999, residual: bool = True) -> Dict:
    """Activation scales from the float model's statistics on ``frames_u8`` (B x H x W x 3 uint8)."""
    def amax(*ts):
        v = torch.cat([t.abs().flatten() for t in ts]).numpy().astype(np.float64)
        return float(max(np.percentile(v, percentile), 1e-8))

    x = torch.from_numpy(frames_u8).permute(0, 3, 1, 2).float() / 255.0
    qp: Dict = {'image': amax(x) / 127.0, 'blocks': []}
    x = F.relu(_cbn(sd, f'{FP}.0', x, 2, 1))
    qp['stem'] = amax(x) / 255.0
    cin, idx = 32, 1
    for t, c, n, s in IR_SETTINGS:
        for i in range(n):
            stride = s if i == 0 else 1
            res = stride == 1 and cin == c and residual
            b: Dict[str, Optional[float]] = {'quant': None, 'expand': None}
            y, j = x, 0
            if t != 1:
                y = F.relu(_cbn(sd, f'{FP}.{idx}.conv.0', y, 1, 1))
                b['expand'] = amax(y) / 255.0
                j = 1
            y = F.relu(_cbn(sd, f'{FP}.{idx}.conv.{j}', y, stride, y.shape[1]))
            b['dw'] = amax(y) / 255.0
            y = _cbn(sd, f'{FP}.{idx}.conv.{j + 1}', y, 1, 1)
            if idx > 1:
                b['quant'] = (amax(x, y) if res else amax(x)) / 127.0
            x = x + y if res else y
            qp['blocks'].append(b)
            cin, idx = c, idx + 1
    qp['final'] = amax(x) / 127.0
    x = F.relu(_cbn(sd, f'{FP}.{idx}', x, 1, 1))
    qp['last'] = amax(x) / 255.0
    return qp


def validate(qp: Dict, residual: bool = True) -> None:
    arch = mobilenet_v2(residual=residual)
    assert len(qp['blocks']) == len(arch.blocks), 'one entry per inverted residual'
    for i, (b, blk) in enumerate(zip(qp['blocks'], arch.blocks)):
        assert (b['quant'] is None) == (i == 0), 'block 1 has no shared quantizer (mobilenet_v2.py:189-197)'
        assert (b['expand'] is None) == (blk.expand == 1)
    for k in ('image', 'stem', 'final', 'last'):
        assert qp[k] > 0
