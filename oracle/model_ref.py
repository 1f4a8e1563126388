"""Float32 CPU restatement of the reference forward pass (ORACLE -- test infrastructure only).

Follows, op for op and in the same order (so it is bit-identical to the reference on CPU):
  * ``ConvBnAct``          src/modeling/common/pytorch_layers.py:35-62
                           conv(bias=False, padding=(k-1)//2) -> BatchNorm2d(eps=1e-5, eval) -> ReLU
  * ``InvertedResidual``   src/modeling/common/pytorch_layers.py:65-98
                           [expand 1x1 if t != 1] -> dw 3x3 (groups=hidden, stride) -> project 1x1 (no act);
                           ``x + conv(x)`` when stride == 1 and cin == cout (:71, :93-96)
  * ``MobileNetV2``        src/modeling/backbone/mobilenet_v2.py:232-271 (settings :240-249)
  * ``URSONetHead``        src/modeling/head/ursonet.py:27-33 -- mean([2,3]); ori = Linear(Dropout(x))
                           (Dropout is identity in eval); pos = Linear(x)
  * ``KeypointRegressionHead`` src/modeling/head/keypoints.py:24-27 -- flatten(NCHW) -> Linear
  * ``SPETorch.predict``   src/spe/spe_torch.py:57-61 -- the forward under ``torch.no_grad()``
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np
import torch
import torch.nn.functional as F

_IR = ((1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2), (6, 320, 1, 1))


def _t(sd, k):
    v = sd[k]
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))


def _conv_bn_act(x, sd, prefix, stride, groups, act):
    w = _t(sd, f'{prefix}.0.weight')
    k = w.shape[-1]
    x = F.conv2d(x, w, None, stride, (k - 1) // 2, 1, groups)
    x = F.batch_norm(x, _t(sd, f'{prefix}.1.running_mean'), _t(sd, f'{prefix}.1.running_var'),
                     _t(sd, f'{prefix}.1.weight'), _t(sd, f'{prefix}.1.bias'), False, 0.1, 1e-5)
    return F.relu(x) if act else x


def backbone(x: torch.Tensor, sd: Dict, residual: bool = True, upto: int | None = None) -> torch.Tensor:
    """features(x): ``B x 3 x H x W`` float32 in [0,1] -> ``B x 1280 x H/32 x W/32``.
    ``upto`` stops after ``features.features[upto]`` (block-boundary activations for debugging)."""
    fp = 'features.features'
    x = _conv_bn_act(x, sd, f'{fp}.0', 2, 1, True)
    if upto == 0:
        return x
    cin, idx = 32, 1
    for t, c, n, s in _IR:
        for i in range(n):
            stride = s if i == 0 else 1
            hidden = int(round(cin * t))
            y, j = x, 0
            if t != 1:
                y = _conv_bn_act(y, sd, f'{fp}.{idx}.conv.{j}', 1, 1, True)
                j += 1
            y = _conv_bn_act(y, sd, f'{fp}.{idx}.conv.{j}', stride, hidden, True)
            y = _conv_bn_act(y, sd, f'{fp}.{idx}.conv.{j + 1}', 1, 1, False)
            x = x + y if (stride == 1 and cin == c and residual) else y
            if upto == idx:
                return x
            cin, idx = c, idx + 1
    return _conv_bn_act(x, sd, f'{fp}.{idx}', 1, 1, True)


def ursonet_head(f: torch.Tensor, sd: Dict) -> Tuple[torch.Tensor, torch.Tensor]:
    x = f.mean([2, 3])
    ori = F.linear(x, _t(sd, 'head.ori.1.weight'), _t(sd, 'head.ori.1.bias'))
    pos = F.linear(x, _t(sd, 'head.pos.0.weight'), _t(sd, 'head.pos.0.bias'))
    return ori, pos


def keypoint_head(f: torch.Tensor, sd: Dict) -> torch.Tensor:
    return F.linear(torch.flatten(f, start_dim=1), _t(sd, 'head.layer.1.weight'), _t(sd, 'head.layer.1.bias'))


@torch.no_grad()
def forward(images: torch.Tensor, sd: Dict, head: str = 'ursonet', residual: bool = True):
    """ModelWrapper.forward (pytorch_layers.py:29-32) on float32 NCHW images in [0,1]."""
    f = backbone(images.float(), sd, residual)
    return ursonet_head(f, sd) if head == 'ursonet' else keypoint_head(f, sd)


def u8_nhwc_to_nchw_f32(frames_u8: np.ndarray) -> torch.Tensor:
    """The reference input contract: ToTensor() of an RGB uint8 image (src/data/utils.py:212-249,
    datasets/speed.py:66-69) = HWC uint8 -> CHW float32 / 255 (no mean/std normalisation)."""
    x = torch.from_numpy(np.ascontiguousarray(frames_u8)).permute(0, 3, 1, 2).float()
    return x.div(255.0)
