"""MobileNet-V2 + URSONet / keypoint head topology, expressed as data.

This is the architecture the reference builds in
``src/modeling/backbone/mobilenet_v2.py:232-271`` (``MobileNetV2``; settings table at :240-249,
stem at :252-254, inverted residuals at :257-262, last 1x1 conv at :264) out of
``src/modeling/common/pytorch_layers.py:35-98`` (``ConvBnAct`` / ``InvertedResidual``) and the heads
``src/modeling/head/ursonet.py:10-33`` (``URSONetHead``) and ``src/modeling/head/keypoints.py:10-27``
(``KeypointRegressionHead``).

The table is used by the blob builder (BN fold + pack), by the synthetic weight generator, and by the
FLOP counter that prices ``roofline.achieved``. Parameter names follow the reference ``state_dict``
layout exactly (316 keys for the URSONet head), so a reference ``parameters.pt`` loads unchanged.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

# (t, c, n, s) -- src/modeling/backbone/mobilenet_v2.py:240-249
IR_SETTINGS = (
    (1, 16, 1, 1),
    (6, 24, 2, 2),
    (6, 32, 3, 2),
    (6, 64, 4, 2),
    (6, 96, 3, 1),
    (6, 160, 3, 2),
    (6, 320, 1, 1),
)
STEM_CHANNELS = 32          # mobilenet_v2.py:237 (input_channel = 32)
LAST_CHANNELS = 1280        # mobilenet_v2.py:232 (out_channels=1280)
BN_EPS = 1e-5               # torch.nn.BatchNorm2d default, pytorch_layers.py:56


@dataclass
class ConvSpec:
    """One ``ConvBnAct`` (conv, BN(eps 1e-5), optional ReLU) -- pytorch_layers.py:35-62."""
    prefix: str               # state_dict prefix, e.g. 'features.features.2.conv.0'
    cin: int
    cout: int
    k: int                    # kernel size (1 or 3)
    stride: int
    groups: int               # 1 or cout (depthwise)
    relu: bool

    @property
    def weight_shape(self) -> Tuple[int, int, int, int]:
        return (self.cout, self.cin // self.groups, self.k, self.k)

    def macs(self, h_out: int, w_out: int) -> int:
        """MACs exactly as nn_stats.py:31-41 counts a Conv2d."""
        return self.cout * (self.cin // self.groups) * self.k * self.k * h_out * w_out


@dataclass
class BlockSpec:
    """One ``InvertedResidual`` -- pytorch_layers.py:65-98."""
    index: int                # position in features.features (1..17)
    cin: int
    cout: int
    stride: int
    expand: int               # t
    hidden: int
    residual: bool            # stride == 1 and cin == cout (pytorch_layers.py:71)
    convs: List[ConvSpec] = field(default_factory=list)   # [expand?], dw, project


@dataclass
class Arch:
    stem: ConvSpec
    blocks: List[BlockSpec]
    last: ConvSpec
    head: str                 # 'ursonet' | 'keypoints'
    n_ori: int                # URSONet orientation outputs (bins or 4)
    n_pos: int                # URSONet position outputs (3 or bins)
    n_kp: int = 24            # keypoint head outputs

    def all_convs(self) -> List[ConvSpec]:
        out = [self.stem]
        for b in self.blocks:
            out.extend(b.convs)
        out.append(self.last)
        return out


def mobilenet_v2(head: str = 'ursonet', n_ori: int = 1728, n_pos: int = 3,
                 residual: bool = True, n_kp: int = 24) -> Arch:
    """Build the topology of ``ModelWrapper(MobileNetV2(3, 1280), head)``.

    ``residual`` mirrors ``MODEL.BACKBONE.RESIDUAL`` (``residual_connections``, mobilenet_v2.py:233).
    """
    assert head in ('ursonet', 'keypoints')
    fp = 'features.features'
    stem = ConvSpec(f'{fp}.0', 3, STEM_CHANNELS, 3, 2, 1, True)
    blocks: List[BlockSpec] = []
    cin = STEM_CHANNELS
    idx = 1
    for t, c, n, s in IR_SETTINGS:
        for i in range(n):
            stride = s if i == 0 else 1
            hidden = int(round(cin * t))
            use_res = stride == 1 and cin == c and residual
            b = BlockSpec(idx, cin, c, stride, t, hidden, use_res)
            j = 0
            if t != 1:
                b.convs.append(ConvSpec(f'{fp}.{idx}.conv.{j}', cin, hidden, 1, 1, 1, True))
                j += 1
            b.convs.append(ConvSpec(f'{fp}.{idx}.conv.{j}', hidden, hidden, 3, stride, hidden, True))
            j += 1
            b.convs.append(ConvSpec(f'{fp}.{idx}.conv.{j}', hidden, c, 1, 1, 1, False))
            blocks.append(b)
            cin = c
            idx += 1
    last = ConvSpec(f'{fp}.{idx}', cin, LAST_CHANNELS, 1, 1, 1, True)
    return Arch(stem, blocks, last, head, n_ori, n_pos, n_kp)


def conv_out(h: int, k: int, s: int) -> int:
    p = (k - 1) // 2          # pytorch_layers.py:51
    return (h + 2 * p - k) // s + 1


def feature_hw(h: int, w: int) -> Tuple[int, int]:
    """Spatial size of the 1280-channel feature map for an h x w input (5 stride-2 stages)."""
    arch = mobilenet_v2()
    for c in arch.all_convs():
        if c.k == 3:
            h, w = conv_out(h, 3, c.stride), conv_out(w, 3, c.stride)
    return h, w


def count_macs(arch: Arch, h: int, w: int) -> dict:
    """Per-image MACs by layer family, counted the way nn_stats.py:31-41 counts them
    (Conv2d: Cout*Cin/g*k*k*Hout*Wout; Linear: in*out; BN/ReLU/add/mean excluded)."""
    out = {'stem': 0, 'pointwise': 0, 'depthwise': 0, 'head': 0}
    hh, ww = h, w
    for c in arch.all_convs():
        ho, wo = conv_out(hh, c.k, c.stride), conv_out(ww, c.k, c.stride)
        m = c.macs(ho, wo)
        if c is arch.stem:
            out['stem'] += m
        elif c.groups > 1:
            out['depthwise'] += m
        else:
            out['pointwise'] += m
        hh, ww = ho, wo
    if arch.head == 'ursonet':
        out['head'] = LAST_CHANNELS * (arch.n_ori + arch.n_pos)
    else:
        out['head'] = LAST_CHANNELS * hh * ww * arch.n_kp
    out['total'] = sum(out.values())
    return out


def flops_per_image(h: int = 512, w: int = 512, n_ori: int = 1728, n_pos: int = 3,
                    head: str = 'ursonet') -> int:
    """Algorithmic FLOPs per image (2 x MACs incl. head), the unit roofline.achieved is priced in."""
    return 2 * count_macs(mobilenet_v2(head, n_ori, n_pos), h, w)['total']


def state_dict_shapes(arch: Arch) -> dict:
    """Reference state_dict key -> shape (pytorch_layers.py / ursonet.py / keypoints.py naming)."""
    shapes = {}
    for c in arch.all_convs():
        shapes[f'{c.prefix}.0.weight'] = c.weight_shape
        for nm in ('weight', 'bias', 'running_mean', 'running_var'):
            shapes[f'{c.prefix}.1.{nm}'] = (c.cout,)
        shapes[f'{c.prefix}.1.num_batches_tracked'] = ()
    if arch.head == 'ursonet':
        shapes['head.pos.0.weight'] = (arch.n_pos, LAST_CHANNELS)
        shapes['head.pos.0.bias'] = (arch.n_pos,)
        shapes['head.ori.1.weight'] = (arch.n_ori, LAST_CHANNELS)
        shapes['head.ori.1.bias'] = (arch.n_ori,)
    else:
        # keypoints.py:20 -- hard-wired 122880 = 1280*8*12 (240x384 input)
        shapes['head.layer.1.weight'] = (arch.n_kp, 122880)
        shapes['head.layer.1.bias'] = (arch.n_kp,)
    return shapes


def arch_from_state_dict(sd, residual: bool = True) -> Arch:
    """Topology of a reference state_dict (``model.py:261-266`` layout): head type and widths from the head
    keys (``head/ursonet.py:17-25`` -> ``head.ori.1`` / ``head.pos.0``; ``head/keypoints.py:20`` ->
    ``head.layer.1``). ``residual`` is ``MODEL.BACKBONE.RESIDUAL`` (not recoverable from the weights)."""
    if 'head.layer.1.weight' in sd:
        return mobilenet_v2('keypoints', residual=residual, n_kp=int(sd['head.layer.1.weight'].shape[0]))
    if 'head.ori.1.weight' in sd and 'head.pos.0.weight' in sd:
        return mobilenet_v2('ursonet', int(sd['head.ori.1.weight'].shape[0]), int(sd['head.pos.0.weight'].shape[0]),
                            residual=residual)
    raise AssertionError('state_dict has neither a URSONet nor a keypoint-regression head')
