"""Seeded, framework-independent synthetic weights in the reference ``state_dict`` layout.

Trained SPEF checkpoints live on Zenodo (reference ``models/README.md``) and the ImageNet download at
``src/modeling/model.py:273`` is a remote fetch, so neither exists offline. Benchmarks and parity
fixtures therefore use weights drawn here: one NumPy PCG64 stream per tensor, keyed by
``(seed, crc32(state_dict key))``, so the same tensors come out on any machine and in any order,
with no torch RNG coupling.

Initialisation follows ``ModelWrapper.__init__`` (``src/modeling/common/pytorch_layers.py:16-27``):
conv weights kaiming-normal (fan_out, gain sqrt(2)), Linear weights N(0, 0.01), biases 0.
BatchNorm statistics are *not* left at (mean 0, var 1): an untrained net with identity BN drifts in
scale through 52 convs, which tells nothing about fp16 storage on a trained net. Each BN is instead
given running statistics that normalise its conv's expected pre-activation (propagated analytically
in float64 from the weights), plus random affine terms -- the state a trained, BN-calibrated
MobileNet-V2 is in. The parity tolerance is thus exercised at realistic activation magnitudes.
"""
from __future__ import annotations

import zlib
from typing import Dict

import numpy as np

from .arch import Arch, ConvSpec, LAST_CHANNELS, mobilenet_v2


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence([seed, zlib.crc32(key.encode())])))


def _kaiming_fan_out(rng: np.random.Generator, shape) -> np.ndarray:
    # torch.nn.init.kaiming_normal_(mode='fan_out'): std = sqrt(2) / sqrt(out * kh * kw)
    fan_out = shape[0] * shape[2] * shape[3]
    return rng.standard_normal(shape) * (np.sqrt(2.0) / np.sqrt(fan_out))


def _conv_bn(sd: Dict[str, np.ndarray], c: ConvSpec, seed: int, m_in: float) -> float:
    """Draw conv + BN params for one ConvBnAct; return the output second moment estimate."""
    w = _kaiming_fan_out(_rng(seed, f'{c.prefix}.0.weight'), c.weight_shape)
    # expected pre-activation variance per output channel: E[x^2] * sum_k w_k^2
    v = m_in * np.sum(w.reshape(c.cout, -1) ** 2, axis=1)
    r = _rng(seed, f'{c.prefix}.1')
    gamma = r.uniform(0.6, 1.4, c.cout)
    beta = r.normal(0.0, 0.15, c.cout)
    mean = r.normal(0.0, 0.1, c.cout) * np.sqrt(v)
    var = v * r.uniform(0.7, 1.4, c.cout)
    sd[f'{c.prefix}.0.weight'] = w
    sd[f'{c.prefix}.1.weight'] = gamma
    sd[f'{c.prefix}.1.bias'] = beta
    sd[f'{c.prefix}.1.running_mean'] = mean
    sd[f'{c.prefix}.1.running_var'] = var
    sd[f'{c.prefix}.1.num_batches_tracked'] = np.array(0, dtype=np.int64)
    m_out = float(np.mean(gamma ** 2 / 1.0 + beta ** 2))
    return 0.5 * m_out if c.relu else m_out


def synthetic_state_dict(arch: Arch | None = None, seed: int = 1001, head_std: float = 0.01,
                         input_m2: float = 0.1, pos_std: float | None = None,
                         pos_bias=None) -> Dict[str, np.ndarray]:
    """Return ``{reference key: float32 ndarray}`` (num_batches_tracked as int64 scalars).

    ``head_std`` is the orientation (or keypoint) Linear's weight std (the reference init is 0.01,
    pytorch_layers.py:25-27); ``pos_std`` the position Linear's (default: ``head_std``); ``pos_bias`` an
    optional position bias vector, e.g. a SPEED-range offset (0.3, -0.2, 12.0) m for regression heads."""
    arch = arch or mobilenet_v2()
    sd: Dict[str, np.ndarray] = {}
    m = _conv_bn(sd, arch.stem, seed, input_m2)
    for b in arch.blocks:
        m_blk = m
        for c in b.convs:
            m = _conv_bn(sd, c, seed, m)
        if b.residual:
            m = m + m_blk
    _conv_bn(sd, arch.last, seed, m)
    if arch.head == 'ursonet':
        for name, n, std in (('head.pos.0', arch.n_pos, head_std if pos_std is None else pos_std),
                             ('head.ori.1', arch.n_ori, head_std)):
            sd[f'{name}.weight'] = _rng(seed, f'{name}.weight').normal(0.0, std, (n, LAST_CHANNELS))
            sd[f'{name}.bias'] = np.zeros(n)
        if pos_bias is not None:
            sd['head.pos.0.bias'] = np.asarray(pos_bias, np.float64).reshape(arch.n_pos)
    else:
        sd['head.layer.1.weight'] = _rng(seed, 'head.layer.1.weight').normal(0.0, head_std,
                                                                             (arch.n_kp, 122880))
        sd['head.layer.1.bias'] = np.zeros(arch.n_kp)
    return {k: (v.astype(np.float32) if v.dtype != np.int64 else v) for k, v in sd.items()}


def plant_keypoint_head(sd: Dict[str, np.ndarray], kp_norm: np.ndarray) -> Dict[str, np.ndarray]:
    """A keypoint-regression head (head/keypoints.py:10-27) whose sigmoid outputs are real keypoints: the head bias
    becomes logit() of ``kp_norm`` (one frame's normalised keypoints, origin first, as KeyPoints.project returns them,
    spe/keypoints_utils.py:47-110), so with small head weights every frame's keypoints spread over the spacecraft's
    image as in the reference's keypoint mode instead of clustering where a random head puts them (an ill-conditioned
    EPnP input). Returns ``sd`` with the bias replaced."""
    k = np.clip(np.asarray(kp_norm, np.float64).reshape(-1), 1e-6, 1 - 1e-6)
    assert sd['head.layer.1.bias'].shape == k.shape, (sd['head.layer.1.bias'].shape, k.shape)
    sd['head.layer.1.bias'] = np.log(k / (1 - k)).astype(np.float32)
    return sd


def state_dict_digest(sd: Dict[str, np.ndarray]) -> str:
    """sha256 over keys and float32 bytes in key order -- pins the generator in the fixtures."""
    import hashlib
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k]).tobytes())
    return h.hexdigest()
