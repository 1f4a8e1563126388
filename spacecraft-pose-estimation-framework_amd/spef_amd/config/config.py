"""YAML config loader mirroring the reference's yacs defaults (src/config/train/config.py:4-42).

Same keys, same defaults, same validation (ORI/POS modes, keypoints on both or neither). Like yacs'
``merge_from_file``, a YAML key that is not in the defaults is an error, and a value must keep the default's
type (tuples and lists interchange). The ``MI355X`` section is this target's build/deploy settings, the analogue
of the reference's src/config/build/nvidia / tvm configs.
"""
from __future__ import annotations

import copy
import os
from typing import Any, Dict

import yaml

DEFAULTS: Dict[str, Any] = {
    'MODEL': {
        'PRETRAINED_PATH': 'models/fp32_12bins_model.pt',
        'MANUAL_COPY': True,
        'QUANTIZATION': False,
        'BACKBONE': {'NAME': 'mobilenet_v2_pytorch', 'RESIDUAL': True},
        'HEAD': {'NAME': 'ursonet_pytorch', 'ORI': 'classification', 'POS': 'regression',
                 'N_ORI_BINS_PER_DIM': 12, 'N_POS_BINS_PER_DIM': 10, 'ORI_DELETE_UNUSED_BINS': False,
                 'KEYPOINTS_PATH': 'models/3d_models/tangoPoints.mat'},
    },
    'DATA': {'BATCH_SIZE': 8, 'PATH': '../datasets/speed', 'IMG_SIZE': (240, 384), 'ORI_SMOOTH_FACTOR': 3,
             'POS_SMOOTH_FACTOR': 100, 'ROT_AUGMENT': True, 'OTHER_AUGMENT': True, 'SHUFFLE': True},
    'TRAIN': {'N_EPOCH': 2, 'LR': 0.01, 'OPTIM': 'SGD', 'MOMENTUM': 0.9, 'DECAY': 0.0, 'SCHEDULER': 'MultiStepLR',
              'MILESTONES': (7, 20), 'GAMMA': 0.1, 'CLIP_BATCHNORM': False},
    # this target: weight storage / arithmetic type (fp16mx | fp16x2 | fp16 | bf16 | int8 | fp32), device, batch,
    # throughput loop length. fp16mx (the default) holds the north star's absolute bound at trained-scale heads.
    'MI355X': {'DTYPE': 'fp16mx', 'DEVICE': 0, 'BATCH_SIZE': 64, 'NUM_PREDICT': 1000, 'CALIB_FRAMES': 16},
}


class Config(dict):
    """dict with attribute access (cfg.MODEL.HEAD.ORI), like yacs' CfgNode."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def _wrap(d):
    return Config({k: _wrap(v) if isinstance(v, dict) else v for k, v in d.items()})


def _merge(base: dict, new: dict, path: str = '') -> None:
    for k, v in new.items():
        full = f'{path}{k}'
        if k not in base:
            raise KeyError(f'Non-existent config key: {full}')
        if isinstance(base[k], dict):
            if not isinstance(v, dict):
                raise ValueError(f'{full} must be a mapping')
            _merge(base[k], v, full + '.')
            continue
        d = base[k]
        if isinstance(d, (tuple, list)) and isinstance(v, (tuple, list)):
            v = tuple(v) if isinstance(d, tuple) else list(v)
        elif d is not None and v is not None and not isinstance(v, type(d)) and \
                not (isinstance(d, float) and isinstance(v, int)):
            raise ValueError(f'Type mismatch for {full}: {type(d).__name__} default, got {type(v).__name__}')
        base[k] = v


def load_config(path: str | None = None) -> Config:
    cfg = copy.deepcopy(DEFAULTS)
    if path is not None:
        assert os.path.isfile(path), f'File {path} does not exist'
        with open(path) as f:
            _merge(cfg, yaml.safe_load(f) or {})
    h = cfg['MODEL']['HEAD']
    assert h['ORI'] in ('classification', 'regression', 'keypoints')
    assert h['POS'] in ('classification', 'regression', 'keypoints')
    if h['ORI'] == 'keypoints' or h['POS'] == 'keypoints':
        assert h['ORI'] == 'keypoints' and h['POS'] == 'keypoints', \
            "Both ORI and POS must be 'keypoints' if one is 'keypoints'"
    assert cfg['MI355X']['DTYPE'] in ('fp16mx', 'fp16', 'bf16', 'int8', 'fp32', 'fp16x2')
    return _wrap(cfg)


def save_config(cfg: dict, path: str) -> None:
    assert os.path.exists(os.path.dirname(os.path.abspath(path))), f'Path {path} does not exist'

    def plain(d):
        return {k: plain(v) if isinstance(v, dict) else (list(v) if isinstance(v, tuple) else v) for k, v in d.items()}
    with open(path, 'w') as f:
        yaml.safe_dump(plain(cfg), f, sort_keys=True)


def to_spe_utils(cfg: Config, camera=None, keypoints=None):
    """SPEUtils(...) exactly as eval.py:29-33 builds it from the config."""
    from ..spe.spe_utils import SPEUtils
    h, d = cfg.MODEL.HEAD, cfg.DATA
    kp = keypoints if keypoints is not None else (h.KEYPOINTS_PATH if h.ORI == 'keypoints' else None)
    return SPEUtils(camera, h.ORI, h.N_ORI_BINS_PER_DIM, d.ORI_SMOOTH_FACTOR, h.ORI_DELETE_UNUSED_BINS, h.POS,
                    h.N_POS_BINS_PER_DIM, d.POS_SMOOTH_FACTOR, kp)
