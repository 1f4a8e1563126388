"""Synthetic SPEED-style inputs (no dataset is available offline).

Frames: uint8 HWC, grayscale replicated to RGB (src/data/utils.py:215) -- dark background, sensor noise and a
bright target -- generated per frame from (seed, global frame index), so any shard of a global batch is
reproducible on its own rank. Poses follow the D-SPEED sampler (create_dspeed.py:69-82): z ~ U(3, 35),
x, y ~ U(-0.3 z, 0.3 z), orientation uniform on SO(3).
"""
from __future__ import annotations

from typing import Iterator, Tuple

import numpy as np


def synth_frames(b: int, h: int, w: int, first_index: int, seed: int = 1001) -> np.ndarray:
    out = np.empty((b, h, w, 3), np.uint8)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    for i in range(b):
        rng = np.random.Generator(np.random.PCG64([seed, first_index + i]))
        cy, cx = rng.uniform(0.25, 0.75) * h, rng.uniform(0.25, 0.75) * w
        r = rng.uniform(0.05, 0.25) * min(h, w)
        g = 200.0 * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * r * r))
        g += 30.0 * np.sin(xx / rng.uniform(2, 8)) * (g > 20)
        g += rng.normal(8.0, 2.0, (h, w)).astype(np.float32)
        out[i] = np.clip(g, 0, 255).astype(np.uint8)[..., None]
    return out


def synth_poses(b: int, first_index: int, seed: int = 1001) -> Tuple[np.ndarray, np.ndarray]:
    """-> (ori B x 4 scalar-first unit quaternions, pos B x 3 metres), D-SPEED ranges."""
    ori = np.empty((b, 4), np.float32)
    pos = np.empty((b, 3), np.float32)
    for i in range(b):
        rng = np.random.Generator(np.random.PCG64([seed, 7, first_index + i]))
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        ori[i] = q * (1 if q[0] >= 0 else -1)
        z = rng.uniform(3.0, 35.0)
        pos[i] = (rng.uniform(-0.3 * z, 0.3 * z), rng.uniform(-0.3 * z, 0.3 * z), z)
    return ori, pos


def speed_like_loader(n_batches: int, batch: int, size, seed: int = 1001) -> Iterator:
    """Yields (images {'torch': uint8 NHWC tensor}, targets {'ori', 'pos'} tensors) like the reference
    DataLoader (utils.py:235-249) -- frames already at ``size`` (H, W)."""
    import torch
    h, w = size
    for k in range(n_batches):
        fr = synth_frames(batch, h, w, k * batch, seed)
        ori, pos = synth_poses(batch, k * batch, seed)
        yield {'torch': torch.from_numpy(fr)}, {'ori': torch.from_numpy(ori), 'pos': torch.from_numpy(pos)}
