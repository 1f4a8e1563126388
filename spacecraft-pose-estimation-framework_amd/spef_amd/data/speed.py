"""SPEED / SPEED+ dataset reader for evaluation on this target (src/data/utils.py:170-249 layout).

Reads ``images/<split>/<filename>`` + the split JSON (pose keys as the reference accepts them,
utils.py:194-196), decodes frames with Pillow to RGB uint8 (utils.py:215), and yields RAW frames: the resize
(``transforms.Resize(img_size)``) runs on the GPU in ``SPEMi355x.predict_frames`` (bit-identical to Pillow).
No dataset ships with this environment; tests use ``data.synthetic``.
"""
from __future__ import annotations

import json
import os
from typing import Iterator

import numpy as np


def _key(d, names):
    for n in names:
        if n in d:
            return n
    raise KeyError(f'none of {names} in the labels')


def speed_frames(images_path: str, labels_path: str, batch: int) -> Iterator:
    """Yields (frames uint8 [B, H, W, 3] tensor, {'ori': [B, 4], 'pos': [B, 3]} tensors), sorted by image
    number like SPEDataset (utils.py:202)."""
    import re

    import torch
    from PIL import Image
    with open(labels_path) as f:
        labels = json.load(f)
    ok, pk = _key(labels[0], ['q', 'q_vbs2tango', 'q_vbs2tango_true']), _key(labels[0], ['t', 'r_Vo2To_vbs_true'])
    labels.sort(key=lambda t: int(re.sub(r'[^0-9]', '', t['filename']) or 0))
    for i in range(0, len(labels), batch):
        chunk = labels[i:i + batch]
        fr = np.stack([np.asarray(Image.open(os.path.join(images_path, t['filename'])).convert('RGB'))
                       for t in chunk])
        yield torch.from_numpy(fr), {'ori': torch.tensor([t[ok] for t in chunk], dtype=torch.float32),
                                     'pos': torch.tensor([t[pk] for t in chunk], dtype=torch.float32)}
