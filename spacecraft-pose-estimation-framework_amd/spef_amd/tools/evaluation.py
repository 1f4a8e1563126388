"""``evaluation()`` on this target: the reference's loop (src/tools/evaluation.py:36-100) -- same running
averages, same score/error records (ESA score via SPEUtils.get_score, std and median absolute deviation of the
per-image errors) -- driving any object with ``predict(images) -> (pose, latency_ms)`` (SPEMi355x)."""
from __future__ import annotations

from typing import Any, Dict, Iterable, Tuple

import numpy as np


def mad(data) -> float:
    """Median absolute deviation (evaluation.py:17-33)."""
    med = np.median(data)
    return float(np.median(np.abs(np.asarray(data) - med)))


class RunningAverage:
    """Batch-size weighted running means (src/tools/utils.py:16-60)."""

    def __init__(self, keys):
        self.tot = {k: 0.0 for k in keys}
        self.n = {k: 0 for k in keys}

    def update(self, values: Dict[str, float], batch_size: int = 1) -> None:
        for k, v in values.items():
            self.tot[k] += float(v) * batch_size
            self.n[k] += batch_size

    def get(self, k: str) -> float:
        return self.tot[k] / self.n[k] if self.n[k] else 0.0


def evaluation(spe_model: Any, dataloader: Dict[str, Iterable], spe_utils,
               split: Tuple[str, ...] = ('test', 'valid')):
    rec_score = {x: {'ori': [], 'pos': [], 'esa': []} for x in split}
    rec_error = {x: {'ori': [], 'pos': [], 'ori_std': [], 'pos_std': [], 'ori_mad': [], 'pos_mad': []} for x in split}
    for phase in split:
        error = {'ori': [], 'pos': []}
        running = RunningAverage(('esa_score', 'ori_score', 'pos_score', 'ori_error', 'pos_error'))
        for images, targets in dataloader[phase]:
            pose, _ = spe_model.predict(images['torch'])
            targets = {k: v.detach().cpu().numpy() for k, v in targets.items()}
            running.update(spe_utils.get_score(targets, pose), images['torch'].size(0))
            error['pos'].extend(np.linalg.norm(targets['pos'] - pose['pos'], axis=1))
            s = np.abs(np.sum(pose['ori'] * targets['ori'], axis=1, keepdims=True))
            s[s > 1] = 1
            error['ori'].extend((2 * np.arccos(s) * 180 / np.pi).reshape(-1))
        rec_score[phase]['ori'].append(running.get('ori_score'))
        rec_score[phase]['pos'].append(running.get('pos_score'))
        rec_score[phase]['esa'].append(running.get('esa_score'))
        rec_error[phase]['ori'].append(running.get('ori_error'))
        rec_error[phase]['pos'].append(running.get('pos_error'))
        rec_error[phase]['ori_std'].append(float(np.std(error['ori'])))
        rec_error[phase]['pos_std'].append(float(np.std(error['pos'])))
        rec_error[phase]['ori_mad'].append(mad(error['ori']))
        rec_error[phase]['pos_mad'].append(mad(error['pos']))
    return rec_score, rec_error
