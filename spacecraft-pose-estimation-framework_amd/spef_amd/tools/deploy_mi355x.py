"""Deploy a built experiment on an MI355X and evaluate it (the analogue of deploy_nvidia.py / deploy_tvm.py).

    python -m spef_amd.tools.deploy_mi355x --build experiments/build/mi355x/<name> [--data PATH | --synthetic N]

Loads ``model.spef`` + ``config.yaml``, builds SPEUtils as eval.py:29-33 does, runs ``evaluation()``
(src/tools/evaluation.py:36-100) on the SPEED split JSONs under ``--data`` (raw frames; resize on the GPU) or on
N synthetic batches, then the throughput test ``predict(img, num_predict=NUM_PREDICT)`` (deploy_nvidia.py:91-95).
Writes ``on_board/{score.json, latency_ms.json}`` next to the build.
"""
from __future__ import annotations

import argparse
import json
import os
import sys


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--build', required=True)
    ap.add_argument('--data', help='SPEED dataset root (images/, valid.json, real.json)')
    ap.add_argument('--synthetic', type=int, default=2, help='synthetic batches when --data is absent')
    ap.add_argument('--num-predict', type=int)
    a = ap.parse_args(argv)
    import torch
    from ..config import load_config, to_spe_utils
    from ..data.synthetic import speed_like_loader
    from ..spe.camera import CAMERAS
    from ..spe_mi355x import SPEMi355x
    from .evaluation import evaluation

    cfg = load_config(os.path.join(a.build, 'config.yaml'))
    dev = torch.device(f'cuda:{cfg.MI355X.DEVICE}')
    camera = CAMERAS['speed_plus' if 'plus' in cfg.DATA.PATH else 'speed']
    su = to_spe_utils(cfg, camera)
    spe = SPEMi355x(os.path.join(a.build, 'model.spef'), dev, su)
    B, size = cfg.MI355X.BATCH_SIZE, tuple(cfg.DATA.IMG_SIZE)

    if a.data:
        from ..data.speed import speed_frames

        class _Resized:   # raw frames -> on-device Resize -> the pose dict (predict_frames)
            def __init__(self, it):
                self.it = it

            def __iter__(self):
                for fr, tgt in self.it:
                    yield {'torch': spe.engine.preprocess(fr.to(dev).contiguous(), size)}, tgt
        loaders = {s: _Resized(speed_frames(os.path.join(a.data, 'images', 'train' if s == 'valid' else s),
                                            os.path.join(a.data, f'{s}.json'), B)) for s in ('valid', 'real')}
        splits = tuple(s for s in ('valid', 'real') if os.path.exists(os.path.join(a.data, f'{s}.json')))
    else:
        loaders = {'synthetic': speed_like_loader(a.synthetic, B, size)}
        splits = ('synthetic',)
    score, error = evaluation(spe, loaders, su, splits)

    img, _ = next(iter(speed_like_loader(1, B, size)))
    n = a.num_predict or cfg.MI355X.NUM_PREDICT
    _, lat = spe.predict(img['torch'], num_predict=n)
    out = os.path.join(a.build, 'on_board')
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, 'score.json'), 'w') as f:
        json.dump({'score': score, 'error': error}, f, indent=1)
    rec = {'mi355x': [lat], 'batch': B, 'img_size': list(size), 'images_per_sec': B / lat * 1e3, 'num_predict': n}
    with open(os.path.join(out, 'latency_ms.json'), 'w') as f:
        json.dump(rec, f, indent=1)
    print(f'MI355X = {lat:.3f} ms per batch of {B} ({rec["images_per_sec"]:.0f} img/s)')
    spe.close()
    return 0


if __name__ == '__main__':
    sys.exit(main())
