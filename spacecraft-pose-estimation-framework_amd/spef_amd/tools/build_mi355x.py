"""Build an experiment for the MI355X target (the analogue of build_nvidia.py / build_tvm.py).

    python -m spef_amd.tools.build_mi355x --experiment experiments/train/<name> [--dtype fp16|bf16|int8]
    python -m spef_amd.tools.build_mi355x --synthetic --out experiments/build/mi355x/synthetic

Reads ``config.yaml`` + ``model/parameters.pt`` (+ ``model/bit_width.json`` for quantized models) of a
reference training experiment (eval.py:20-27 layout; the checkpoint is loaded with ``weights_only=True``),
folds BN and packs the weight blob (fp16/bf16, or int8 with activation scales calibrated on frames), and writes
``experiments/build/mi355x/<name>/{model.spef, config.yaml, build.json}``.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time


def build(sd, cfg, out_dir: str, dtype: str, calib_frames=None, bit_width=None) -> dict:
    """``bit_width``: the experiment's bit_width.json as quant.BitWidths (int8 only; None = all 8 bits)."""
    from .. import blob as Bl
    from ..arch import arch_from_state_dict
    os.makedirs(out_dir, exist_ok=True)
    arch = arch_from_state_dict(sd, residual=cfg.MODEL.BACKBONE.RESIDUAL)
    t0 = time.time()
    if dtype == 'int8':
        from ..blob_q8 import pack_int8
        from ..quant import calibrate
        assert calib_frames is not None, 'int8 builds calibrate activation scales on frames'
        qp = calibrate(sd, calib_frames, residual=cfg.MODEL.BACKBONE.RESIDUAL, bw=bit_width)
        blob = pack_int8(sd, qp, arch)
        import dataclasses
        with open(os.path.join(out_dir, 'qparams.json'), 'w') as f:
            json.dump(dict(qp, bits=dataclasses.asdict(qp['bits'])), f, indent=1)
    else:
        blob = Bl.pack(sd, arch, dtype=dtype)
    with open(os.path.join(out_dir, 'model.spef'), 'wb') as f:
        f.write(blob)
    cfg.MI355X.DTYPE = dtype
    from ..config import save_config
    save_config(cfg, os.path.join(out_dir, 'config.yaml'))
    info = {'dtype': dtype, 'bytes': len(blob), 'sha256': hashlib.sha256(blob).hexdigest(), 'head': arch.head,
            'n_ori': arch.n_ori, 'n_pos': arch.n_pos, 'pack_seconds': round(time.time() - t0, 3)}
    with open(os.path.join(out_dir, 'build.json'), 'w') as f:
        json.dump(info, f, indent=1)
    return info


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--experiment', help='reference experiment dir with config.yaml and model/parameters.pt')
    ap.add_argument('--synthetic', action='store_true', help='seeded synthetic weights (no checkpoint offline)')
    ap.add_argument('--dtype', choices=['fp16', 'bf16', 'int8'])
    ap.add_argument('--out')
    a = ap.parse_args(argv)
    import torch
    from ..config import load_config
    from ..data.synthetic import synth_frames
    if a.experiment:
        cfg = load_config(os.path.join(a.experiment, 'config.yaml'))
        sd = torch.load(os.path.join(a.experiment, 'model', 'parameters.pt'), map_location='cpu', weights_only=True)
        bit_width = None
        bw_path = os.path.join(a.experiment, 'model', 'bit_width.json')
        if os.path.exists(bw_path):
            from ..quant import parse_bit_width
            bit_width = parse_bit_width(bw_path)
        name = os.path.basename(os.path.normpath(a.experiment))
    elif a.synthetic:
        bit_width = None
        from ..arch import mobilenet_v2
        from ..weights import synthetic_state_dict
        cfg = load_config(None)
        h = cfg.MODEL.HEAD
        from ..spe.spe_utils import SPEUtils
        su = SPEUtils(None, h.ORI, h.N_ORI_BINS_PER_DIM, cfg.DATA.ORI_SMOOTH_FACTOR, h.ORI_DELETE_UNUSED_BINS, h.POS,
                      h.N_POS_BINS_PER_DIM, cfg.DATA.POS_SMOOTH_FACTOR)
        n_ori = su.orientation.n_bins if h.ORI == 'classification' else 4
        n_pos = su.position.n_bins if h.POS == 'classification' else 3
        sd = synthetic_state_dict(mobilenet_v2('ursonet', n_ori, n_pos), seed=1001)
        name = 'synthetic'
    else:
        ap.error('--experiment or --synthetic')
    dtype = a.dtype or cfg.MI355X.DTYPE
    out = a.out or os.path.join('experiments', 'build', 'mi355x', name)
    calib = synth_frames(cfg.MI355X.CALIB_FRAMES, *cfg.DATA.IMG_SIZE, 900) if dtype == 'int8' else None
    info = build(sd, cfg, out, dtype, calib, bit_width)
    print(json.dumps(info))
    return 0


if __name__ == '__main__':
    sys.exit(main())
