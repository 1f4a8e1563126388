"""Outputs of one library build (SPEF_LIB) for bit-identity checks between builds (GPU box):
python tools/lib_cmp.py <dtype> <out.npz> -- URSONet 512x512 B=64 logits and keypoint-mode 240x384 B=64 raw outputs.
Compare two files with: python tools/lib_cmp.py --cmp a.npz b.npz"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd')]

import numpy as np


def main():
    if sys.argv[1] == '--cmp':
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        for k in a.files:
            d = np.abs(a[k] - b[k]).max()
            print(k, 'bit-identical' if np.array_equal(a[k], b[k]) else f'max |diff| {d:.3e}')
        return
    import torch
    from spef_amd import blob as Bl
    from spef_amd.arch import mobilenet_v2
    from spef_amd.engine import Engine
    from spef_amd.weights import synthetic_state_dict
    dt, out = sys.argv[1], sys.argv[2]
    rng = np.random.Generator(np.random.PCG64(0))
    res = {}
    for head, (H, W) in (('ursonet', (512, 512)), ('keypoints', (240, 384))):
        arch = mobilenet_v2('keypoints') if head == 'keypoints' else mobilenet_v2('ursonet', 1728, 3)
        sd = synthetic_state_dict(arch, seed=1001, head_std=0.002 if head == 'keypoints' else 0.01)
        eng = Engine(Bl.pack(sd, arch, dtype=dt), 'cuda:0')
        eng.reserve(64, H, W)
        fr = torch.from_numpy(rng.integers(0, 256, (64, H, W, 3), dtype=np.uint8)).cuda()
        o, p = eng.forward(fr)
        torch.cuda.synchronize()
        res[head + '_out0'] = o.cpu().numpy()
        if p is not None:
            res[head + '_out1'] = p.cpu().numpy()
        eng.close()
    np.savez(out, **res)
    print('saved', out, {k: v.shape for k, v in res.items()})


if __name__ == '__main__':
    main()
