"""EPnP kernel timing (GPU box): the reference's own projections (tests/golden/keypoints.npz), B = 64 and 512 problems
per launch, HIP-event kernel time and KAT error. SPEF_LIB selects an A/B build (tools/build_variant.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd')]
import numpy as np
import torch

from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.engine import Engine
from spef_amd.quaternion import angle_deg
from spef_amd.weights import synthetic_state_dict

g = np.load(os.path.join(ROOT, 'tests', 'golden', 'keypoints.npz'))
arch = mobilenet_v2('keypoints')
eng = Engine(Bl.pack(synthetic_state_dict(arch, seed=1001, head_std=0.002), arch, dtype='fp32'), 'cuda:0')
eng.set_keypoints(g['kp3d'], g['K'], float(g['nu']), float(g['nv']))
for P in (64, 512, 1800):
    kp = torch.from_numpy(np.ascontiguousarray(g['kp2d'][:P], np.float32)).cuda()
    o = eng.decode_keypoints(kp, apply_sigmoid=False)
    torch.cuda.synchronize()
    if os.environ.get('EPNP_DUMP'):   # outputs for a bit-identity check of two builds
        np.savez(f"{os.environ['EPNP_DUMP']}_{P}.npz", ori=o['ori'].cpu().numpy(), pos=o['pos'].cpu().numpy())
    kat = float(np.max(angle_deg(o['ori'].cpu().numpy(), g['q'][:P])))
    katp = float(np.linalg.norm(o['pos'].cpu().numpy() - g['t'][:P], axis=1).max())
    for _ in range(5):
        eng.decode_keypoints(kp, apply_sigmoid=False)
    eng.profile_begin()
    for _ in range(50):
        eng.decode_keypoints(kp, apply_sigmoid=False)
    prof = eng.profile_end()
    n, ms = prof['epnp_kernel'][0], prof['epnp_kernel'][1]
    print(f'P={P}: {ms / n * 1e3:.1f} us per launch, {P * n / (ms / 1e3) / 1e6:.2f} M problems/s, '
          f'KAT {kat:.2e} deg {katp:.2e} m')
