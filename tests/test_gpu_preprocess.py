"""On-device input preprocessing (Resize(img_size) on decoded frames) vs Pillow and the resize oracle."""
import numpy as np
import pytest
import torch
from PIL import Image

from oracle import resize_ref as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def engine():
    from spef_amd import blob as Bl
    from spef_amd.arch import mobilenet_v2
    from spef_amd.engine import Engine
    from spef_amd.weights import synthetic_state_dict
    sd = synthetic_state_dict(mobilenet_v2(), seed=1001)
    e = Engine(Bl.pack(sd), 'cuda:0')
    yield e, sd
    e.close()


def _frames(b, h, w, seed):
    rng = np.random.default_rng(seed)
    g = rng.integers(0, 256, (b, h, w), dtype=np.uint8)
    f = np.repeat(g[..., None], 3, axis=3)
    f[..., 2] ^= rng.integers(0, 8, (b, h, w), dtype=np.uint8)
    return f


@pytest.mark.parametrize('src,dst', [((1200, 1920), (512, 512)), ((1200, 1920), (240, 384)), ((50, 70), (64, 96))])
def test_resize_bit_exact_vs_pillow(engine, src, dst):
    eng, _ = engine
    fr = _frames(2, *src, seed=src[0] + dst[1])
    got = eng.preprocess(torch.from_numpy(fr).cuda(), dst).cpu().numpy()
    for i in range(2):
        want = np.asarray(Image.fromarray(fr[i]).resize((dst[1], dst[0]), Image.BILINEAR))
        np.testing.assert_array_equal(got[i], want)
        np.testing.assert_array_equal(got[i], R.pil_resize(fr[i], *dst))


def test_predict_frames_matches_host_resize(engine):
    """predict_frames(raw) == predict(PIL resize(raw)) -- the reference DataLoader's Resize, done on the host."""
    from spef_amd.spe.spe_utils import SPEUtils
    from spef_amd.spe_mi355x import SPEMi355x
    eng, _ = engine
    su = SPEUtils(None, 'classification', 12, 3, False, 'regression')
    spe = SPEMi355x(eng, 'cuda:0', su)
    fr = _frames(2, 1200, 1920, seed=4)
    pose_dev, lat = spe.predict_frames(torch.from_numpy(fr), (512, 512))
    small = np.stack([np.asarray(Image.fromarray(f).resize((512, 512), Image.BILINEAR)) for f in fr])
    pose_host, _ = spe.predict(torch.from_numpy(small))          # uint8 NHWC frames, same fused path
    assert lat > 0
    for k in ('ori_soft', 'ori', 'pos'):
        np.testing.assert_array_equal(pose_dev[k], pose_host[k])
