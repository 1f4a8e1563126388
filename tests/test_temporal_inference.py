"""Host logic of the Inference engine slot (spef_amd/inference.py, src/temporal/inference.py:19-191) and of its
temporal filter (spef_amd/temporal.py vs the reference's TemporalPDF, tests/golden/temporal_pdf.npz). No GPU:
the per-frame post-processing is exercised with a stub engine standing in for SPEMi355x."""
import numpy as np
import pytest

from spef_amd import temporal as T


@pytest.mark.parametrize('metric', T.METRICS)
def test_temporal_pdf_matches_reference(golden, metric):
    g = golden('temporal_pdf.npz')
    for n, alpha, tag in ((0.8, 16.49, 'ori'), (0.5, 48.64, 'pos')):
        f = T.TemporalPDF(n=n, alpha=alpha, distance_metric=metric)
        for i in range(g['seq'].shape[0]):
            pdf, d = f.update_pdf(g['seq'][i])
            np.testing.assert_allclose(pdf, g[f'{metric}_{tag}_pdf'][i], rtol=1e-6, atol=1e-12)
            np.testing.assert_allclose(d, g[f'{metric}_{tag}_dist'][i], rtol=1e-6, atol=1e-12)
        f.reset()
        assert f.previous_pdf is None


def test_temporal_pdf_rejects_unknown_metric():
    f = T.TemporalPDF(distance_metric='cosine')
    f.update_pdf(np.ones(4))
    with pytest.raises(ValueError):
        f.update_pdf(np.ones(4))


class _StubEngine:
    """predict() -> a fixed sequence of batch-1 pose dicts (what SPEMi355x.predict returns)."""

    def __init__(self, poses):
        self.poses = list(poses)
        self.closed = False

    def predict(self, image):
        return self.poses.pop(0), 1.25

    def close(self):
        self.closed = True


def _inference(poses, su):
    from spef_amd.inference import Inference
    stub = _StubEngine(poses)
    return Inference(None, 'gpu_host', su, engine_factories={'gpu_host': lambda m, s: stub}), stub


def test_inference_device_names():
    from spef_amd.inference import DEVICES, Inference
    from spef_amd.spe.spe_utils import SPEUtils
    assert DEVICES[-1] == 'gpu_mi355x' and set(DEVICES[:4]) == {'gpu_host', 'cpu_host', 'gpu_jetson', 'cpu_ultra96'}
    su = SPEUtils()
    with pytest.raises(AssertionError):
        Inference(None, 'tpu', su)
    with pytest.raises(ValueError):          # a reference target without an engine factory
        Inference(None, 'cpu_host', su)


def test_inference_pole_continuity_and_bbox():
    """inference.py:128-155: batch squeeze, the quaternion sign follows the previous still frame (an outlier with
    |dot| <= 0.5 does not move the pole), keypoints + bbox from the pose for visualisation."""
    import torch
    from oracle import decode_ref as D
    from spef_amd.spe.camera import SpeedCamera
    from spef_amd.spe.keypoints import KeyPoints
    from spef_amd.spe.spe_utils import SPEUtils
    kp3d = np.random.default_rng(0).normal(0, 0.3, (11, 3)).astype(np.float32)
    su = SPEUtils(SpeedCamera, keypoints_path=KeyPoints(SpeedCamera, kp3d))
    q0 = np.array([0.5, 0.5, 0.5, 0.5], np.float32)
    t0 = np.array([0.1, -0.2, 8.0], np.float32)
    out = np.array([0.0, 0.0, 0.0, 1.0], np.float32)              # |dot| = 0.5 with q0: an outlier
    poses = [{'ori': q0[None], 'pos': t0[None]}, {'ori': -q0[None], 'pos': t0[None]},
             {'ori': out[None], 'pos': t0[None]}, {'ori': -q0[None], 'pos': t0[None]}]
    inf, stub = _inference(poses, su)
    x = torch.zeros(1, 3, 8, 8)
    p1, lat, pv = inf.predict(x)
    assert lat == 1.25 and pv is None and p1['ori'].shape == (4,) and inf.img_size == (1, 3, 8, 8)
    np.testing.assert_array_equal(p1['keypoints'], D.create_keypoints2d(q0, t0, kp3d))
    np.testing.assert_array_equal(p1['bbox'], D.create_bbox_from_keypoints(p1['keypoints']))
    p2, _, _ = inf.predict(x)
    np.testing.assert_array_equal(p2['ori'], q0)                   # sign flipped back
    p3, _, _ = inf.predict(x)
    np.testing.assert_array_equal(p3['ori'], out)                  # kept, and the pole stays at q0
    np.testing.assert_array_equal(inf.prev_still_ori, q0)
    p4, _, _ = inf.predict(x)
    np.testing.assert_array_equal(p4['ori'], q0)
    with pytest.raises(ValueError):
        stub.poses.append({'ori': q0[None], 'pos': t0[None]})
        inf.predict(x, video_type='Kalman')
    inf.reset()
    assert inf.prev_still_ori is None
    inf.close()
    assert stub.closed and inf.inference_engine is None
