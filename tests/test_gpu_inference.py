"""The Inference engine slot 'gpu_mi355x' (spef_amd/inference.py; reference src/temporal/inference.py:46-80) on the
GPU: still-frame poses equal SPEMi355x.predict, and the 'Adaptative' video filter's poses equal the oracle's decode
of the filtered PDFs (TemporalPDF, pdf_compare.py:94)."""
import numpy as np
import pytest
import torch

from oracle import decode_ref as D

pytestmark = pytest.mark.gpu


def test_inference_gpu_mi355x_still_and_adaptive_video(golden):
    from spef_amd.arch import mobilenet_v2
    from spef_amd.inference import Inference
    from spef_amd.spe.spe_utils import SPEUtils
    from spef_amd.spe_mi355x import SPEMi355x
    from spef_amd.temporal import TemporalPDF
    from spef_amd.weights import synthetic_state_dict
    su = SPEUtils(None, 'classification', 12, 3, False, 'classification')
    sd = synthetic_state_dict(mobilenet_v2('ursonet', su.orientation.n_bins, su.position.n_bins), seed=1001)
    inf = Inference(sd, 'gpu_mi355x', su)                          # a reference-layout state_dict, packed here
    assert isinstance(inf.inference_engine, SPEMi355x)
    rng = np.random.Generator(np.random.PCG64(21))
    frames = [torch.from_numpy(rng.random((1, 3, 128, 160), dtype=np.float32)) for _ in range(3)]
    f_ori, f_pos = TemporalPDF(0.8, 16.49, 'l2'), TemporalPDF(0.5, 48.64, 'l2')
    prev = None
    for x in frames:
        still, lat, video = inf.predict(x, video_type='Adaptative')
        ref, _ = inf.inference_engine.predict(x)                   # the same frame straight through SPEMi355x
        assert abs(float(np.dot(ref['ori'][0], still['ori']))) == pytest.approx(1.0, abs=1e-6)   # up to the pole
        np.testing.assert_array_equal(ref['pos'][0], still['pos'])
        assert lat > 0 and set(still) >= {'ori', 'pos', 'ori_soft', 'pos_soft'} and still['ori'].shape == (4,)
        po, do = f_ori.update_pdf(still['ori_soft'])
        pp, dp = f_pos.update_pdf(still['pos_soft'])
        np.testing.assert_allclose(video['ori_soft'], po, rtol=1e-6)
        np.testing.assert_allclose(video['pos_soft'], pp, rtol=1e-6)
        assert video['ori_distance'] == pytest.approx(do) and video['pos_distance'] == pytest.approx(dp)
        rq = D.decode_orientation(po, su.orientation.histogram)
        assert D.angle_deg_stable(video['ori'][None], rq[None]).max() < 1e-3
        rp = D.decode_position_batch(pp[None], su.position.histogram)[0]
        assert np.abs(video['pos'] - rp).max() < 1e-4
        if prev is not None:
            assert np.dot(prev, video['ori']) >= 0 or abs(np.dot(prev, video['ori'])) <= 0.5
        prev = video['ori']
    inf.close()
