"""GPU keypoint mode: batched EPnP kernel and the keypoint-regression head vs the CPU oracle."""
import numpy as np
import pytest
import torch

from oracle import decode_ref as D
from oracle import epnp_ref as E
from oracle import model_ref as M
from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.weights import plant_keypoint_head, synthetic_state_dict

pytestmark = pytest.mark.gpu


KP_TOL = 1e-3        # north_star: raw head outputs within 1e-3 of the float32 reference (fp32 keypoint blobs)
KP_TOL_FP16 = 2e-3   # the fp16 fast variant: the unpooled 122,880-wide head sees fp16 storage noise


@pytest.fixture(scope='module')
def kp_sd():
    return synthetic_state_dict(mobilenet_v2('keypoints'), seed=1001, head_std=0.002)


@pytest.fixture(scope='module')
def kp_engine(kp_sd):
    """The keypoint parity variant: fp32 blob (k_f32.hip schedule, exact-fp32 MFMA) -- build_mi355x's default for
    keypoint experiments."""
    from spef_amd.engine import Engine
    e = Engine(Bl.pack(kp_sd, mobilenet_v2('keypoints'), dtype='fp32'), 'cuda:0')
    yield e, kp_sd
    e.close()


@pytest.fixture(scope='module')
def kp_engine16(kp_sd):
    from spef_amd.engine import Engine
    e = Engine(Bl.pack(kp_sd, mobilenet_v2('keypoints'), dtype='fp16'), 'cuda:0')
    yield e, kp_sd
    e.close()


def _cfg(engine, golden):
    g = golden('keypoints.npz')
    engine.set_keypoints(g['kp3d'], g['K'], float(g['nu']), float(g['nv']))
    return g


def test_epnp_noise_free_kat(kp_engine, golden):
    eng, _ = kp_engine
    g = _cfg(eng, golden)
    kp = torch.from_numpy(g['kp2d']).cuda()
    out = eng.decode_keypoints(kp, apply_sigmoid=False)
    q, t = out['ori'].cpu().numpy(), out['pos'].cpu().numpy()
    assert not out['status'].cpu().numpy().any()
    assert D.angle_deg_stable(q, g['q']).max() < 5e-4            # 1,800 reference poses
    assert np.linalg.norm(t - g['t'], axis=1).max() < 2e-4


def test_epnp_matches_oracle_on_noisy_keypoints(kp_engine, golden):
    eng, _ = kp_engine
    g = _cfg(eng, golden)
    rng = np.random.default_rng(3)
    kp = (g['kp2d'][:256] + rng.normal(0, 3 / 1920, (256, 24))).astype(np.float32)
    out = eng.decode_keypoints(torch.from_numpy(kp).cuda(), apply_sigmoid=False)
    rq, rt = E.decode_batch(kp, g['kp3d'], g['K'])
    ang = D.angle_deg_stable(out['ori'].cpu().numpy(), rq)
    dt = np.linalg.norm(out['pos'].cpu().numpy() - rt, axis=1)
    assert np.median(ang) < 1e-4 and ang.max() < 0.1              # north_star: < 0.1 deg
    assert np.median(dt) < 1e-5 and dt.max() < 1e-3               # < 1 mm


def _cfg_plus(engine, golden):
    g = golden('keypoints_speedplus.npz')
    engine.set_keypoints(g['kp3d'], g['K'], float(g['nu']), float(g['nv']), g['dist'])
    return g


def test_epnp_with_lens_distortion_kat(kp_engine, golden):
    """SPEED+ camera (lens distortion, speed_plus.py:18-40): the reference's own distorted projections of the 1,800
    valid.json poses (tests/golden/keypoints_speedplus.npz) -> undistortPoints (5 iterations, as cv2.solvePnP) +
    EPnP on the GPU recovers every pose, and agrees with the oracle's restatement of the same steps."""
    eng, _ = kp_engine
    try:
        g = _cfg_plus(eng, golden)
        out = eng.decode_keypoints(torch.from_numpy(g['kp2d']).cuda(), apply_sigmoid=False)
        q, t = out['ori'].cpu().numpy(), out['pos'].cpu().numpy()
        assert not out['status'].cpu().numpy().any()
        assert D.angle_deg_stable(q, g['q']).max() < 5e-4
        assert np.linalg.norm(t - g['t'], axis=1).max() < 2e-4
        rq, rt = E.decode_batch(g['kp2d'][:200], g['kp3d'], g['K'], float(g['nu']), float(g['nv']), g['dist'])
        assert D.angle_deg_stable(q[:200], rq).max() < 1e-5
        assert np.abs(t[:200] - rt).max() < 1e-5
    finally:
        _cfg(eng, golden)


def test_epnp_with_lens_distortion_noisy(kp_engine, golden):
    eng, _ = kp_engine
    try:
        g = _cfg_plus(eng, golden)
        rng = np.random.default_rng(4)
        kp = (g['kp2d'][:256] + rng.normal(0, 3 / 1920, (256, 24))).astype(np.float32)
        out = eng.decode_keypoints(torch.from_numpy(kp).cuda(), apply_sigmoid=False)
        rq, rt = E.decode_batch(kp, g['kp3d'], g['K'], float(g['nu']), float(g['nv']), g['dist'])
        ang = D.angle_deg_stable(out['ori'].cpu().numpy(), rq)
        dt = np.linalg.norm(out['pos'].cpu().numpy() - rt, axis=1)
        assert np.median(ang) < 1e-4 and ang.max() < 0.1
        assert np.median(dt) < 1e-5 and dt.max() < 1e-3
    finally:
        _cfg(eng, golden)


def test_sigmoid_then_epnp(kp_engine, golden):
    eng, _ = kp_engine
    g = _cfg(eng, golden)
    inside = np.all((g['kp2d'] > 1e-3) & (g['kp2d'] < 1 - 1e-3), axis=1)   # keypoints in the frame
    kp = g['kp2d'][inside][:64].astype(np.float64)
    logit = np.log(kp / (1 - kp)).astype(np.float32)
    out = eng.decode_keypoints(torch.from_numpy(logit).cuda(), apply_sigmoid=True)
    sig = D.sigmoid_f32(logit)
    np.testing.assert_allclose(out['keypoints'].cpu().numpy(), sig, rtol=2e-6, atol=1e-7)
    rq, rt = E.decode_batch(sig, g['kp3d'], g['K'])
    assert D.angle_deg_stable(out['ori'].cpu().numpy(), rq).max() < 1e-3
    assert D.angle_deg_stable(out['ori'].cpu().numpy(), g['q'][inside][:64]).max() < 0.05


def test_keypoint_head_forward(kp_engine):
    """KeypointRegressionHead (flatten NCHW -> Linear 122880 -> 24) at 240x384 vs the oracle, fp32 blob: within the
    north-star 1e-3 (measured ~1e-6: the same fp32 products, only the summation order differs)."""
    eng, sd = kp_engine
    rng = np.random.Generator(np.random.PCG64(5))
    fr = rng.integers(0, 256, (3, 240, 384, 3), dtype=np.uint8)
    raw, _ = eng.forward(torch.from_numpy(fr).cuda())
    ref = M.forward(M.u8_nhwc_to_nchw_f32(fr), sd, head='keypoints')
    assert np.abs(raw.cpu().numpy() - ref.numpy()).max() < KP_TOL


def test_keypoint_head_vs_reference_fixture(kp_engine, golden):
    """Raw outputs and keypoint-mode sigmoid against the reference's own ModelWrapper(MobileNetV2,
    KeypointRegressionHead) (tests/golden/kp_head_240x384_b2.npz, generated by importing the reference), fp32 blob:
    within the north-star 1e-3."""
    from spef_amd.weights import state_dict_digest
    eng, sd = kp_engine
    g = golden('kp_head_240x384_b2.npz')
    assert state_dict_digest(sd) == str(g['digest'])
    raw, _ = eng.forward(torch.from_numpy(g['frames']).cuda())
    raw = raw.cpu().numpy()
    assert np.abs(raw - g['raw']).max() < KP_TOL
    out = eng.decode_keypoints(torch.from_numpy(raw).cuda(), apply_sigmoid=True)
    assert np.abs(out['keypoints'].cpu().numpy() - g['sigmoid']).max() < KP_TOL / 4     # sigmoid' <= 1/4


def test_keypoint_head_fp16_fast_variant(kp_engine16, golden):
    """fp16 keypoint blob (fused kernels, the URSONet speed path): stated bound 2e-3 on raw outputs of magnitude
    ~0.8 (measured 1.17e-3). The URSONet heads average fp16 storage rounding over 256 pixels before their FC; this
    head reads all 122,880 values individually. tools/kp_error_budget.py splits the budget by rounding class: no class
    dominates (weights 9.0e-4, block outputs 8.3e-4, hidden 5.0e-4, depthwise out 4.4e-4 alone), so fp32 storage, not a
    targeted fix, is what reaches 1e-3 -- the fp32 blob above."""
    eng, sd = kp_engine16
    g = golden('kp_head_240x384_b2.npz')
    raw, _ = eng.forward(torch.from_numpy(g['frames']).cuda())
    assert np.abs(raw.cpu().numpy() - g['raw']).max() < KP_TOL_FP16
    rng = np.random.Generator(np.random.PCG64(5))
    fr = rng.integers(0, 256, (3, 240, 384, 3), dtype=np.uint8)
    raw, _ = eng.forward(torch.from_numpy(fr).cuda())
    ref = M.forward(M.u8_nhwc_to_nchw_f32(fr), sd, head='keypoints')
    assert np.abs(raw.cpu().numpy() - ref.numpy()).max() < KP_TOL_FP16


def test_predict_keypoint_mode(kp_engine, golden):
    """SPEMi355x.predict in keypoint mode: pose dict keys of SPETorch (spe_torch.py:63-76), sigmoid keypoints
    matching the oracle forward, ori/pos equal to the EPnP kernel on those keypoints."""
    from spef_amd.spe.keypoints import KeyPoints
    from spef_amd.spe.spe_utils import SPEUtils
    from spef_amd.spe_mi355x import SPEMi355x
    eng, sd = kp_engine
    g = golden('keypoints.npz')

    class Cam:
        K, nu, nv = g['K'], float(g['nu']), float(g['nv'])
    su = SPEUtils(Cam, 'keypoints', pos_mode='keypoints', keypoints_path=KeyPoints(Cam, g['kp3d']))
    spe = SPEMi355x(eng, 'cuda:0', su)
    rng = np.random.Generator(np.random.PCG64(9))
    x = torch.from_numpy(rng.random((2, 3, 240, 384), dtype=np.float32))
    pose, lat = spe.predict(x)
    assert set(pose) == {'keypoints', 'ori', 'pos'} and lat > 0
    ref = D.sigmoid_f32(M.forward(x, sd, head='keypoints').numpy())
    assert np.abs(pose['keypoints'] - ref).max() < KP_TOL / 4   # sigmoid' <= 1/4
    chk = eng.decode_keypoints(torch.from_numpy(pose['keypoints']).cuda(), apply_sigmoid=False)
    np.testing.assert_array_equal(chk['ori'].cpu().numpy(), pose['ori'])
    np.testing.assert_array_equal(chk['pos'].cpu().numpy(), pose['pos'])


def test_stream_pipeline_keypoint_mode_matches_single_engine(kp_sd, golden):
    """StreamPipeline.submit_keypoints (the bench's keypoint timing path: batches on three streams, each with its own
    context) gives every batch the same raw outputs, poses and status as one engine on one stream."""
    from spef_amd.pipeline import StreamPipeline
    g = golden('keypoints.npz')
    rng = np.random.Generator(np.random.PCG64(31))
    batches = [torch.from_numpy(rng.integers(0, 256, (3, 240, 384, 3), dtype=np.uint8)).cuda() for _ in range(4)]
    pipe = StreamPipeline(Bl.pack(kp_sd, mobilenet_v2('keypoints'), dtype='fp16x2'), 'cuda:0', depth=3)
    try:
        pipe.set_keypoints(g['kp3d'], g['K'], float(g['nu']), float(g['nv']))
        outs = [pipe.submit_keypoints(x) for x in batches]
        pipe.synchronize()
        ref = pipe.engines[0]
        for x, o in zip(batches, outs):
            raw, _ = ref.forward(x)
            r = ref.decode_keypoints(raw)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(o['raw'].cpu().numpy(), raw.cpu().numpy())
            for k in ('keypoints', 'ori', 'pos', 'status'):
                np.testing.assert_array_equal(o[k].cpu().numpy(), r[k].cpu().numpy(), err_msg=k)
    finally:
        pipe.close()


def _planted_kp_sd(golden):
    """Keypoint head whose sigmoid outputs are real keypoints: the head bias is logit() of the reference projection
    (KeyPoints.project, tests/golden/keypoints.npz) of the valid.json pose at the median distance, and the weights are
    small (std 2e-4: W . features moves each normalised keypoint by ~1e-2, ~20 px, per frame), so every frame's 11
    keypoints span the spacecraft's image as in the reference's keypoint mode (keypoints_utils.py:112-174) instead of
    the clustered, ill-conditioned points of a random head."""
    g = golden('keypoints.npz')
    i = int(np.argmin(np.abs(g['t'][:, 2] - np.median(g['t'][:, 2]))))
    sd = plant_keypoint_head(synthetic_state_dict(mobilenet_v2('keypoints'), seed=1001, head_std=2e-4), g['kp2d'][i])
    return sd, g, i


def test_keypoint_mode_b64_pipeline_vs_oracle(golden):
    """keypoint mode at the bench workload -- B = 64 synthetic SPEED-style 240 x 384
    frames (bench.py's generator), the fp16x2 keypoint blob (build_mi355x's keypoint default), StreamPipeline
    .submit_keypoints on three streams (forward + sigmoid + batched EPnP) -- against the FP32 oracle forward
    (oracle/model_ref.py) and the EPnP restatement (oracle/epnp_ref.py) at the north-star bounds (raw outputs 1e-3,
    orientation < 0.1 deg, position < 1 mm), for every batch of the pipeline, with a head that outputs real keypoints
    (_planted_kp_sd), so the pose bound is held with margin: the position error must stay under 0.3 mm. The EPnP kernel
    alone (on the GPU's own keypoints, against the oracle EPnP) is reported and bounded separately."""
    from spef_amd.data.synthetic import synth_frames
    from spef_amd.pipeline import StreamPipeline
    sd, g, i = _planted_kp_sd(golden)
    fr = synth_frames(64, 240, 384, 20_000)
    torch.set_num_threads(16)
    raw_ref = M.forward(M.u8_nhwc_to_nchw_f32(fr), sd, head='keypoints').numpy()
    kp_ref = D.sigmoid_f32(raw_ref)
    rq, rt = E.decode_batch(kp_ref, g['kp3d'], g['K'])
    # the planted head gives frames spread around the planted pose (not one degenerate cluster)
    spread_px = (kp_ref[:, 2::2].max(1) - kp_ref[:, 2::2].min(1)) * float(g['nu'])
    assert spread_px.min() > 50, spread_px.min()
    assert D.angle_deg_stable(rq, np.repeat(g['q'][i:i + 1], 64, 0)).max() < 20
    pipe = StreamPipeline(Bl.pack(sd, mobilenet_v2('keypoints'), dtype='fp16x2'), 'cuda:0', depth=3)
    try:
        pipe.set_keypoints(g['kp3d'], g['K'], float(g['nu']), float(g['nv']))
        pipe.reserve(64, 240, 384)
        xg = torch.from_numpy(fr).cuda()
        outs = [pipe.submit_keypoints(xg) for _ in range(3)]
        pipe.synchronize()
        for o in outs:
            raw = o['raw'].cpu().numpy()
            assert not o['status'].any().item()
            d_raw = np.abs(raw - raw_ref).max()
            ang = D.angle_deg_stable(o['ori'].cpu().numpy().astype(np.float64), rq)
            dpos = np.linalg.norm(o['pos'].cpu().numpy().astype(np.float64) - rt, axis=1)
            # decomposition: the GPU EPnP against the oracle EPnP on the GPU's own keypoints (solver parity alone)
            sq, st = E.decode_batch(D.sigmoid_f32(raw), g['kp3d'], g['K'])
            s_ang = D.angle_deg_stable(o['ori'].cpu().numpy().astype(np.float64), sq)
            s_pos = np.linalg.norm(o['pos'].cpu().numpy().astype(np.float64) - st, axis=1)
            print(f'B=64 keypoint step (pose {i}, z {g["t"][i, 2]:.1f} m, keypoint spread >= {spread_px.min():.0f} px): '
                  f'raw {d_raw:.2e}, ori max {ang.max():.2e} deg, pos max {dpos.max():.2e} m; '
                  f'EPnP alone {s_ang.max():.2e} deg, {s_pos.max():.2e} m')
            assert d_raw < KP_TOL and ang.max() < 0.1 and dpos.max() < 1e-3
            assert dpos.max() < 3e-4 and ang.max() < 0.03      # the bound with margin
            assert s_ang.max() < 0.01 and s_pos.max() < 1e-4
    finally:
        pipe.close()
