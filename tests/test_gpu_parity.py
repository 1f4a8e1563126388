"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the reference golden fixtures.

Tolerances (north_star): raw head outputs ("heatmap logits") within 1e-3 absolute of the float32 reference;
recovered pose within 0.1 deg / 1 mm on identical inputs. fp16 storage is the parity default; bf16 is a
measured variant with its own stated bound.
"""
import numpy as np
import pytest
import torch

from oracle import decode_ref as D
from oracle import model_ref as M
from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

LOGIT_TOL = 1e-3          # north_star: outputs within 1e-3 of the FP32 reference
LOGIT_TOL_BF16 = 6e-3     # bf16 storage variant: 2x the 3.1e-3 measured over 32 x 1731 logits at C2 (test_gpu_c2_precision)


@pytest.fixture(scope='module')
def sd():
    return synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=1001)


@pytest.fixture(scope='module')
def engine(sd):
    from spef_amd.engine import Engine
    e = Engine(Bl.pack(sd, dtype='fp16'), 'cuda:0')
    yield e
    e.close()


@pytest.fixture(scope='module')
def engine_bf16(sd):
    from spef_amd.engine import Engine
    e = Engine(Bl.pack(sd, dtype='bf16'), 'cuda:0')
    yield e
    e.close()


def _frames(b, h, w, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    base = rng.integers(0, 40, (b, h, w, 1), dtype=np.uint8)
    blob = rng.integers(0, 215, (b, h // 4, w // 4, 1), dtype=np.uint8).repeat(4, 1).repeat(4, 2)
    return np.repeat(np.clip(base.astype(np.int32) + blob, 0, 255).astype(np.uint8), 3, axis=3)


@pytest.mark.parametrize('name', ['fwd_64x64_b2.npz', 'fwd_240x384_b1.npz', 'fwd_512x512_b1.npz'])
@pytest.mark.parametrize('layout', ['u8_nhwc', 'f32_nchw'])
def test_forward_vs_reference_golden(engine, golden, name, layout):
    g = golden(name)
    fr = g['frames']
    if layout == 'u8_nhwc':
        x = torch.from_numpy(fr).cuda()
    else:
        x = M.u8_nhwc_to_nchw_f32(fr).contiguous().cuda()
    ori, pos = engine.forward(x)
    torch.cuda.synchronize()
    d_ori = np.abs(ori.cpu().numpy() - g['ori']).max()
    d_pos = np.abs(pos.cpu().numpy() - g['pos']).max()
    assert d_ori < LOGIT_TOL and d_pos < LOGIT_TOL, (d_ori, d_pos)


def test_block_activations_vs_oracle(engine, sd):
    fr = _frames(2, 96, 128, 5)
    x = M.u8_nhwc_to_nchw_f32(fr)
    xg = torch.from_numpy(fr).cuda()
    for op in range(0, 18):
        ref = M.backbone(x, sd, upto=op).permute(0, 2, 3, 1).numpy()
        got = engine.probe(xg, op).cpu().numpy()
        assert got.shape == ref.shape, (op, got.shape, ref.shape)
        err = np.abs(got - ref).max() / max(1e-6, np.abs(ref).max())
        assert err < 2e-2, (op, err)


@pytest.mark.parametrize('b,h,w', [(3, 64, 96), (8, 512, 512)])
def test_forward_vs_oracle_batches(engine, sd, b, h, w):
    fr = _frames(b, h, w, b * 7 + h)
    ref_o, ref_p = M.forward(M.u8_nhwc_to_nchw_f32(fr), sd)
    ori, pos = engine.forward(torch.from_numpy(fr).cuda())
    assert np.abs(ori.cpu().numpy() - ref_o.numpy()).max() < LOGIT_TOL
    assert np.abs(pos.cpu().numpy() - ref_p.numpy()).max() < LOGIT_TOL


def test_backbone_features_mse(engine, sd):
    """C2: backbone features vs the CPU reference (MSE + the finn/spe_finn.py:116-149 statistics)."""
    fr = _frames(2, 256, 256, 3)
    ref = M.backbone(M.u8_nhwc_to_nchw_f32(fr), sd).permute(0, 2, 3, 1).numpy()
    got = engine.backbone(torch.from_numpy(fr).cuda()).cpu().numpy()
    mse = float(np.mean((got - ref) ** 2))
    assert mse < 1e-5, mse
    assert np.mean((got == 0) == (ref == 0)) > 0.99     # zero-pattern similarity (ReLU map)


def test_bf16_variant(engine_bf16, golden):
    g = golden('fwd_512x512_b1.npz')
    ori, pos = engine_bf16.forward(torch.from_numpy(g['frames']).cuda())
    d = max(np.abs(ori.cpu().numpy() - g['ori']).max(), np.abs(pos.cpu().numpy() - g['pos']).max())
    assert d < LOGIT_TOL_BF16, d


def test_decode_orientation_random(engine, golden):
    g = golden('decode_ori.npz')
    h, _ = D.orientation_histogram(12, False)
    engine.set_decode_tables(h, D.position_histogram(10))
    lg = torch.from_numpy(g['rand_logits']).cuda()
    pos_raw = torch.zeros((lg.shape[0], 3), device='cuda')
    out = engine.decode(1, 0, lg, pos_raw)
    soft = out['ori_soft'].cpu().numpy()
    np.testing.assert_allclose(soft[:16], g['rand_soft'], rtol=1e-5, atol=1e-9)
    assert D.angle_deg_stable(out['ori'].cpu().numpy(), g['rand_q']).max() < 1e-3
    assert not out['status'].cpu().numpy().any()


def test_decode_orientation_planted(engine, golden):
    g = golden('decode_ori.npz')
    h, red = D.orientation_histogram(12, False)
    engine.set_decode_tables(h, None)
    for ti, T in enumerate(g['temps']):
        n = g['planted_q'].shape[1]
        enc = np.stack([D.encode_orientation(q, h, red) for q in g['q_true'][:n]])
        lg = np.maximum((np.log(np.maximum(enc, 1e-30)) / T).astype(np.float32), np.float32(-80.0 / T))
        out = engine.decode(1, 0, torch.from_numpy(lg).cuda(), torch.zeros((n, 3), device='cuda'))
        ok = ~g['planted_raised'][ti]
        err = D.angle_deg_stable(out['ori'].cpu().numpy()[ok], g['planted_q'][ti][ok])
        assert err.max() < 1e-3, (T, err.max())


@pytest.mark.parametrize('scale', [0.0, 1e-4, 1e-2])
def test_decode_orientation_flat_softmax(engine, scale):
    """Flat and near-flat softmaxes (the random-weight bench regime and the degenerate limit): the moment matrix is
    close to I/4, where the decode's repeated squaring is slowest and its Gershgorin shift (k_head.hip) matters.
    The eigenvector there is ill-conditioned, so instead of comparing against numpy's choice the test checks the
    property the decode must satisfy: a finite unit quaternion whose Rayleigh quotient is the top eigenvalue of
    a = sum_i p_i q_i q_i^T (classification_utils.py:137-141)."""
    h, _ = D.orientation_histogram(12, False)
    engine.set_decode_tables(h, None)
    rng = np.random.Generator(np.random.PCG64(11))
    lg = (scale * rng.standard_normal((8, h.shape[0]))).astype(np.float32)
    out = engine.decode(1, 0, torch.from_numpy(lg).cuda(), torch.zeros((8, 3), device='cuda'))
    q = out['ori'].cpu().numpy().astype(np.float64)
    assert np.isfinite(q).all() and not out['status'].cpu().numpy().any()
    np.testing.assert_allclose(np.linalg.norm(q, axis=1), 1.0, atol=1e-6)
    p = D.softmax_f32(lg).astype(np.float64)
    hb = np.asarray(h, np.float64)
    for b in range(8):
        a = (hb * p[b][:, None]).T @ hb
        lam = np.linalg.eigvalsh(a)
        assert q[b] @ a @ q[b] >= lam[-1] - 1e-6 * (lam[-1] - lam[0] + 1e-12) - 1e-7, (scale, b)


def test_decode_position_classification(engine, golden):
    g = golden('decode_pos.npz')
    engine.set_decode_tables(None, g['grid'])
    lg = torch.from_numpy(g['logits']).cuda()
    out = engine.decode(0, 1, torch.ones((lg.shape[0], 4), device='cuda'), lg)
    np.testing.assert_allclose(out['pos_soft'].cpu().numpy()[:8], g['soft'], rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(out['pos'].cpu().numpy(), g['pos'], rtol=0, atol=1e-4)   # < 1 mm


def test_decode_nan_raises(engine):
    from spef_amd.spe.spe_utils import SPEUtils
    from spef_amd.spe_mi355x import SPEMi355x
    su = SPEUtils(None, 'classification', 12, 3, False, 'regression')
    h, _ = D.orientation_histogram(12, False)
    engine.set_decode_tables(h, None)
    lg = torch.full((2, 1728), float('nan'), device='cuda')
    out = engine.decode(1, 0, lg, torch.zeros((2, 3), device='cuda'))
    assert (out['status'].cpu().numpy() & 1).all()


def test_predict_end_to_end():
    """SPEMi355x.predict == oracle forward + reference decode on identical inputs (<0.1 deg, <1 mm absolute).
    A sharper orientation head (std 0.3) gives peaked orientation histograms: with the reference init (std 0.01)
    the softmax is near-uniform and the top eigenvector of `a` is ill-conditioned for ANY implementation. The
    position head keeps the reference init (pytorch_layers.py:25-27) with a SPEED-range bias (12 m range)."""
    from spef_amd.spe.spe_utils import SPEUtils
    from spef_amd.spe_mi355x import SPEMi355x
    sd = synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=1001, head_std=0.3, pos_std=0.01,
                              pos_bias=(0.4, -0.3, 12.0))
    su = SPEUtils(None, 'classification', 12, 3, False, 'regression')
    tgt = SPEMi355x(Bl.pack(sd, dtype='fp16'), 'cuda:0', su)
    fr = _frames(4, 240, 384, 9)
    x = M.u8_nhwc_to_nchw_f32(fr)
    pose, ms = tgt.predict(x)
    assert ms > 0
    ro, rp = M.forward(x, sd)
    h, _ = D.orientation_histogram(12, False)
    rq = D.decode_orientation_batch(D.softmax_f32(ro.numpy()), h)
    assert D.angle_deg_stable(pose['ori'], rq).max() < 0.1
    assert np.abs(pose['pos'] - rp.numpy()).max() < 1e-3           # < 1 mm, absolute
    assert np.abs(rp.numpy()[:, 2] - 12.0).max() < 1.0              # the position is at SPEED range
    assert pose['ori_soft'].shape == (4, 1728)
    tgt.close()


@pytest.mark.parametrize('b,h,w', [(2, 512, 512), (3, 240, 384), (2, 100, 136), (1, 64, 64)])
def test_fused_blocks_bit_identical_to_unfused(engine, b, h, w):
    """The fused inverted-residual kernel rounds and accumulates exactly like the one-kernel-per-conv
    schedule, so every block output (and the logits) must be bit-identical -- including partial edge tiles.
    (float32 NCHW input: the uint8 path replaces stem + block 1 by the front kernel, checked separately.)"""
    fr = M.u8_nhwc_to_nchw_f32(_frames(b, h, w, 100 + h)).contiguous().cuda()
    try:
        for op in range(1, 18):
            engine.set_fused(False)
            u = engine.probe(fr, op).cpu().numpy()
            engine.set_fused(True)
            f = engine.probe(fr, op).cpu().numpy()
            assert np.array_equal(u, f), (op, np.abs(u - f).max())
        engine.set_fused(False)
        uo, up = [t.cpu().numpy() for t in engine.forward(fr)]
        engine.set_fused(True)
        fo, fp = [t.cpu().numpy() for t in engine.forward(fr)]
        assert np.array_equal(uo, fo) and np.array_equal(up, fp)
    finally:
        engine.set_fused(True)


@pytest.mark.parametrize('b,h,w', [(2, 512, 512), (3, 240, 384), (2, 100, 136)])
def test_front_kernel_vs_stem_block1(engine, sd, b, h, w):
    """uint8 path: fused stem+block-1 front kernel (MFMA stem, split-fp16 weights) vs the fp32 VALU stem +
    separate block-1 kernel, and vs the oracle's block-1 output."""
    fr = _frames(b, h, w, 7 + w)
    x8 = torch.from_numpy(fr).cuda()
    xf = M.u8_nhwc_to_nchw_f32(fr).contiguous().cuda()
    got = engine.probe(x8, 1).cpu().numpy()
    sep = engine.probe(xf, 1).cpu().numpy()
    ref = M.backbone(M.u8_nhwc_to_nchw_f32(fr), sd, upto=1).permute(0, 2, 3, 1).numpy()
    scale = np.abs(ref).max()
    assert np.abs(got - sep).max() / scale < 4e-3
    assert np.abs(got - ref).max() / scale < 4e-3


@pytest.mark.parametrize('b,h,w', [(2, 512, 512), (2, 100, 136), (1, 240, 384)])
def test_role_split_blocks_bit_identical_to_slab(engine, b, h, w):
    """k_irp.hip (three-stage pipeline: MFMA waves expand + project, VALU waves depthwise) and k_irw.hip (expand
    waves pipelined against depthwise/project waves) keep the slab kernel's rounding points and accumulation order:
    every late-block output is bit-identical under SPEF_OPT_WAVESPEC 0, 1 and 2 (ragged maps included: 100x136
    frames give 7x9 and 4x5 maps, partial tiles everywhere)."""
    from spef_amd import _lib as L
    fr = torch.from_numpy(_frames(b, h, w, 31 + w)).cuda()
    try:
        for op in range(8, 18):
            outs = []
            for mode in (0, 1, 2):
                engine.set_option(L.OPT_WAVESPEC, mode)
                outs.append(engine.probe(fr, op).cpu().numpy())
            for mode in (1, 2):
                assert np.array_equal(outs[0], outs[mode]), (
                    op, mode, np.abs(outs[0].astype(np.float32) - outs[mode].astype(np.float32)).max())
    finally:
        engine.set_option(L.OPT_WAVESPEC, 2)


def test_fp32_variant_vs_reference_golden(sd, golden):
    """fp32 blob (k_f32.hip: exact-fp32 MFMA, one kernel per conv): the reference's own arithmetic, so the head
    outputs agree with the reference's fixtures to fp32 summation-order noise."""
    from spef_amd.engine import Engine
    e = Engine(Bl.pack(sd, dtype='fp32'), 'cuda:0')
    try:
        for name in ('fwd_64x64_b2.npz', 'fwd_240x384_b1.npz', 'fwd_512x512_b1.npz'):
            g = golden(name)
            for x in (torch.from_numpy(g['frames']).cuda(), M.u8_nhwc_to_nchw_f32(g['frames']).contiguous().cuda()):
                ori, pos = e.forward(x)
                d = max(np.abs(ori.cpu().numpy() - g['ori']).max(), np.abs(pos.cpu().numpy() - g['pos']).max())
                assert d < 1e-4, (name, d)
        fr = _frames(2, 96, 128, 5)
        x = M.u8_nhwc_to_nchw_f32(fr)
        for op in (0, 1, 2, 7, 17):
            ref = M.backbone(x, sd, upto=op).permute(0, 2, 3, 1).numpy()
            got = e.probe(torch.from_numpy(fr).cuda(), op).cpu().numpy()
            assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-5, op
    finally:
        e.close()
