"""GPU: the fp16x2 schedule (blob dtype 5, csrc/k_x2.hip) -- fp32 activations with hi + lo fp16 MFMA operands, the
parity variant for heads the fp16 schedule cannot bound.

Tolerances are the north star's, absolute, with no scaling by the head's weight scale: raw head outputs 1e-3,
orientation < 0.1 deg, position < 1 mm. The sharp-head case (head_std 0.3, the reference-generated predict fixtures'
scale, tests/golden/cases.py) is where the fp16 schedule does not meet 1e-3 (tools/sharp_head_budget.py, DESIGN.md
section 5); the same test states the fp16 figure it measures.
"""
import numpy as np
import pytest
import torch

from oracle import decode_ref as D
from oracle import model_ref as M
from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.weights import state_dict_digest, synthetic_state_dict

pytestmark = pytest.mark.gpu

LOGIT_TOL = 1e-3      # north_star, absolute
X2_GOLDEN_TOL = 1e-4  # vs the reference's fixtures: split operands carry 22 significant bits (measured ~1e-5, below)


def _frames(b, h, w, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    base = rng.integers(0, 40, (b, h, w, 1), dtype=np.uint8)
    blob = rng.integers(0, 215, (b, h // 4, w // 4, 1), dtype=np.uint8).repeat(4, 1).repeat(4, 2)
    return np.repeat(np.clip(base.astype(np.int32) + blob, 0, 255).astype(np.uint8), 3, axis=3)


@pytest.fixture(scope='module')
def sd():
    return synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=1001)


@pytest.fixture(scope='module')
def x2(sd):
    from spef_amd.engine import Engine
    e = Engine(Bl.pack(sd, dtype='fp16x2'), 'cuda:0')
    yield e
    e.close()


def test_blob_layout(sd):
    info = Bl.describe(Bl.pack(sd, dtype='fp16x2'))
    assert info['dtype'] == 5
    from spef_amd import _lib as L
    import ctypes as C
    b = Bl.pack(sd, dtype='fp16x2')
    dt = C.c_int()
    L.check(L.load().spef_validate_blob(C.create_string_buffer(b, len(b)), len(b), C.byref(dt), None, None, None))
    assert dt.value == 5


@pytest.mark.parametrize('name', ['fwd_64x64_b2.npz', 'fwd_240x384_b1.npz', 'fwd_512x512_b1.npz'])
def test_forward_vs_reference_golden(x2, golden, name):
    g = golden(name)
    for x in (torch.from_numpy(g['frames']).cuda(), M.u8_nhwc_to_nchw_f32(g['frames']).contiguous().cuda()):
        ori, pos = x2.forward(x)
        d = max(np.abs(ori.cpu().numpy() - g['ori']).max(), np.abs(pos.cpu().numpy() - g['pos']).max())
        assert d < X2_GOLDEN_TOL, (name, d)


@pytest.mark.parametrize('b,h,w', [(2, 96, 128), (1, 100, 136)])
def test_block_outputs_vs_oracle(x2, sd, b, h, w):
    """Every block output (ragged maps: partial tiles) within 5e-5 of the FP32 oracle, relative to the map's max (measured
    2.1e-5 at block 2: 22-bit operands; the u8 front kernel folds /255 into the weights instead of rounding x / 255)."""
    fr = _frames(b, h, w, 5 + h)
    x = M.u8_nhwc_to_nchw_f32(fr)
    xg = torch.from_numpy(fr).cuda()
    for op in range(0, 18):
        ref = M.backbone(x, sd, upto=op).permute(0, 2, 3, 1).numpy()
        got = x2.probe(xg, op).cpu().numpy()
        assert got.shape == ref.shape, (op, got.shape, ref.shape)
        err = np.abs(got - ref).max() / max(1e-6, np.abs(ref).max())
        assert err < 5e-5, (op, err)


def test_hidden_split_blocks_vs_oracle(x2, sd):
    """B=24 at 240x384 (the keypoint head's input size): blocks 15-17 on 8x12 maps run the hidden-split form (two
    workgroups per 8x8 tile, ordered partial-sum join); their outputs, and those of the blocks before them, within the
    block-output bound of test_block_outputs_vs_oracle."""
    fr = _frames(24, 240, 384, 41)
    x = M.u8_nhwc_to_nchw_f32(fr)
    xg = torch.from_numpy(fr).cuda()
    torch.set_num_threads(16)
    for op in (8, 10, 15, 17):
        ref = M.backbone(x, sd, upto=op).permute(0, 2, 3, 1).numpy()
        got = x2.probe(xg, op).cpu().numpy()
        assert got.shape == ref.shape, (op, got.shape, ref.shape)
        err = np.abs(got - ref).max() / max(1e-6, np.abs(ref).max())
        assert err < 5e-5, (op, err)


def test_sharp_head_logits_absolute(golden):
    """the bench weights with a sharp orientation head (head_std 0.3: logits up to ~20, peaked
    histograms) at 512x512 -- max |d logit| against the FP32 oracle at the north star's absolute 1e-3.
    fp16x2 meets it; the fp16 schedule's figure is measured and stated (it does not: weight rounding is systematic
    and the 1280-wide head adds it up)."""
    from spef_amd.engine import Engine
    sd = synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=1001, head_std=0.3, pos_std=0.01,
                              pos_bias=(0.3, -0.2, 12.0))
    fr = _frames(4, 512, 512, 77)
    torch.set_num_threads(16)
    ro, rp = M.forward(M.u8_nhwc_to_nchw_f32(fr), sd)
    ro, rp = ro.numpy(), rp.numpy()
    h, _ = D.orientation_histogram(12, False)
    rq = D.decode_orientation_batch(D.softmax_f32(ro), h)
    res = {}
    for dt in ('fp16x2', 'fp16'):
        e = Engine(Bl.pack(sd, dtype=dt), 'cuda:0')
        try:
            e.set_decode_tables(h, None)
            o, p = e.forward(torch.from_numpy(fr).cuda())
            dec = e.decode(1, 0, o, p)
            res[dt] = (np.abs(o.cpu().numpy() - ro).max(), np.abs(p.cpu().numpy() - rp).max(),
                       D.angle_deg_stable(dec['ori'].cpu().numpy().astype(np.float64), rq).max())
        finally:
            e.close()
    print('sharp head (std 0.3) max|d logit|, max|d pos|, max deg:', res)
    assert np.abs(ro).max() > 5.0                          # really a sharp head
    lo, po, ao = res['fp16x2']
    assert lo < LOGIT_TOL and po < 1e-3 and ao < 0.1, res['fp16x2']
    assert res['fp16'][2] < 0.1 and res['fp16'][1] < 1e-3   # the fp16 pose still holds ...
    assert 2e-3 < res['fp16'][0] < 5e-2, res['fp16']       # ... its logits do not (stated figure)


def test_keypoint_head_vs_reference_fixture(golden):
    """fp16x2 keypoint blob against the reference's own ModelWrapper(MobileNetV2, KeypointRegressionHead) outputs
    (tests/golden/kp_head_240x384_b2.npz): within the north-star 1e-3 (the fp16 fast variant is not)."""
    from spef_amd.engine import Engine
    arch = mobilenet_v2('keypoints')
    sd = synthetic_state_dict(arch, seed=1001, head_std=0.002)
    g = golden('kp_head_240x384_b2.npz')
    assert state_dict_digest(sd) == str(g['digest'])
    e = Engine(Bl.pack(sd, arch, dtype='fp16x2'), 'cuda:0')
    try:
        raw, _ = e.forward(torch.from_numpy(g['frames']).cuda())
        d = np.abs(raw.cpu().numpy() - g['raw']).max()
        assert d < X2_GOLDEN_TOL, d
        rng = np.random.Generator(np.random.PCG64(5))
        fr = rng.integers(0, 256, (3, 240, 384, 3), dtype=np.uint8)
        raw, _ = e.forward(torch.from_numpy(fr).cuda())
        ref = M.forward(M.u8_nhwc_to_nchw_f32(fr), sd, head='keypoints')
        assert np.abs(raw.cpu().numpy() - ref.numpy()).max() < X2_GOLDEN_TOL
    finally:
        e.close()


def _oracle_block(x, sd, op):
    """Block ``op`` (features.features[op], 1-17) of the oracle on its own input (NCHW fp32)."""
    fp, cin, idx = 'features.features', 32, 1
    for t, c, n, s in M._IR:
        for i in range(n):
            if idx == op:
                stride, hidden, j = (s if i == 0 else 1), int(round(cin * t)), 0
                y = x
                if t != 1:
                    y = M._conv_bn_act(y, sd, f'{fp}.{idx}.conv.{j}', 1, 1, True)
                    j += 1
                y = M._conv_bn_act(y, sd, f'{fp}.{idx}.conv.{j}', stride, hidden, True)
                y = M._conv_bn_act(y, sd, f'{fp}.{idx}.conv.{j + 1}', 1, 1, False)
                return x + y if (stride == 1 and cin == c) else y
            cin, idx = c, idx + 1
    raise ValueError(op)


@pytest.mark.parametrize('b,h,w', [(33, 512, 512), (257, 100, 136)])
def test_persistent_tile_blocks_vs_oracle(x2, sd, b, h, w):
    """Blocks 8-14 with more tiles than CUs run persistent workgroups (x2_irw_kernel PT: ceil(tiles / CUs) tiles per
    workgroup as one chunk stream). 33 frames at 512^2: 264 tiles of blocks 8-13, two per workgroup; 257 frames at
    100 x 136: one 7 x 9 tile per frame, 129 workgroups, the last with a single tile (uneven split). Each block's
    output against the oracle's block applied to the GPU's own input of that block, relative to the map's max."""
    fr = _frames(b, h, w, 3 + b)
    xg = torch.from_numpy(fr).cuda()
    torch.set_num_threads(16)
    prev = x2.probe(xg, 7).cpu()
    for op in range(8, 15):
        got = x2.probe(xg, op).cpu()
        ref = _oracle_block(prev.permute(0, 3, 1, 2).contiguous(), sd, op).permute(0, 2, 3, 1).numpy()
        assert got.shape == ref.shape, (op, got.shape, ref.shape)
        err = np.abs(got.numpy() - ref).max() / max(1e-6, np.abs(ref).max())
        assert err < 2e-5, (op, err)
        prev = got
