"""GPU: the fp16mx schedule (blob dtype 6) -- the headline: the fp16x2 kernels and weights (hi + lo fp16 MFMA
operands, fp32 accumulation, fp32 depthwise) with the stem map, the block outputs of blocks 1-3 and the hidden tensors
of blocks 2-4 stored fp16 and every other activation fp32 (tools/precision_budget.py: 4.2e-4 max |d logit| at head
std 0.3 in float64 on this file's frames, against 1.3e-2 for the fp16 schedule).

Tolerances are the north star's, absolute, with no scaling by the head's weight scale: raw head outputs 1e-3,
orientation < 0.1 deg, position < 1 mm -- at the reference init (std 0.01) and at a sharp head (std 0.3, the
reference-generated predict fixtures' scale), up to the bench workload (B = 64, 512 x 512, StreamPipeline).
"""
import numpy as np
import pytest
import torch

from oracle import decode_ref as D
from oracle import model_ref as M
from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.data.synthetic import synth_frames
from spef_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

LOGIT_TOL = 1e-3      # north_star, absolute
POS_TOL_M = 1e-3
ORI_TOL_DEG = 0.1
MX_GOLDEN_TOL = 2e-4  # reference init (std 0.01): ~30x below the sharp-head figure (measured, printed below)
F16_BLOCKS = range(1, 4)   # blocks whose output the schedule stores in fp16 (cout <= 24: the 256^2 / 128^2 maps)
F16_HIDDEN = range(2, 5)   # blocks whose expanded hidden tensor the schedule stores in fp16 (csrc/k_mx.hip)


def _frames(b, h, w, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    base = rng.integers(0, 40, (b, h, w, 1), dtype=np.uint8)
    blob = rng.integers(0, 215, (b, h // 4, w // 4, 1), dtype=np.uint8).repeat(4, 1).repeat(4, 2)
    return np.repeat(np.clip(base.astype(np.int32) + blob, 0, 255).astype(np.uint8), 3, axis=3)


def _sharp_sd():
    return synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=1001, head_std=0.3, pos_std=0.01,
                                pos_bias=(0.3, -0.2, 12.0))


def _oracle_block(x, sd, idx, f16_hidden=F16_HIDDEN):
    """features.features[idx] of the oracle (oracle/model_ref.py: the reference's float32 arithmetic, op for op) on
    the activation x, with the schedule's fp16 hidden storage of blocks 2-4 restated (the expand output rounded to
    fp16 before the depthwise); idx 0 = the stem."""
    fp = 'features.features'
    if idx == 0:
        return M._conv_bn_act(x, sd, f'{fp}.0', 2, 1, True)
    cin, i = 32, 1
    for t, c, n, s in M._IR:
        for k in range(n):
            if i == idx:
                stride = s if k == 0 else 1
                y, j = x, 0
                if t != 1:
                    y = M._conv_bn_act(y, sd, f'{fp}.{idx}.conv.{j}', 1, 1, True)
                    if idx in f16_hidden:
                        y = y.half().float()
                    j += 1
                y = M._conv_bn_act(y, sd, f'{fp}.{idx}.conv.{j}', stride, int(round(cin * t)), True)
                y = M._conv_bn_act(y, sd, f'{fp}.{idx}.conv.{j + 1}', 1, 1, False)
                return x + y if (stride == 1 and cin == c) else y
            cin, i = c, i + 1
    raise ValueError(idx)


@pytest.fixture(scope='module')
def sd():
    return synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=1001)


@pytest.fixture(scope='module')
def mx(sd):
    from spef_amd.engine import Engine
    e = Engine(Bl.pack(sd, dtype='fp16mx'), 'cuda:0')
    yield e
    e.close()


def test_blob_layout(sd):
    import ctypes as C
    from spef_amd import _lib as L
    b = Bl.pack(sd, dtype='fp16mx')
    assert Bl.describe(b)['dtype'] == 6
    dt = C.c_int()
    L.check(L.load().spef_validate_blob(C.create_string_buffer(b, len(b)), len(b), C.byref(dt), None, None, None))
    assert dt.value == 6
    ops = Bl.describe(b)['ops']
    assert ops[0][0] == Bl.OP_STEM and ops[0][15] != Bl.ABSENT   # + the front kernel's row-triple stem operand (x1)
    assert [o[:7] for o in ops] == [o[:7] for o in Bl.describe(Bl.pack(sd, dtype='fp16x2'))['ops']]


@pytest.mark.parametrize('name', ['fwd_64x64_b2.npz', 'fwd_240x384_b1.npz', 'fwd_512x512_b1.npz'])
def test_forward_vs_reference_golden(mx, golden, name):
    g = golden(name)
    for x in (torch.from_numpy(g['frames']).cuda(), M.u8_nhwc_to_nchw_f32(g['frames']).contiguous().cuda()):
        ori, pos = mx.forward(x)
        d = max(np.abs(ori.cpu().numpy() - g['ori']).max(), np.abs(pos.cpu().numpy() - g['pos']).max())
        print(name, 'max |d| vs the reference fixture:', d)
        assert d < MX_GOLDEN_TOL, (name, d)


@pytest.mark.parametrize('mx_kernels', [1, 0])
@pytest.mark.parametrize('b,h,w', [(2, 96, 128), (1, 100, 136)])
def test_block_outputs_vs_oracle(mx, sd, b, h, w, mx_kernels):
    """Every block kernel (ragged maps: partial tiles) against the oracle's block applied to the GPU's own input for
    that block (the previous probe), so each kernel is checked on its own, with the schedule's fp16 storage points
    restated in the oracle (hidden tensors of blocks 2-4, outputs of blocks 1-3): blocks 1-3 store fp16, so the oracle's
    output is rounded to fp16 too and the two may differ by one fp16 rounding step where the exact value sits next to a
    rounding boundary (bound 1.2e-3 of the map's max: one ulp is at most 2^-10 of it); block 4 (fp16 hidden, fp32
    out) 2e-4; blocks 5-17 keep fp32 throughout (the fp16x2 bound, 5e-5 of the map's max). (The stem map is fp16 only
    inside the fused front kernel; the probe at op 0 runs the stem alone, in fp32.) Block 1 runs fused with the stem (front kernel) and is compared from the
    frames.

    mx_kernels = 0 (SPEF_OPT_MX_KERNELS, the library's fallback schedule for the same blob): stem + block 1 and blocks
    2-4 run on the fp16x2 kernels' fp16-I/O template variants (k_x2.hip IO = 1 / 2 / 3: fp16 input fragments with the
    two-MFMA expand, fp16 residual read, fp16 output) with fp32 hidden tensors, so the oracle restates no hidden
    rounding and block 4 is held to the fp32 bound; the fp16 outputs of blocks 1-3 keep the one-step bound."""
    from spef_amd import _lib as L
    f16_hidden = F16_HIDDEN if mx_kernels else ()
    mx.set_option(L.OPT_MX_KERNELS, mx_kernels)
    fr = _frames(b, h, w, 5 + h)
    x = M.u8_nhwc_to_nchw_f32(fr)
    xg = torch.from_numpy(fr).cuda()
    errs = {}
    try:
        prev = None
        for op in range(0, 18):
            got = mx.probe(xg, op).cpu()
            if op == 0:
                ref = _oracle_block(x, sd, 0)
            elif op == 1:
                ref = _oracle_block(_oracle_block(x, sd, 0), sd, 1)
            else:
                ref = _oracle_block(prev.permute(0, 3, 1, 2).contiguous(), sd, op, f16_hidden)
            if op in F16_BLOCKS:
                ref = ref.half().float()
            ref = ref.permute(0, 2, 3, 1).numpy()
            assert got.shape == ref.shape, (op, got.shape, ref.shape)
            errs[op] = float(np.abs(got.numpy() - ref).max() / max(1e-6, np.abs(ref).max()))
            prev = got
    finally:
        mx.set_option(L.OPT_MX_KERNELS, 1)
    print(f'mx_kernels={mx_kernels} block output error / map max:', {k: f'{v:.1e}' for k, v in errs.items()})
    for op, err in errs.items():
        # fp16 output: one fp16 step; block 4 (fp16 hidden, fp32 output): the hidden tensor's rare one-step rounding
        # differences (values within ~1e-7 of a rounding boundary) carried through depthwise and project; fp32: fp16x2
        assert err < (1.2e-3 if op in F16_BLOCKS else 2e-4 if op in f16_hidden else 5e-5), (op, err)


def test_sharp_head_logits_absolute():
    """The headline schedule at a sharp head (std 0.3: logits to ~20) meets the north star's absolute 1e-3 on the
    logits and the pose bounds, at 512 x 512."""
    from spef_amd.engine import Engine
    sd = _sharp_sd()
    fr = _frames(4, 512, 512, 77)
    torch.set_num_threads(16)
    ro, rp = M.forward(M.u8_nhwc_to_nchw_f32(fr), sd)
    ro, rp = ro.numpy(), rp.numpy()
    h, _ = D.orientation_histogram(12, False)
    rq = D.decode_orientation_batch(D.softmax_f32(ro), h)
    e = Engine(Bl.pack(sd, dtype='fp16mx'), 'cuda:0')
    try:
        e.set_decode_tables(h, None)
        o, p = e.forward(torch.from_numpy(fr).cuda())
        dec = e.decode(1, 0, o, p)
        lo = np.abs(o.cpu().numpy() - ro).max()
        po = np.abs(p.cpu().numpy() - rp).max()
        ao = D.angle_deg_stable(dec['ori'].cpu().numpy().astype(np.float64), rq).max()
    finally:
        e.close()
    print(f'fp16mx sharp head: max|d logit| {lo:.2e}, max|d pos| {po:.2e} m, max {ao:.2e} deg')
    assert np.abs(ro).max() > 5.0
    assert lo < LOGIT_TOL and po < POS_TOL_M and ao < ORI_TOL_DEG


def test_bench_workload_stream_pipeline_sharp_head():
    """The timed configuration itself: B = 64 synthetic SPEED-style 512 x 512 frames (bench.py's generator) through
    StreamPipeline.submit (three streams, forward + decode), sharp head, against the FP32 oracle at the absolute
    north-star bounds -- every batch of the pipeline, not one engine call."""
    from spef_amd import _lib as L
    from spef_amd.pipeline import StreamPipeline
    sd = _sharp_sd()
    fr = synth_frames(64, 512, 512, 10_000)
    torch.set_num_threads(16)
    ro, rp = M.forward(M.u8_nhwc_to_nchw_f32(fr), sd)
    ro, rp = ro.numpy(), rp.numpy()
    h, _ = D.orientation_histogram(12, False)
    rq = D.decode_orientation_batch(D.softmax_f32(ro), h)
    pipe = StreamPipeline(Bl.pack(sd, dtype='fp16mx'), 'cuda:0', depth=3, ori_bins=h)
    try:
        pipe.reserve(64, 512, 512)
        xg = torch.from_numpy(fr).cuda()
        outs = []
        for _ in range(4):   # four steps over the three streams; each output read before its stream is reused
            o = pipe.submit(xg, L.CLASSIFICATION, L.REGRESSION, want_soft=True)
            pipe.synchronize()
            outs.append({k: (v.cpu().numpy() if torch.is_tensor(v) else v) for k, v in o.items()})
    finally:
        pipe.close()
    for o in outs:
        assert not o['status'].any()
        lo = np.abs(o['raw0'] - ro).max()
        po = np.abs(o['pos'] - rp).max()
        ao = D.angle_deg_stable(o['ori'].astype(np.float64), rq).max()
        print(f'B=64 pipeline step: max|d logit| {lo:.2e}, max|d pos| {po:.2e} m, max {ao:.2e} deg')
        assert lo < LOGIT_TOL and po < POS_TOL_M and ao < ORI_TOL_DEG
