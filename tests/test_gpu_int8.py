"""INT8 path (C5) on the GPU vs oracle/int8_ref.py: BIT-EXACT integer activations and head outputs.

Parity vs Brevitas itself is unpinned (brevitas absent; see oracle/int8_ref.py); the integer semantics are
pinned here, and their distance to the float fake-quant graph and to FP32 is measured in test_int8_oracle.py.
"""
import numpy as np
import pytest
import torch

from bench import synth_frames
from oracle import int8_ref as Q
from oracle import model_ref as M
from spef_amd.arch import mobilenet_v2
from spef_amd.blob_q8 import pack_int8
from spef_amd.quant import calibrate
from spef_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def q8():
    from spef_amd.engine import Engine
    sd = synthetic_state_dict(mobilenet_v2(), seed=1001)
    qp = calibrate(sd, synth_frames(4, 128, 128, 900))
    e = Engine(pack_int8(sd, qp), 'cuda:0')
    yield e, sd, qp
    e.close()


def _nhwc(a):
    return a.transpose(0, 2, 3, 1)


@pytest.mark.parametrize('b,h,w', [(2, 64, 64), (1, 128, 96)])
def test_int8_activations_bit_exact(q8, b, h, w):
    eng, sd, qp = q8
    fr = synth_frames(b, h, w, 7)
    x = torch.from_numpy(fr).cuda()
    for op in (0, 1, 2, 3, 5, 8, 12, 16, 17):
        got = eng.probe(x, op).cpu().numpy()
        ref = _nhwc(Q.int8_forward(fr, sd, qp, upto=op))
        assert got.shape == ref.shape, op
        np.testing.assert_array_equal(got, ref.astype(np.float32), err_msg=f'op {op}')


@pytest.mark.parametrize('b,h,w', [(2, 64, 64), (3, 96, 128), (1, 512, 512)])
def test_int8_head_outputs_bit_exact(q8, b, h, w):
    eng, sd, qp = q8
    fr = synth_frames(b, h, w, 11)
    o, p = eng.forward(torch.from_numpy(fr).cuda())
    ro, rp = Q.int8_forward(fr, sd, qp)
    np.testing.assert_array_equal(o.cpu().numpy(), ro)
    np.testing.assert_array_equal(p.cpu().numpy(), rp)


@pytest.mark.parametrize('b,h,w', [(2, 64, 64), (1, 100, 136), (2, 512, 512)])
def test_int8_role_split_blocks_bit_identical_to_slab(q8, b, h, w):
    """SPEF_OPT_Q8_ROLESPLIT 1 runs blocks 8-17 as role-split kernels (k_q8irw.hip), 0 (default) as slab kernels
    (k_q8irb.hip). Every late-block output is bit-identical (ragged maps included)."""
    from spef_amd import _lib as L
    eng, sd, qp = q8
    x = torch.from_numpy(synth_frames(b, h, w, 21)).cuda()
    try:
        for op in range(8, 18):
            outs = []
            for mode in (1, 0):
                eng.set_option(L.OPT_Q8_ROLESPLIT, mode)
                outs.append(eng.probe(x, op).cpu().numpy())
            np.testing.assert_array_equal(outs[0], outs[1], err_msg=f'op {op}')
    finally:
        eng.set_option(L.OPT_Q8_ROLESPLIT, 0)


def test_int8_f32_input_matches_u8(q8):
    """NCHW float32 [0,1] input (the reference `images['torch']`) quantises to the same codes as the u8 LUT."""
    eng, sd, qp = q8
    fr = synth_frames(2, 64, 96, 3)
    o8, p8 = eng.forward(torch.from_numpy(fr).cuda())
    of, pf = eng.forward(M.u8_nhwc_to_nchw_f32(fr).contiguous().cuda())
    np.testing.assert_array_equal(o8.cpu().numpy(), of.cpu().numpy())
    np.testing.assert_array_equal(p8.cpu().numpy(), pf.cpu().numpy())


def test_int8_batch_64_512(q8):
    """C5 shape (B=64, 512x512): outputs equal the oracle on a sample of rows (rows are independent)."""
    eng, sd, qp = q8
    fr = synth_frames(64, 512, 512, 100)
    o, p = eng.forward(torch.from_numpy(fr).cuda())
    idx = [0, 37, 63]
    ro, rp = Q.int8_forward(fr[idx], sd, qp)
    np.testing.assert_array_equal(o.cpu().numpy()[idx], ro)
    np.testing.assert_array_equal(p.cpu().numpy()[idx], rp)


def test_int8_general_shift_kernels_bit_exact(q8):
    """The fused blocks' general-shift variant (blob flag 4 cleared) gives the same bits as the shift-free one."""
    from spef_amd.engine import Engine
    _, sd, qp = q8
    fr = synth_frames(2, 96, 64, 13)
    e = Engine(pack_int8(sd, qp, shift32=False), 'cuda:0')
    try:
        ro, rp = Q.int8_forward(fr, sd, qp)
        from spef_amd import _lib as L
        for rolesplit in (0, 1):   # slab and role-split late blocks, general-shift requant
            e.set_option(L.OPT_Q8_ROLESPLIT, rolesplit)
            o, p = e.forward(torch.from_numpy(fr).cuda())
            np.testing.assert_array_equal(o.cpu().numpy(), ro)
            np.testing.assert_array_equal(p.cpu().numpy(), rp)
    finally:
        e.close()


def _mixed_widths():
    from spef_amd.quant import parse_bit_width
    return parse_bit_width({'image': '6', 'first_conv': '(4, 5)', 'last_conv': '(5, 4)', 'fully_connected': '(6, 7)',
                            'shared_act': '5', 'pooling': '7',
                            'inverted_residual': ['[(None, None), (6, 5), (7,)]'] +
                                                 ['[(5, 4), (6, 3), (4,)]', '[(3, 6), (4, 7), (5,)]'] * 8})


@pytest.fixture(scope='module', params=['qmobilenet_default', 'mixed'])
def q8low(request):
    """Sub-8-bit quantizers in int8 containers (f2): the reference QMobileNetV2's default 3-bit / 4-bit-shared
    config (mobilenet_v2.py:140-167) and a mixed 3..7-bit bit_width.json."""
    from spef_amd.engine import Engine
    from spef_amd.quant import BitWidths
    sd = synthetic_state_dict(mobilenet_v2(), seed=1001)
    bw = BitWidths.qmobilenet_default() if request.param == 'qmobilenet_default' else _mixed_widths()
    qp = calibrate(sd, synth_frames(4, 128, 128, 900), bw=bw)
    e = Engine(pack_int8(sd, qp), 'cuda:0')
    yield e, sd, qp
    e.close()


def test_low_bit_activations_bit_exact(q8low):
    eng, sd, qp = q8low
    fr = synth_frames(2, 96, 64, 17)
    x = torch.from_numpy(fr).cuda()
    for op in (0, 1, 2, 3, 5, 8, 12, 14, 16, 17):
        got = eng.probe(x, op).cpu().numpy()
        ref = _nhwc(Q.int8_forward(fr, sd, qp, upto=op))
        np.testing.assert_array_equal(got, ref.astype(np.float32), err_msg=f'op {op}')


def test_low_bit_head_outputs_bit_exact(q8low):
    """u8 frames and float NCHW frames (input quantizer of the configured width), and the general-shift fused
    variant: every output bit-identical to the oracle."""
    from spef_amd.engine import Engine
    eng, sd, qp = q8low
    fr = synth_frames(3, 128, 96, 19)
    ro, rp = Q.int8_forward(fr, sd, qp)
    o, p = eng.forward(torch.from_numpy(fr).cuda())
    np.testing.assert_array_equal(o.cpu().numpy(), ro)
    np.testing.assert_array_equal(p.cpu().numpy(), rp)
    of, pf = eng.forward(M.u8_nhwc_to_nchw_f32(fr).contiguous().cuda())
    np.testing.assert_array_equal(of.cpu().numpy(), ro)
    np.testing.assert_array_equal(pf.cpu().numpy(), rp)
    e = Engine(pack_int8(sd, qp, shift32=False), 'cuda:0')
    from spef_amd import _lib as L
    try:
        for rolesplit in (0, 1):   # low-bit quantizers through the role-split late blocks as well
            e.set_option(L.OPT_Q8_ROLESPLIT, rolesplit)
            eng.set_option(L.OPT_Q8_ROLESPLIT, rolesplit)
            for en in (e, eng):
                o2, p2 = en.forward(torch.from_numpy(fr).cuda())
                np.testing.assert_array_equal(o2.cpu().numpy(), ro)
                np.testing.assert_array_equal(p2.cpu().numpy(), rp)
    finally:
        eng.set_option(L.OPT_Q8_ROLESPLIT, 0)
        e.close()


def test_low_bit_unfused_schedule_bit_exact(q8low):
    """The one-kernel-per-conv int8 schedule honours the same widths (stem, GEMM epilogues, depthwise, pool)."""
    eng, sd, qp = q8low
    fr = synth_frames(2, 64, 96, 23)
    ro, rp = Q.int8_forward(fr, sd, qp)
    eng.set_fused(False)
    try:
        o, p = eng.forward(torch.from_numpy(fr).cuda())
    finally:
        eng.set_fused(True)
    np.testing.assert_array_equal(o.cpu().numpy(), ro)
    np.testing.assert_array_equal(p.cpu().numpy(), rp)
