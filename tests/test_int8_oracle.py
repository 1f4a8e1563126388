"""INT8 oracle and packer on the CPU: integer semantics vs the Brevitas float fake-quant graph and FP32,
blob structure, bit-width config handling."""
import numpy as np
import pytest

from bench import synth_frames
from oracle import int8_ref as Q
from oracle import model_ref as M
from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.blob_q8 import pack_int8
from spef_amd.quant import calibrate, check_bit_width, validate
from spef_amd.weights import synthetic_state_dict


@pytest.fixture(scope='module')
def model():
    sd = synthetic_state_dict(mobilenet_v2(), seed=1001)
    qp = calibrate(sd, synth_frames(4, 128, 128, 900))
    validate(qp)
    return sd, qp


def test_integer_semantics_close_to_fake_quant(model):
    """The fixed-point requant differs from Brevitas' float graph only by rare 1-LSB rounding flips; measured
    on the head outputs (parity vs Brevitas itself is unpinned: brevitas is absent)."""
    sd, qp = model
    fr = synth_frames(2, 96, 96, 5)
    o, p = Q.int8_forward(fr, sd, qp)
    fo, fp = Q.fake_quant_forward(fr, sd, qp)
    scale = np.abs(fo.numpy()).max()
    assert np.abs(o - fo.numpy()).max() < 0.05 * scale
    stem_i = Q.int8_forward(fr, sd, qp, upto=0)
    assert stem_i.min() >= 0 and stem_i.max() <= 255


def test_int8_vs_fp32_accuracy(model):
    """INT8 (calibrated PTQ stand-in for QAT) vs the FP32 model: logits within a few percent of their range."""
    sd, qp = model
    fr = synth_frames(2, 128, 128, 77)
    o, p = Q.int8_forward(fr, sd, qp)
    ro, rp = M.forward(M.u8_nhwc_to_nchw_f32(fr), sd)
    assert np.abs(o - ro.numpy()).max() < 0.06 * np.abs(ro.numpy()).max()
    assert np.abs(p - rp.numpy()).max() < 0.1 * np.abs(rp.numpy()).max()


def test_pack_int8_structure(model):
    sd, qp = model
    info = Bl.describe(pack_int8(sd, qp))
    assert info['dtype'] == Bl.DT_I8 and info['n_out0'] == 1728 and info['n_out1'] == 3
    kinds = [o[0] for o in info['ops']]
    assert kinds == [Bl.OP_QSTEM] + [Bl.OP_QIRB] * 17 + [Bl.OP_QLAST, Bl.OP_QFC]
    res = [o[6] & 1 for o in info['ops'][1:18]]
    assert sum(res) == 10                                   # residual blocks of MobileNetV2
    assert info['ops'][1][6] & 2                            # block 1 takes the unsigned stem output
    assert all(o[14] != Bl.ABSENT for o in info['ops'][1:18])   # projection init present


def test_fixed_point_requant_matches_float():
    rng = np.random.default_rng(0)
    m = rng.uniform(1e-6, 1.0, 64) * rng.choice([-1, 1], 64)
    b = rng.uniform(-300, 300, 64)
    M_, B_, S_ = Q.fixed(m, b)
    # accumulators whose requantised value lands in (or near) the 8-bit range, as in the network
    acc = np.rint(rng.uniform(-400, 400, (1000, 64)) / np.abs(m) - b / m).astype(np.int64)
    got = Q.requant(acc, M_, B_, S_, -128, 255)
    want = np.clip(np.floor(acc * m + b + 0.5), -128, 255)
    assert np.abs(got - want).max() <= 1 and (got != want).mean() < 1e-4


def test_bit_width_config(golden):
    """bit_width.json (model.py:16-45 string format) -> BitWidths: the reference's exp_1 file is all 8; the
    QMobileNetV2 built-in default (mobilenet_v2.py:140-167) is 3-bit with a 4-bit shared quantizer; widths 1-2
    (Brevitas binary / ternary quantizers) are rejected, as are malformed block lists."""
    from spef_amd.quant import BitWidths, parse_bit_width
    exp1 = {'image': '8', 'first_conv': '(8, 8)', 'last_conv': '(8, 8)', 'fully_connected': '(8, 8)',
            'shared_act': '8', 'pooling': '8', 'inverted_residual': ['[(8, 8), (8, 8), (8,)]'] * 17}
    assert parse_bit_width(exp1) == BitWidths() and check_bit_width(exp1) == BitWidths()
    q = BitWidths.qmobilenet_default()
    assert q.block(0) == (None, None, 3, 3, 3) and q.block(16) == (3, 3, 3, 3, 3) and q.shared_act == 4
    mixed = dict(exp1, first_conv='(4, 5)', inverted_residual=['[(None, None), (6, 5), (7,)]'] +
                 ['[(5, 4), (6, 3), (4,)]'] * 16)
    bw = parse_bit_width(mixed)
    assert bw.first_conv == (4, 5) and bw.block(3) == (5, 4, 6, 3, 4)
    with pytest.raises(NotImplementedError):
        check_bit_width(dict(exp1, shared_act='2'))
    with pytest.raises(ValueError):
        parse_bit_width(dict(exp1, inverted_residual=['[(8, 8), (8, 8), (8,)]']))


def test_low_bit_widths_oracle_and_blob(model):
    """3/4-bit (QMobileNetV2 default): codes stay inside each quantizer's range, the blob carries the widths in
    each op's qbits, and the integer network still tracks the FP32 model's head outputs."""
    from spef_amd.quant import BitWidths
    sd, _ = model
    bw = BitWidths.qmobilenet_default()
    qp = calibrate(sd, synth_frames(4, 128, 128, 900), bw=bw)
    validate(qp)
    fr = synth_frames(2, 64, 64, 5)
    stem = Q.int8_forward(fr, sd, qp, upto=0)
    assert stem.min() >= 0 and stem.max() <= 7
    for op in (1, 4, 10, 17):
        a = Q.int8_forward(fr, sd, qp, upto=op)
        assert a.min() >= -8 and a.max() <= 7, op
    last = Q.int8_forward(fr, sd, qp, upto='last')
    assert last.min() >= 0 and last.max() <= 7
    info = Bl.describe(pack_int8(sd, qp))
    raw = pack_int8(sd, qp)
    qb = [raw[info['ops_off'] + i * Bl._OP.size + 104: info['ops_off'] + i * Bl._OP.size + 108]
          for i in range(info['n_ops'])]
    assert qb[0][:2] == bytes([3, 8]) and qb[2][:3] == bytes([3, 3, 4]) and qb[18][:2] == bytes([3, 8])
    assert qb[19][:1] == bytes([8])
    o, p = Q.int8_forward(fr, sd, qp)
    fo, fp = Q.fake_quant_forward(fr, sd, qp)
    assert np.abs(o - fo.numpy()).max() < 0.05 * np.abs(fo.numpy()).max()


def test_fixed_point_shift_rule():
    """sh = 32 exactly for 2**-12 <= |m| < 0.5 (the fused kernels' shift-free requant), finer shifts below."""
    M_, B_, S_ = Q.fixed(np.array([0.3, 1e-2, 2.0 ** -12, 1e-5, 0.7]), np.zeros(5))
    assert list(S_[:3]) == [32, 32, 32] and S_[3] > 32 and S_[4] < 32
    assert np.all(np.abs(M_) < 2 ** 31)


def test_int8_pose_error_within_int8_bound(model):
    """The INT8 accuracy bound the bench reports against (bench.py INT8_BOUND): pose decoded
    from the integer network vs from FP32 on the same frames (8 SPEED-style frames at 256x256)."""
    import bench
    from oracle import decode_ref as D
    sd, qp = model
    fr = synth_frames(8, 256, 256, 10000)
    o, p = Q.int8_forward(fr, sd, qp)
    ro, rp = M.forward(M.u8_nhwc_to_nchw_f32(fr), sd)
    h, _ = D.orientation_histogram(12, False)
    ang = D.angle_deg_stable(D.decode_orientation_batch(D.softmax_f32(o), h),
                             D.decode_orientation_batch(D.softmax_f32(ro.numpy()), h))
    lb, pb, ab = bench.INT8_BOUND
    assert np.abs(o - ro.numpy()).max() < lb and np.abs(p - rp.numpy()).max() < pb and ang.max() < ab


def test_mse_calibration_option(model):
    """calibrate(method='mse') (quantisation-MSE-optimal clip per tensor) gives valid scales and stays within the
    same accuracy class."""
    sd, _ = model
    qp = calibrate(sd, synth_frames(2, 96, 96, 900), method='mse')
    validate(qp)
    fr = synth_frames(2, 96, 96, 31)
    o, _ = Q.int8_forward(fr, sd, qp)
    ro, _ = M.forward(M.u8_nhwc_to_nchw_f32(fr), sd)
    assert np.abs(o - ro.numpy()).max() < 0.08 * np.abs(ro.numpy()).max()
