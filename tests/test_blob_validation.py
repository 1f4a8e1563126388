"""spef_validate_blob (host-only C ABI): every blob the packers emit validates; truncated or corrupted blobs are
rejected before anything would reach the device (the same checks run inside spef_load_weights[_device])."""
import ctypes as C
import struct

import pytest

from spef_amd import _lib as L
from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.weights import synthetic_state_dict


def _validate(b: bytes):
    lib = L.load()
    dt, hd, n0, n1 = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    rc = lib.spef_validate_blob(C.create_string_buffer(b, len(b)), len(b), C.byref(dt), C.byref(hd), C.byref(n0),
                                C.byref(n1))
    return rc, (dt.value, hd.value, n0.value, n1.value), lib.spef_last_error().decode()


@pytest.fixture(scope='module')
def fp16_blob():
    return Bl.pack(synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=7), dtype='fp16')


@pytest.mark.parametrize('head,n0,n1,dtype', [('ursonet', 1728, 3, 'fp16'), ('ursonet', 1232, 1000, 'bf16'),
                                              ('ursonet', 4, 3, 'fp16'), ('keypoints', 24, 0, 'fp16')])
def test_packed_blobs_validate(head, n0, n1, dtype):
    arch = mobilenet_v2(head, n0, n1) if head == 'ursonet' else mobilenet_v2('keypoints')
    b = Bl.pack(synthetic_state_dict(arch, seed=3), arch, dtype=dtype)
    rc, info, msg = _validate(b)
    assert rc == L.OK, msg
    assert info == (Bl.DTYPES[dtype], Bl.HEAD_URSONET if head == 'ursonet' else Bl.HEAD_KEYPOINTS, n0, n1)


def test_int8_blob_validates():
    from spef_amd.blob_q8 import pack_int8
    from spef_amd.data.synthetic import synth_frames
    from spef_amd.quant import calibrate
    sd = synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=3)
    qp = calibrate(sd, synth_frames(2, 64, 64, 900))
    for shift32 in (True, False):
        rc, info, msg = _validate(pack_int8(sd, qp, shift32=shift32))
        assert rc == L.OK, msg
        assert info == (Bl.DT_I8, Bl.HEAD_URSONET, 1728, 3)


def test_truncated_blob_rejected(fp16_blob):
    for cut in (1, 4096, len(fp16_blob) - 200):
        rc, _, msg = _validate(fp16_blob[:-cut])
        assert rc == L.ERR_BLOB and 'truncated' in msg, (cut, msg)


def test_bad_magic_rejected(fp16_blob):
    rc, _, msg = _validate(b'X' + fp16_blob[1:])
    assert rc == L.ERR_BLOB and 'magic' in msg


def test_tensor_extent_past_data_section_rejected(fp16_blob):
    """An offset inside the data section whose tensor runs past its end (the check parse_blob lacked before)."""
    info = Bl.describe(fp16_blob)
    op = info['ops'][-1]                                         # the FC head: w0 [1744][1280] fp32
    data_bytes = info['data_bytes']
    bad_off = (data_bytes - 1024) // 256 * 256                   # aligned, in range, but far too short for w0
    pos = info['ops_off'] + (info['n_ops'] - 1) * 128 + 32       # w0 follows the eight uint32 fields
    b = bytearray(fp16_blob)
    struct.pack_into('<Q', b, pos, bad_off)
    assert op[0] == Bl.OP_FC
    rc, _, msg = _validate(bytes(b))
    assert rc == L.ERR_BLOB and 'extent' in msg, msg


def test_head_width_mismatch_rejected(fp16_blob):
    b = bytearray(fp16_blob)
    struct.pack_into('<I', b, 24, 1232)                          # header n_out0 != FC rows - 3
    rc, _, msg = _validate(bytes(b))
    assert rc == L.ERR_BLOB and 'head' in msg, msg


def test_ops_offset_overflow_rejected(fp16_blob):
    """ops_off near 2^64 must not wrap ops_off + n_ops * 128 into range (the memcpy would read before the buffer)."""
    b = bytearray(fp16_blob)
    struct.pack_into('<Q', b, 48, 0xFFFFFFFFFFFFFFC0)             # header ops_off (after 8s + 10 uint32)
    rc, _, msg = _validate(bytes(b))
    assert rc == L.ERR_BLOB and 'truncated' in msg, msg


def test_old_blob_version_rejected(fp16_blob):
    """Version 1 blobs hold the fp16 stem operand in the old k order: they must fail to load, not run wrongly."""
    assert struct.unpack_from('<I', fp16_blob, 8)[0] == Bl.VERSION == 2
    b = bytearray(fp16_blob)
    struct.pack_into('<I', b, 8, 1)
    rc, _, msg = _validate(bytes(b))
    assert rc == L.ERR_BLOB and 'version' in msg, msg


@pytest.mark.parametrize('bits', [1, 2, 9])
def test_int8_qbits_outside_3_to_8_rejected(bits):
    """The C validator and quant.check_bit_width agree: widths 1-2 (Brevitas binary / ternary quantizers,
    quantizers.py:85-88) change the arithmetic, so only 0 (= 8) or 3..8 are accepted."""
    from spef_amd.blob_q8 import pack_int8
    from spef_amd.data.synthetic import synth_frames
    from spef_amd.quant import calibrate
    sd = synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=3)
    good = pack_int8(sd, calibrate(sd, synth_frames(2, 64, 64, 900)))
    info = Bl.describe(good)
    b = bytearray(good)
    struct.pack_into('<B', b, info['ops_off'] + 1 * 128 + 104, bits)   # op 1 (first QIRB): qbits[0]
    rc, _, msg = _validate(bytes(b))
    assert rc == L.ERR_BLOB and 'bit widths' in msg, msg
