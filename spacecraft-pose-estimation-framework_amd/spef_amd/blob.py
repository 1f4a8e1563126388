"""BatchNorm folding and weight packing: reference ``state_dict`` -> SPEF MI355X weight blob.

Input is the reference checkpoint layout (``save_model`` / ``load_state_dict``,
``src/modeling/model.py:70-89, 261-266``; 316 keys for MobileNetV2 + URSONetHead). Output is the
binary blob ``csrc/spef_blob.hpp`` documents -- keep the two in sync.

Folding (eval-mode ``BatchNorm2d``, eps 1e-5, ``pytorch_layers.py:53-56``), done in float64:
    s  = gamma / sqrt(running_var + eps)
    w' = w * s[:, None, None, None]         b' = beta - running_mean * s
Pointwise weights are stored [Np][Kp] in the activation dtype (fp16 default, bf16 variant), zero padded
(Kp = K up to a multiple of 32, Np = N up to a multiple of 16) so the MFMA kernels never mask weight loads.
Depthwise weights are fp16 in fp16 blobs (fp32 in bf16 blobs); stem, bias and head weights stay fp32.

``fp16x2`` (dtype 5, the fp32-accurate fused schedule of csrc/k_x2.hip): every 1x1 weight is stored as two fp16
planes [2][rows][Kp], hi = fp16(w) and lo = fp16(w - hi) of the float64 folded weight (22 significant bits), expand
rows padded to 32; depthwise weights fp32 [9][H32] and the hidden-width biases padded to H32 = hidden rounded up to
32 (zeros), so the kernel never masks a channel; the stem's /255-folded MFMA operand x0 as [2][3 ky][32][32] hi / lo
planes with k = 4 kx + ci (the front kernel's fragment order).

``fp16mx`` (dtype 6, the headline schedule): the fp16x2 layout, plus the stem operand in the fp16 front kernel's
row-triple k order as a second tensor (x1, hi / lo [2][32][32]); the schedule stores the stem map, the block
outputs of blocks 1-3 and the hidden tensors of blocks 2-4 in fp16 and every other activation in fp32, with every
weight exact (tools/precision_budget.py: ~5e-4 max |d logit| at head std 0.3 against 1.3e-2 for the fp16 schedule).
"""
from __future__ import annotations

import struct
from typing import Dict, List, Optional

import numpy as np

from .arch import Arch, BN_EPS, ConvSpec, LAST_CHANNELS, arch_from_state_dict, mobilenet_v2

MAGIC = b'SPEFMI35'
VERSION = 2   # 2: fp16 stem MFMA operand in the front_vp_kernel row-triple k order (csrc/spef_blob.hpp)
DTYPES = {'fp16': 1, 'bf16': 2, 'fp32': 4, 'fp16x2': 5, 'fp16mx': 6}   # fp32: the reference's own arithmetic
# (k_f32.hip); fp16x2: fp32 activations with hi + lo fp16 MFMA operands (k_x2.hip); fp16mx: the same weights,
# fp16 stem map, block outputs of blocks 1-3, hidden tensors of blocks 2-4
X2_DTYPES = ('fp16x2', 'fp16mx')   # the split-fp16 weight layout
DT_I8 = 3
OP_STEM, OP_IRB, OP_LAST, OP_FC, OP_FCKP = 1, 2, 3, 4, 5
OP_QSTEM, OP_QIRB, OP_QLAST, OP_QFC = 11, 12, 13, 14
HEAD_URSONET, HEAD_KEYPOINTS = 0, 1
ABSENT = (1 << 64) - 1
_HDR = struct.Struct('<8sIIII' + 'IIIIII' + 'QQQ' + '56s')
_OP = struct.Struct('<IIIIIIII' + 'QQQQQQ' + 'QQQ' + '24s')
assert _HDR.size == 128 and _OP.size == 128


def _np(v) -> np.ndarray:
    if hasattr(v, 'detach'):
        v = v.detach().cpu().numpy()
    return np.asarray(v)


def fold_bn(sd: Dict, c: ConvSpec):
    """-> (w' float64 [cout, cin/g, k, k], b' float64 [cout])."""
    w = _np(sd[f'{c.prefix}.0.weight']).astype(np.float64)
    g = _np(sd[f'{c.prefix}.1.weight']).astype(np.float64)
    beta = _np(sd[f'{c.prefix}.1.bias']).astype(np.float64)
    mean = _np(sd[f'{c.prefix}.1.running_mean']).astype(np.float64)
    var = _np(sd[f'{c.prefix}.1.running_var']).astype(np.float64)
    s = g / np.sqrt(var + BN_EPS)
    return w * s[:, None, None, None], beta - mean * s


def _to_act(a: np.ndarray, dtype: str) -> bytes:
    a = np.ascontiguousarray(a, dtype=np.float32)
    if dtype == 'fp16':
        return a.astype(np.float16).tobytes()
    if dtype == 'fp32':
        return a.tobytes()
    # bf16: round-to-nearest-even on the fp32 bits (finite weights only)
    u = a.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    return r.tobytes()


def _round_act(a: np.ndarray, dtype: str) -> np.ndarray:
    """float32 -> nearest value of the activation dtype, returned as float32."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    if dtype == 'fp16':
        return a.astype(np.float16).astype(np.float32)
    if dtype == 'fp32':
        return a
    return np.frombuffer(_to_act(a, 'bf16'), np.uint16).astype(np.uint32).__lshift__(16).view(np.float32).reshape(a.shape)


class _Data:
    def __init__(self):
        self.chunks: List[bytes] = []
        self.size = 0

    def add(self, b: bytes) -> int:
        off = self.size
        pad = (-len(b)) % 256
        self.chunks.append(b + b'\0' * pad)
        self.size += len(b) + pad
        return off


def _pw_tensor(w: np.ndarray, b: np.ndarray, dtype: str, data: _Data):
    cout, cin = w.shape[0], w.shape[1]
    kp, np_ = (cin + 31) // 32 * 32, (cout + 15) // 16 * 16
    wp = np.zeros((np_, kp), np.float32)
    wp[:cout, :cin] = w[:, :, 0, 0]
    bp = np.zeros(np_, np.float32)
    bp[:cout] = b
    return data.add(_to_act(wp, dtype)), data.add(bp.tobytes())


def split_f16(a: np.ndarray):
    """float64 / float32 -> (hi, lo) fp16 with hi = fp16(a), lo = fp16(a - hi)."""
    a = np.asarray(a, np.float64)
    hi = a.astype(np.float16)
    return hi, (a - hi.astype(np.float64)).astype(np.float16)


def _pw_x2(w: np.ndarray, b: np.ndarray, data: _Data, rows: int):
    """fp16x2 1x1 weights: [2][rows][Kp] fp16 (hi plane, lo plane), bias fp32 [rows]; zero padded."""
    cout, cin = w.shape[0], w.shape[1]
    kp = (cin + 31) // 32 * 32
    wp = np.zeros((rows, kp), np.float64)
    wp[:cout, :cin] = w[:, :, 0, 0]
    hi, lo = split_f16(wp)
    bp = np.zeros(rows, np.float32)
    bp[:cout] = b
    return data.add(np.concatenate([hi, lo]).tobytes()), data.add(bp.tobytes())


def _dw_x2(w: np.ndarray, b: np.ndarray, data: _Data, hp: int):
    c = w.shape[0]
    w9 = np.zeros((9, hp), np.float32)
    w9[:, :c] = w[:, 0].reshape(c, 9).T
    bb = np.zeros(hp, np.float32)
    bb[:c] = b
    return data.add(w9.tobytes()), data.add(bb.tobytes())


def _dw_tensor(w: np.ndarray, b: np.ndarray, data: _Data, dtype: str):
    """Depthwise weights [9][C] (tap = ky*3+kx): fp16 in fp16 blobs (the kernels' v_fma_mix operand), fp32 in
    bf16 blobs; bias fp32."""
    c = w.shape[0]
    w9 = np.ascontiguousarray(w[:, 0].reshape(c, 9).T, dtype=np.float32)
    w9b = w9.astype(np.float16).tobytes() if dtype == 'fp16' else w9.tobytes()
    return data.add(w9b), data.add(np.asarray(b, np.float32).tobytes())


def pack(sd: Dict, arch: Optional[Arch] = None, dtype: str = 'fp16', kp_feat_hw=(8, 12)) -> bytes:
    """Fold BN and pack a reference-layout state_dict into a blob (bytes). ``arch`` defaults to the topology
    the state_dict's head keys describe (``arch.arch_from_state_dict``)."""
    assert dtype in DTYPES, dtype
    arch = arch or arch_from_state_dict(sd)
    data = _Data()
    ops = []

    # stem: [27][32], k = ky*9 + kx*3 + ci
    w, b = fold_bn(sd, arch.stem)
    ws = np.ascontiguousarray(w.transpose(2, 3, 1, 0).reshape(27, arch.stem.cout), dtype=np.float32)
    # MFMA A operand of the fused front kernel (uint8 input): ToTensor's /255 folded in float32, split
    # hi + lo in the activation dtype, [2][32 ch][32 k]. bf16: k = ky*9 + kx*3 + ci (27..31 zero). fp16: the front
    # kernel's Lr order (k_front.hip front_vp_kernel) -- k = 2 d + h, dword d = 3 c + ky (c < 5), half h: tap
    # j = 2 c + h = kx*3 + ci of input row ky (j = 9 and d = 15 are zero-weight pads)
    w255 = ws / np.float32(255.0)
    hi = np.zeros((arch.stem.cout, 32), np.float32)
    if dtype in ('fp16', 'fp16mx'):
        for k in range(30):
            d, h = divmod(k, 2)
            c, ky = divmod(d, 3)
            j = 2 * c + h
            if j < 9:
                hi[:, k] = w255[ky * 9 + j]
    else:
        hi[:, :27] = w255.T
    x1 = None
    if dtype in X2_DTYPES:   # x2_front_kernel's operand: [plane][ky][32 ch][32 k], k = 4 kx + ci (k >= 12 zero)
        a = np.zeros((3, arch.stem.cout, 32), np.float64)
        for ky in range(3):
            for kx in range(3):
                for ci in range(3):
                    a[ky, :, 4 * kx + ci] = w255[ky * 9 + kx * 3 + ci]
        x0 = np.concatenate(split_f16(a)).tobytes()
        if dtype == 'fp16mx':   # + the fp16 front kernel's row-triple k order, hi / lo [2][32][32] (front_mx_kernel)
            x1 = data.add(np.concatenate(split_f16(hi)).tobytes())
    else:
        hi_r = _round_act(hi, dtype)
        x0 = _to_act(np.concatenate([hi_r, _round_act(hi - hi_r, dtype)]), dtype)
    stem = (OP_STEM, 3, arch.stem.cout, 0, 2, 1, 0,
            data.add(ws.tobytes()), data.add(np.asarray(b, np.float32).tobytes()), ABSENT, ABSENT, ABSENT, ABSENT,
            data.add(x0))
    ops.append(stem if x1 is None else stem + (x1,))

    for blk in arch.blocks:
        convs = list(blk.convs)
        if dtype in X2_DTYPES:
            hp = (blk.hidden + 31) // 32 * 32
            e = (ABSENT, ABSENT)
            if blk.expand != 1:
                e = _pw_x2(*fold_bn(sd, convs.pop(0)), data, hp)
            d = _dw_x2(*fold_bn(sd, convs[0]), data, hp)
            p = _pw_x2(*fold_bn(sd, convs[1]), data, (blk.cout + 15) // 16 * 16)
            ops.append((OP_IRB, blk.cin, blk.cout, blk.hidden, blk.stride, blk.expand, 1 if blk.residual else 0,
                        e[0], e[1], d[0], d[1], p[0], p[1]))
            continue
        e = (ABSENT, ABSENT)
        if blk.expand != 1:
            e = _pw_tensor(*fold_bn(sd, convs.pop(0)), dtype, data)
        d = _dw_tensor(*fold_bn(sd, convs[0]), data, dtype)
        p = _pw_tensor(*fold_bn(sd, convs[1]), dtype, data)
        ops.append((OP_IRB, blk.cin, blk.cout, blk.hidden, blk.stride, blk.expand, 1 if blk.residual else 0,
                    e[0], e[1], d[0], d[1], p[0], p[1]))

    if dtype in X2_DTYPES:
        lw, lb = _pw_x2(*fold_bn(sd, arch.last), data, (arch.last.cout + 15) // 16 * 16)
    else:
        lw, lb = _pw_tensor(*fold_bn(sd, arch.last), dtype, data)
    ops.append((OP_LAST, arch.last.cin, arch.last.cout, 0, 1, 1, 0, lw, lb, ABSENT, ABSENT, ABSENT, ABSENT))

    if arch.head == 'ursonet':
        wo, bo = _np(sd['head.ori.1.weight']), _np(sd['head.ori.1.bias'])
        wpos, bpos = _np(sd['head.pos.0.weight']), _np(sd['head.pos.0.bias'])
        n = wo.shape[0] + wpos.shape[0]
        np_ = (n + 15) // 16 * 16
        wf = np.zeros((np_, LAST_CHANNELS), np.float32)
        wf[:wo.shape[0]] = wo
        wf[wo.shape[0]:n] = wpos
        bf = np.zeros(np_, np.float32)
        bf[:wo.shape[0]] = bo
        bf[wo.shape[0]:n] = bpos
        ops.append((OP_FC, LAST_CHANNELS, n, 0, 1, 1, 0, data.add(wf.tobytes()), data.add(bf.tobytes()),
                    ABSENT, ABSENT, ABSENT, ABSENT))
        head, n0, n1, fh, fw = HEAD_URSONET, wo.shape[0], wpos.shape[0], 0, 0
    else:
        fh, fw = kp_feat_hw
        wk, bk = _np(sd['head.layer.1.weight']), _np(sd['head.layer.1.bias'])
        n = wk.shape[0]
        assert wk.shape[1] == LAST_CHANNELS * fh * fw, 'keypoint head size / feature map mismatch'
        # torch.flatten of NCHW (keypoints.py:25) -> our NHWC flatten order
        wn = wk.reshape(n, LAST_CHANNELS, fh, fw).transpose(0, 2, 3, 1).reshape(n, -1)
        np_ = (n + 15) // 16 * 16
        wf = np.zeros((np_, wn.shape[1]), np.float32)
        wf[:n] = wn
        bf = np.zeros(np_, np.float32)
        bf[:n] = bk
        ops.append((OP_FCKP, wn.shape[1], n, 0, 1, 1, 0, data.add(wf.tobytes()), data.add(bf.tobytes()),
                    ABSENT, ABSENT, ABSENT, ABSENT))
        head, n0, n1 = HEAD_KEYPOINTS, n, 0

    return assemble(DTYPES[dtype], head, n0, n1, fh, fw, ops, data)


def assemble(dtype_code: int, head: int, n0: int, n1: int, fh: int, fw: int, ops, data: _Data) -> bytes:
    """Header + op table + data section. An op is (kind, cin, cout, hidden, stride, expand, flags,
    w0, b0, w1, b1, w2, b2[, x0, x1, x2[, qbits]]) with qbits up to 4 quantizer widths (int8 ops)."""
    ops_off = _HDR.size
    data_off = ops_off + _OP.size * len(ops)
    data_off += (-data_off) % 256
    hdr = _HDR.pack(MAGIC, VERSION, dtype_code, head, len(ops), n0, n1, LAST_CHANNELS, fh, fw, 0,
                    ops_off, data_off, data.size, b'\0' * 56)
    out = bytearray(hdr)
    for o in ops:
        x = tuple(o[13:16]) + (ABSENT,) * (16 - max(13, min(len(o), 16)))
        qb = bytes(o[16]) if len(o) > 16 else b''
        out += _OP.pack(*o[:7], 0, *o[7:13], *x, qb + b'\0' * (24 - len(qb)))
    out += b'\0' * (data_off - len(out))
    for ch in data.chunks:
        out += ch
    return bytes(out)


def describe(blob: bytes) -> dict:
    """Parse a blob header + op table (for tests and tooling)."""
    h = _HDR.unpack_from(blob, 0)
    if h[0] != MAGIC:
        raise ValueError('not a SPEF MI355X blob')
    info = dict(version=h[1], dtype=h[2], head=h[3], n_ops=h[4], n_out0=h[5], n_out1=h[6], feat_c=h[7],
                kp_fh=h[8], kp_fw=h[9], ops_off=h[11], data_off=h[12], data_bytes=h[13])
    info['ops'] = [_OP.unpack_from(blob, info['ops_off'] + i * _OP.size)[:17] for i in range(info['n_ops'])]
    return info
