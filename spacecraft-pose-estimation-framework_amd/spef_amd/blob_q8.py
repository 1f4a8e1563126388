"""INT8 weight blob: reference ``state_dict`` + activation scales (``quant.QParams``) -> blob dtype 3.

Quantisation follows the reference's Brevitas layers (quantizers.py:16-20 per-channel int8 weights; the
conv -> BatchNorm -> QuantReLU / shared-quantizer chain of brevitas_layers.py:10-136) in the integer form the
MI355X kernels execute (csrc/k_q8.hip); the formulas are written out in oracle/int8_ref.py's header and the
op layout in csrc/spef_blob.hpp. Everything is computed in float64 on the host, once:

  * weights: s_w[c] = max|W[c]| / L, q_w = clip(rint(W / s_w), -L, L), L = 2^(b-1) - 1 (127 at 8 bits)
  * bit widths (qp['bits'], bit_width.json as quant.BitWidths): weights quantised here; the activation
    quantizers' widths go into each op's qbits (spef_blob.hpp) and set the kernels' clamp ranges
  * conv + BN + quant: m = (s_in * s_w * g) / s_out, b = h / s_out  (g = gamma/sqrt(var+eps), h = beta - mean*g),
    as fixed point (M, B, sh): q = (acc * M + B) >> sh
  * unsigned MFMA operands are stored offset by -128; the accumulator starts at 128 * sum_k q_w
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np

from .arch import Arch, LAST_CHANNELS, arch_from_state_dict
from .blob import ABSENT, DT_I8, HEAD_URSONET, OP_QFC, OP_QIRB, OP_QLAST, OP_QSTEM, _Data, _np, assemble
from .quant import BitWidths, validate

BN_EPS = 1e-5


def weight_q(w, bits: int = 8):
    w = _np(w).astype(np.float64)
    L = (1 << (bits - 1)) - 1
    s = np.maximum(np.abs(w.reshape(w.shape[0], -1)).max(axis=1) / L, 2e-16)
    q = np.clip(np.rint(w / s.reshape((-1,) + (1,) * (w.ndim - 1))), -L, L).astype(np.int64)
    return q, s


def _bn(sd, prefix):
    g = _np(sd[f'{prefix}.1.weight']).astype(np.float64) / np.sqrt(
        _np(sd[f'{prefix}.1.running_var']).astype(np.float64) + BN_EPS)
    h = _np(sd[f'{prefix}.1.bias']).astype(np.float64) - _np(sd[f'{prefix}.1.running_mean']).astype(np.float64) * g
    return g, h


def fixed(m, b):
    """x * m + b in fixed point: (M, B incl. rounding half, sh): sh = 32 when 2**-12 <= |m| < 0.5, otherwise
    |m| 2**sh in [2**29, 2**30); |b| 2**sh < 2**61 (oracle/int8_ref.fixed states the same rule)."""
    m = np.atleast_1d(np.asarray(m, np.float64))
    b = np.broadcast_to(np.atleast_1d(np.asarray(b, np.float64)), m.shape)
    M = np.zeros(m.shape, np.int64)
    B = np.zeros(m.shape, np.int64)
    S = np.zeros(m.shape, np.int64)
    for i in range(m.size):
        em = math.frexp(abs(m[i]))[1] if m[i] != 0 else -30
        eb = math.frexp(abs(b[i]))[1] if b[i] != 0 else -200
        sh0 = 30 - em
        if 2.0 ** -12 <= abs(m[i]) < 0.5:
            # sh = 32 exactly: M = rint(m 2**32) in [2**20, 2**31) keeps the requant error below 2**-13 LSB for
            # outputs in the 8-bit range, and the fused kernels take the high word of acc * M + B with no shift
            sh0 = 32
        sh = int(min(sh0, 61 - eb, 62))
        if sh < 1:
            raise ValueError(f'requant scale out of range (m={m[i]}, b={b[i]})')
        M[i] = int(np.rint(math.ldexp(m[i], sh)))
        B[i] = int(np.rint(math.ldexp(b[i], sh))) + (1 << (sh - 1))
        S[i] = sh
    return M, B, S


def _rq(data: _Data, M, B, S) -> int:
    n = M.size
    np_ = (n + 15) // 16 * 16
    m = np.zeros(np_, np.int64)
    bb = np.zeros(np_, np.int64)
    ss = np.ones(np_, np.int32)
    m[:n], bb[:n], ss[:n] = M, B, S
    return data.add(m.tobytes() + bb.tobytes() + ss.tobytes())


def _conv(sd, prefix, s_in, s_out, wbits: int = 8):
    q, s_w = weight_q(sd[f'{prefix}.0.weight'], wbits)
    g, h = _bn(sd, prefix)
    return q, fixed((s_in * s_w * g) / s_out, h / s_out)


def _pw(data: _Data, q):
    """int8 [Np][Kp64] (zero padded) + the offset-correction init 128 * sum_k q_w as int32 [Np]."""
    cout, cin = q.shape[0], q.shape[1]
    kp, np_ = (cin + 63) // 64 * 64, (cout + 15) // 16 * 16
    w = np.zeros((np_, kp), np.int8)
    w[:cout, :cin] = q.reshape(cout, cin)
    init = np.zeros(np_, np.int32)
    init[:cout] = 128 * q.reshape(cout, cin).sum(axis=1)
    return data.add(w.tobytes()), init


def _rq16(M, B, S, n_pad: int) -> bytes:
    """RQ16 records {int32 M, int32 S, int64 B} over n_pad channels (padding: M = B = 0, S = 1 -> 0)."""
    rec = np.zeros(n_pad, dtype=[('M', '<i4'), ('S', '<i4'), ('B', '<i8')])
    rec['S'] = 1
    n = M.size
    assert np.all(np.abs(M) < 2 ** 31)
    rec['M'][:n], rec['S'][:n], rec['B'][:n] = M, S, B
    return rec.tobytes()


def _fused_tables(e_rq, d_rq, p_rq, qdw, hidden: int, cout: int) -> bytes:
    """x2 of an expand block: the fused int8 kernel's per-channel tables (spef_blob.hpp).

    The fused kernel keeps each hidden u8 value n in LDS as the fp16 number 1024 + n (bit pattern 0x6400 | n: no
    int -> float conversion in the expand epilogue), so its depthwise sum is acc + 1024 * sum_taps q_wd. The
    depthwise requant offset absorbs that exactly: B' = B - 1024 * M * sum_taps q_wd (same q for every acc)."""
    h32 = (hidden + 31) // 32 * 32
    np_ = (cout + 15) // 16 * 16
    w9 = qdw[:, 0].reshape(hidden, 9).astype(np.int64)
    wd = np.zeros((9, h32), np.float16)
    wd[:, :hidden] = w9.T                                     # int8 values, exact in fp16
    M, B, S = d_rq
    B = np.asarray(B, np.int64) - 1024 * np.asarray(M, np.int64) * w9.sum(axis=1)
    return _rq16(*e_rq, h32) + _rq16(M, B, S, h32) + _rq16(*p_rq, np_) + wd.tobytes()


def pack_int8(sd: Dict, qp: Dict, arch: Optional[Arch] = None, shift32: bool = True) -> bytes:
    """Pack a reference-layout FP32 state_dict + activation scales into an int8 blob (URSONet head).

    ``shift32=False`` never sets the "every shift is 32" flag, so the fused blocks run their general-shift kernel
    variant (same results; kept for the tests)."""
    arch = arch or arch_from_state_dict(sd)
    if arch.head != 'ursonet':
        raise NotImplementedError('the int8 path mirrors QURSONetHead (ursonet.py:36-93) only')
    validate(qp)
    bw = qp.get('bits') or BitWidths()
    fp = 'features.features'
    data = _Data()
    ops = []

    # stem + input quant
    q, (M, B, S) = _conv(sd, f'{fp}.0', qp['image'], qp['stem'], bw.first_conv[0])
    w28 = np.zeros((32, 28), np.int8)
    w28[:, :27] = q.transpose(0, 2, 3, 1).reshape(32, 27)        # k = ky*9 + kx*3 + ci
    x = np.arange(256, dtype=np.float32) / np.float32(255.0)
    ib = bw.image
    lut = np.clip(np.rint(x / np.float32(qp['image'])), -(1 << (ib - 1)), (1 << (ib - 1)) - 1).astype(np.int8)
    ops.append((OP_QSTEM, 3, 32, 0, 2, 1, 0, data.add(w28.tobytes()), _rq(data, M, B, S), data.add(lut.tobytes()),
                ABSENT, ABSENT, ABSENT, data.add(np.float32(qp['image']).tobytes()), ABSENT, ABSENT,
                (bw.first_conv[1], ib)))

    s_x = qp['stem']
    nb = len(arch.blocks)
    for n, blk in enumerate(arch.blocks):
        bq = qp['blocks'][n]
        s_q = bq['quant']
        s_next = qp['blocks'][n + 1]['quant'] if n + 1 < nb else qp['final']
        s_in = s_q if s_q is not None else s_x
        ew, ea, dwb, da, pw = bw.block(n)
        j = 0
        e_w = e_b = ABSENT
        e_rq = None
        if blk.expand != 1:
            q, e_rq = _conv(sd, f'{fp}.{blk.index}.conv.0', s_in, bq['expand'], ew)
            e_w, _ = _pw(data, q)
            e_b = _rq(data, *e_rq)
            s_y, j = bq['expand'], 1
        else:
            s_y = s_in
        qdw, d_rq = _conv(sd, f'{fp}.{blk.index}.conv.{j}', s_y, bq['dw'], dwb)
        w9 = np.ascontiguousarray(qdw[:, 0].reshape(qdw.shape[0], 9).T.astype(np.int8))   # [9][C], tap = ky*3+kx
        d_w, d_b = data.add(w9.tobytes()), _rq(data, *d_rq)
        p_out = s_q if blk.residual else s_next
        q, p_rq = _conv(sd, f'{fp}.{blk.index}.conv.{j + 1}', bq['dw'], p_out, pw)
        p_w, init = _pw(data, q)
        p_b = _rq(data, *p_rq)
        x2 = ABSENT
        # the fused kernel's requant takes the high word of acc * M + B: every shift must be >= 32 and |M| < 2**31
        if e_rq is None:     # t == 1: no expand table (zero records, unused by the kernel)
            e_rq = (np.zeros(blk.hidden, np.int64), np.zeros(blk.hidden, np.int64), np.full(blk.hidden, 32))
        fusable = all(np.all(r[2] >= 32) and np.all(np.abs(r[0]) < 2 ** 31) for r in (e_rq, d_rq, p_rq))
        if fusable:
            x2 = data.add(_fused_tables(e_rq, d_rq, p_rq, qdw, blk.hidden, blk.cout))
        x1 = ABSENT
        if blk.residual:
            R, RB, RS = fixed(s_q / s_next, 0.0)
            x1 = data.add(np.array([R[0], RB[0], RS[0]], np.int64).tobytes())
        flags = (1 if blk.residual else 0) | (2 if s_q is None else 0)
        if shift32 and fusable and all(np.all(r[2] == 32) for r in (e_rq, d_rq, p_rq)):
            flags |= 4       # every fused requant shift is exactly 32: the kernel's shift-free variant
        ops.append((OP_QIRB, blk.cin, blk.cout, blk.hidden, blk.stride, blk.expand, flags,
                    e_w, e_b, d_w, d_b, p_w, p_b, data.add(init.tobytes()), x1, x2,
                    (ea if ea is not None else 8, da, bw.shared_act)))

    q, (M, B, S) = _conv(sd, arch.last.prefix, qp['final'], qp['last'], bw.last_conv[0])
    l_w, _ = _pw(data, q)
    ops.append((OP_QLAST, arch.last.cin, arch.last.cout, 0, 1, 1, 0, l_w, _rq(data, M, B, S),
                ABSENT, ABSENT, ABSENT, ABSENT, ABSENT, ABSENT, ABSENT, (bw.last_conv[1], bw.pooling)))

    rows, sws, bs = [], [], []
    for key in ('head.ori.1', 'head.pos.0'):
        q, s_w = weight_q(sd[f'{key}.weight'], bw.fully_connected[0])
        rows.append(q)
        sws.append(s_w)
        bs.append(_np(sd[f'{key}.bias']).astype(np.float64))
    q = np.concatenate(rows)
    n = q.shape[0]
    np_ = (n + 15) // 16 * 16
    w = np.zeros((np_, LAST_CHANNELS), np.int8)
    w[:n] = q
    sw = np.zeros(np_, np.float64)
    sw[:n] = np.concatenate(sws)
    bias = np.zeros(np_, np.float64)
    bias[:n] = np.concatenate(bs)
    wsum = np.zeros(np_, np.int32)
    wsum[:n] = 128 * q.sum(axis=1)
    ops.append((OP_QFC, LAST_CHANNELS, n, 0, 1, 1, 0, data.add(w.tobytes()), data.add(sw.tobytes()),
                data.add(bias.tobytes()), ABSENT, ABSENT, ABSENT, data.add(wsum.tobytes()),
                data.add(np.float64(qp['last']).tobytes()), ABSENT, (bw.fully_connected[1],)))
    return assemble(DT_I8, HEAD_URSONET, rows[0].shape[0], rows[1].shape[0], 0, 0, ops, data)
