"""Blob builder: BN folding is exact (float64) and the packed layout matches csrc/spef_blob.hpp."""
import numpy as np
import torch
import torch.nn.functional as F

from spef_amd import blob as Bl
from spef_amd.arch import count_macs, mobilenet_v2, state_dict_shapes
from spef_amd.weights import synthetic_state_dict


def test_state_dict_layout_matches_reference_keys():
    arch = mobilenet_v2()
    shapes = state_dict_shapes(arch)
    sd = synthetic_state_dict(arch)
    assert len(shapes) == 316 == len(sd)
    for k, s in shapes.items():
        assert tuple(sd[k].shape) == tuple(s), k


def test_macs_match_survey():
    m = count_macs(mobilenet_v2(), 512, 512)
    assert m['total'] == 1_566_920_448          # SURVEY §8a R3 (nn_stats.py:31-41 counting)
    assert count_macs(mobilenet_v2(), 240, 384)['total'] == 561_955_584


def test_bn_fold_equals_conv_then_bn():
    arch = mobilenet_v2()
    sd = synthetic_state_dict(arch)
    c = arch.blocks[3].convs[0]
    w, b = Bl.fold_bn(sd, c)
    x = torch.randn(2, c.cin, 5, 5, dtype=torch.float64)
    ref = F.batch_norm(F.conv2d(x, torch.from_numpy(sd[f'{c.prefix}.0.weight']).double()),
                       torch.from_numpy(sd[f'{c.prefix}.1.running_mean']).double(),
                       torch.from_numpy(sd[f'{c.prefix}.1.running_var']).double(),
                       torch.from_numpy(sd[f'{c.prefix}.1.weight']).double(),
                       torch.from_numpy(sd[f'{c.prefix}.1.bias']).double(), False, 0.1, 1e-5)
    got = F.conv2d(x, torch.from_numpy(w), torch.from_numpy(b))
    assert torch.allclose(ref, got, atol=1e-12)


def test_pack_layout():
    arch = mobilenet_v2()
    sd = synthetic_state_dict(arch)
    for dt in ('fp16', 'bf16'):
        b = Bl.pack(sd, arch, dtype=dt)
        info = Bl.describe(b)
        assert info['n_ops'] == 1 + 17 + 1 + 1
        assert info['n_out0'] == 1728 and info['n_out1'] == 3 and info['feat_c'] == 1280
        assert info['data_off'] % 256 == 0 and info['data_off'] + info['data_bytes'] == len(b)
        kinds = [o[0] for o in info['ops']]
        assert kinds == [Bl.OP_STEM] + [Bl.OP_IRB] * 17 + [Bl.OP_LAST, Bl.OP_FC]
        for o in info['ops']:
            for off in o[8:]:
                assert off == Bl.ABSENT or (off % 256 == 0 and off < info['data_bytes'])
        # block 1 (t=1) has no expand conv
        assert info['ops'][1][8] == Bl.ABSENT and info['ops'][2][8] != Bl.ABSENT


def test_pointwise_tensor_padding_fp16():
    arch = mobilenet_v2()
    sd = synthetic_state_dict(arch)
    b = Bl.pack(sd, arch, dtype='fp16')
    info = Bl.describe(b)
    op = info['ops'][3]                       # block 3: 24 -> 144 -> 24 (residual)
    assert op[1:4] == (24, 24, 144) and op[6] == 1
    w_off = info['data_off'] + op[8]
    wp = np.frombuffer(b, np.float16, count=144 * 32, offset=w_off).reshape(144, 32)
    w, _ = Bl.fold_bn(sd, arch.blocks[2].convs[0])
    np.testing.assert_allclose(wp[:, :24], w[:, :, 0, 0].astype(np.float16))
    assert not wp[:, 24:].any()


def test_pack_infers_head_from_state_dict():
    """pack(sd) without an explicit arch reads the head type/widths from the reference keys."""
    from spef_amd.arch import arch_from_state_dict, mobilenet_v2
    from spef_amd.weights import synthetic_state_dict
    for a in (mobilenet_v2('ursonet', 1232, 1000), mobilenet_v2('keypoints')):
        sd = synthetic_state_dict(a, seed=3)
        b = arch_from_state_dict(sd)
        assert (b.head, b.n_ori, b.n_pos, b.n_kp) == (a.head, a.n_ori, a.n_pos, a.n_kp)
        assert Bl.pack(sd) == Bl.pack(sd, a)
