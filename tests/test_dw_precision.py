"""Precision budget of the packed-fp16 depthwise (CPU). Blocks 2-7 of the fp16 schedule accumulate their
3x3 depthwise in fp16 (v_pk_fma_f16, k_irb.hip irb_pk); tools/dw_acc_budget.py restates that schedule in float64 with
an fp16 rounding after every tap. The URSONet outputs must stay within the north star's 1e-3 of float32 (BASELINE.json)
and within a small margin of the fp32-accumulation schedule the rest of the network uses. The GPU side of the same
claim is the bench line's pose_err_vs_fp32 and tests/test_gpu_parity.py's golden-forward bounds."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'tools'), os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd')]

import dw_acc_budget as D  # noqa: E402
from spef_amd.arch import mobilenet_v2  # noqa: E402
from spef_amd.weights import synthetic_state_dict  # noqa: E402

PK_BLOCKS = (2, 3, 4, 5, 6, 7)   # irb_pk: expand blocks up to hidden width 192


def test_pk_blocks_match_kernel_rule():
    arch = mobilenet_v2('ursonet', 1728, 3)
    pk = tuple(b.index for b in arch.blocks if b.expand != 1 and b.hidden <= 192)
    assert pk == PK_BLOCKS


def test_fp16_accumulated_depthwise_within_north_star():
    arch = mobilenet_v2('ursonet', 1728, 3)
    sd = synthetic_state_dict(arch, seed=1001)
    fr = np.random.Generator(np.random.PCG64(5)).integers(0, 256, (1, 256, 256, 3), dtype=np.uint8)
    x = torch.from_numpy(fr).permute(0, 3, 1, 2).to(torch.float64) / 255.0
    with torch.no_grad():
        ref = D.forward(x, sd, arch, False)
        fp32acc = D.forward(x, sd, arch, True)
        pk = D.forward(x, sd, arch, True, PK_BLOCKS)
    e_ori, e_pos = [(p - r).abs().max().item() for p, r in zip(pk, ref)]
    base_ori = (fp32acc[0] - ref[0]).abs().max().item()
    assert e_ori < 1e-3 and e_pos < 1e-3, (e_ori, e_pos)
    assert e_ori < 1.25 * base_ori + 1e-4, (e_ori, base_ori)


def test_fp16_accumulation_costs_nothing_with_wide_bn_statistics():
    """trained nets may carry larger folded BN biases than synthetic_state_dict's. With every BN beta and
    running mean scaled 10x (activations and logits ~8x larger), the packed fp16 accumulation still adds nothing to
    the fp16-storage schedule's error (measured 3.20e-3 vs 3.26e-3 at logit magnitude 4.9). That error itself grows
    with the output scale -- fp16 storage is ~7e-4 of the logit range -- so the absolute 1e-3 bound is met by the
    fp16x2 schedule (tests/test_gpu_x2.py), and build_mi355x flags every variant beyond it (within_north_star)."""
    arch = mobilenet_v2('ursonet', 1728, 3)
    sd = synthetic_state_dict(arch, seed=1001)
    for k in list(sd):
        if k.endswith('.1.bias') or k.endswith('.1.running_mean'):
            sd[k] = (sd[k] * 10.0).astype(np.float32)
    fr = np.random.Generator(np.random.PCG64(5)).integers(0, 256, (1, 256, 256, 3), dtype=np.uint8)
    x = torch.from_numpy(fr).permute(0, 3, 1, 2).to(torch.float64) / 255.0
    with torch.no_grad():
        ref = D.forward(x, sd, arch, False)
        fp32acc = D.forward(x, sd, arch, True)
        pk = D.forward(x, sd, arch, True, PK_BLOCKS)
    e_pk = (pk[0] - ref[0]).abs().max().item()
    e_32 = (fp32acc[0] - ref[0]).abs().max().item()
    assert ref[0].abs().max().item() > 3.0                       # the wide statistics did widen the outputs
    assert e_pk < 1.25 * e_32 + 1e-4, (e_pk, e_32)
