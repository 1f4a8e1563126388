"""GPU: the profiling table names the kernel the library actually launched for each fp16mx block (spef_api.cpp asks
k_x2.hip's dispatch table walk, x2_irb_kernel_name), so the bench line's ``roofline.kernel`` and its PMC-traffic lookup
refer to the real symbol: at the bench workload (B = 64, 512^2) blocks 5-7 run the slab kernel, 8-10 and 14 the
role-split kernel with persistent tiles, 11-13 and 15-17 the three-stage kernel."""
import numpy as np
import pytest
import torch

from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.engine import Engine
from spef_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu


def test_profile_keys_name_launched_kernels():
    sd = synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=1001)
    eng = Engine(Bl.pack(sd, mobilenet_v2('ursonet', 1728, 3), dtype='fp16mx'), 'cuda:0')
    fr = torch.from_numpy(np.random.Generator(np.random.PCG64(3)).integers(0, 256, (64, 512, 512, 3),
                                                                          dtype=np.uint8)).cuda()
    eng.forward(fr)
    torch.cuda.synchronize()
    eng.profile_begin()
    eng.forward(fr)
    prof = eng.profile_end()
    eng.close()
    keys = set(prof)
    expect = {'mx_irb_kernel<16,96,24,s2>', 'mx_irb_kernel<24,144,24,s1>', 'mx_irb_kernel<24,144,32,s2>',
              'x2_irb_kernel<32,192,32,s1>', 'x2_irb_kernel<32,192,64,s2>',
              'x2_irw_kernel<64,384,64,s1>', 'x2_irp_kernel<64,384,96,s1>', 'x2_irp_kernel<96,576,96,s1>',
              'x2_irw_kernel<96,576,160,s2>', 'x2_irp_kernel<160,960,160,s1>', 'x2_irp_kernel<160,960,320,s1>'}
    assert expect <= keys, sorted(keys)
    assert prof['x2_irp_kernel<96,576,96,s1>'][0] == 2 and prof['x2_irw_kernel<64,384,64,s1>'][0] == 3
