"""GPU, two devices: spef_bcast_weights over a real 2-rank RCCL communicator (the receive side had only run
with one rank). Launched as its own torch.distributed.run job (tests/_bcast2_worker.py) so no rank inherits this
process's HIP state; skipped on boxes with fewer than two GPUs (torch.cuda.device_count() initialises nothing)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason='needs two GPUs on one node')
def test_two_rank_rccl_weight_broadcast():
    from spef_amd import _lib as L
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2', '--master-addr',
           '127.0.0.1', '--master-port', str(_free_port()), os.path.join(REPO, 'tests', '_bcast2_worker.py')]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{')][-1])
    r0, r1 = rec['ranks']
    for mode, code in ((1, L.ERR_HIP), (2, L.ERR_BLOB)):
        for rr in (r0, r1):   # every rank returns the same code, naming rank 1, and keeps its model
            assert rr[f'fail{mode}'][0] == code and 'rank 1' in rr[f'fail{mode}'][1], (mode, rr)
            assert rr[f'fail{mode}_model_kept'], (mode, rr)
    assert rec['identical_after_bcast'] and rec['rank1_changed'], rec
