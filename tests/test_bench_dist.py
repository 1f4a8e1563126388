"""bench.py's multi-process branch, on CPU: torch.distributed.run launches 2 ranks of ``bench.py --dry-run``, which
runs the same control flow as the GPU job (env rank/world parsing, process-group init, weight broadcast from rank 0
with every rank validating the received blob through the C ABI, barrier-bracketed timing of exactly K steps,
max over ranks, one JSON line from rank 0) with gloo and no device work."""
import json
import os
import socket
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def test_bench_two_rank_dry_run():
    env = dict(os.environ, OMP_NUM_THREADS='1')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2', '--master-addr',
           '127.0.0.1', '--master-port', str(_free_port()), os.path.join(REPO, 'bench.py'), '--gpus', '2',
           '--steps', '3', '--warmup', '1', '--dry-run']
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout                      # exactly one JSON line, from rank 0
    rec = json.loads(lines[0])
    assert rec['dry_run'] is True and rec['n_gpus'] == 2 and rec['steps'] == 3 and rec['warmup'] == 1
    assert rec['config']['global_batch'] == 128 and rec['scaling'] == 'weak'
    assert rec['value'] > 0 and rec['unit'] == 'images/sec'
