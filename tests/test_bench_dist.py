"""bench.py's multi-process branch, on CPU: torch.distributed.run launches 2 ranks of ``bench.py --dry-run``, which
runs the same control flow as the GPU job (env rank/world parsing, process-group init, weight broadcast from rank 0
with every rank validating the received blob through the C ABI, barrier-bracketed timing of exactly K steps,
max over ranks, one JSON line from rank 0) with gloo and no device work."""
import importlib.util
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


def _bench_module():
    spec = importlib.util.spec_from_file_location('spef_bench', os.path.join(REPO, 'bench.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bench_two_rank_dry_run(tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS='1')
    detail = tmp_path / 'detail.json'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2', '--master-addr',
           '127.0.0.1', '--master-port', str(_free_port()), os.path.join(REPO, 'bench.py'), '--gpus', '2',
           '--steps', '3', '--warmup', '1', '--dry-run', '--detail-out', str(detail)]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout                      # exactly one JSON line, from rank 0
    assert r.stdout.rstrip().splitlines()[-1] == lines[0]  # ... and it is the last stdout line (the driver parses it)
    assert len(lines[0]) < 6000
    rec = json.loads(lines[0])
    assert json.loads(detail.read_text())['value'] == rec['value']
    assert rec['dry_run'] is True and rec['n_gpus'] == 2 and rec['steps'] == 3 and rec['warmup'] == 1
    assert rec['config']['global_batch'] == 128 and rec['scaling'] == 'weak'
    assert rec['value'] > 0 and rec['unit'] == 'images/sec'


def test_headline_line_compact_on_a_full_gpu_record():
    """The round-5 GPU record (every sub-record and per-kernel table: a 22.5 KB line the driver could not parse,
    BENCH_r05.json ``parsed: null``) compacts to a headline under 6 KB that still carries the contract fields,
    ``roofline`` (with traffic over algorithmic bytes), ``cpu_baseline``, the pose errors and each sub-record's img/s."""
    bench = _bench_module()
    with open(os.path.join(REPO, 'profiles', 'r05_bench.json')) as f:
        full = json.load(f)
    assert len(json.dumps(full)) > 20000
    line = json.dumps(bench.compact_record(full, 'gpurun_out/bench_detail.json'))
    assert len(line) < bench.HEADLINE_MAX_BYTES <= 6000
    rec = json.loads(line)
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better', 'scaling',
              'vs_baseline', 'dtype', 'config', 'roofline', 'cpu_baseline', 'pose_err_vs_fp32'):
        assert k in rec, k
    assert rec['value'] == full['value'] and rec['roofline']['frac'] == full['roofline']['frac']
    assert rec['cpu_baseline']['cores'] and rec['cpu_baseline']['kind'] == 'port'
    assert 'kernels' not in rec and 'keypoint_mode' not in rec
    assert set(rec['sub_records']) == {'c5', 'fp16x2', 'fp16', 'keypoint_mode', 'epnp'}
    assert rec['pose_err_vs_fp32_sharp_head']['fp16mx']['within_tolerance'] is True


def test_roofline_traffic_lookup_by_launched_kernel():
    """bench.py's PMC-traffic lookup for the roofline kernel: the profiling key names the kernel the library launched
    (x2_irb / x2_irw / x2_irp, spef_api.cpp); each key must resolve to exactly one profiled instantiation of the
    committed round-6 fp16mx traffic file, and the dominant kernel's bytes must be the file's entry for it."""
    import json
    bench = _bench_module()
    path = os.path.join(REPO, 'profiles', 'r06_mx_pmc_traffic.json')
    with open(path) as f:
        kernels = json.load(f)['kernels']
    keys = {'x2_irp_kernel<96,576,96,s1>': 'x2_irp_kernel<96,576,96,1,8,16,1,1>',
            'x2_irw_kernel<64,384,64,s1>': 'x2_irw_kernel<64,384,64,1,8,16,1,1,1,1,1>',
            'x2_irb_kernel<32,192,32,s1>': 'x2_irb_kernel<32,192,32,1,8,16,1,1,4,1,0>',
            'x2_irp_kernel<160,960,320,s1>': 'x2_irp_kernel<160,960,320,1,8,8,0,0>',
            'mx_irb_kernel<24,144,24,s1>': 'mx_irb_kernel<24,144,24,1,16,1,1,1>'}
    for key, sym in keys.items():
        assert bench.pmc_traffic(key, path) == kernels[sym]['hbm_bytes_per_launch'], key
    assert bench.pmc_traffic('x2_irp_kernel<1,2,3,s1>', path) is None     # no such instantiation: no traffic figure


def test_plant_keypoint_head_outputs_the_planted_keypoints():
    """weights.plant_keypoint_head (the bench's keypoint sub-record and the B=64 keypoint test): with zero head weights
    the sigmoid of the head output is exactly the planted keypoints (float32 logit / sigmoid round trip)."""
    import numpy as np
    from spef_amd.arch import mobilenet_v2
    from spef_amd.weights import plant_keypoint_head, synthetic_state_dict
    g = np.load(os.path.join(REPO, 'tests', 'golden', 'keypoints.npz'))
    sd = plant_keypoint_head(synthetic_state_dict(mobilenet_v2('keypoints'), seed=1001, head_std=2e-4), g['kp2d'][7])
    b = sd['head.layer.1.bias'].astype(np.float64)
    np.testing.assert_allclose(1.0 / (1.0 + np.exp(-b)), g['kp2d'][7], rtol=0, atol=2e-7)
