"""SPEF MI355X benchmark: images/sec at 512x512, batch 64 per GPU (BASELINE.json metric).

A "step" = one pass of the hot path over one batch: uint8 NHWC frames already resident in HBM ->
MobileNet-V2 backbone -> URSONet head -> on-device decode (softmax + Markley orientation average, position
regression), i.e. SPEMi355x.predict minus the host copies. Weights: seeded synthetic (spef_amd.weights),
BN folded, fp16 storage / fp32 accumulate. Frames: synthetic SPEED-style (dark background + noise + bright
target), generated once per rank from (seed, global frame index). Consecutive steps alternate over --inflight
HIP streams (spef_amd.pipeline.StreamPipeline, default 3 batches in flight): every step is still the complete
forward + decode of its batch, but one batch's low-occupancy tail overlaps the next batch's front kernels.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process per GPU,
rank 0 packs the weight blob and RCCL-broadcasts it (torch.distributed 'nccl' = RCCL over xGMI); every rank
then runs independent batches of 64 (frame-parallel, weak scaling, no data-path collective). Timing: barrier +
device sync on both sides of exactly K steps, max over ranks; value = all ranks' images / that time.

Rank 0 prints ONE JSON line (see DESIGN.md "Measurement" for every field).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd'))
sys.path.insert(0, ROOT)

from spef_amd.data.synthetic import synth_frames  # noqa: E402  (SPEED-style frames)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_PEAK_TFLOPS = 2500.0      # dense fp16/bf16 MFMA, no sparsity


def pmc_traffic(kernel_key: str, path: str):
    """HBM bytes per launch of ``kernel_key`` from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes
    (tools/rocprof_summary.py: bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024, the gfx950 correction), or None when
    the file is absent or the profiled symbol for this key is ambiguous."""
    try:
        with open(path) as f:
            kernels = json.load(f)['kernels']
    except (OSError, KeyError, ValueError):
        return None
    if kernel_key in kernels:
        return kernels[kernel_key]['hbm_bytes_per_launch']
    import re
    m = re.fullmatch(r'(ir[bsw]_kernel)<(\d+),(\d+),(\d+),s(\d+)>', kernel_key)
    if m:   # fused block key -> the one template instantiation profiled for that geometry
        geo = ','.join(m.groups()[1:]) + ','
        hits = [v for k, v in kernels.items() if re.match(m.group(1) + r'<B?F16,' + re.escape(geo), k)]
    else:
        prefix = kernel_key.split('<')[0] + '<'
        hits = [v for k, v in kernels.items() if k.startswith(prefix)]
    return hits[0]['hbm_bytes_per_launch'] if len(hits) == 1 else None


def cpu_baseline(args, sd):
    """The CPU oracle (FP32 PyTorch restatement of the reference eval path: forward + softmax + Markley decode,
    pinned to the reference by tests/golden) timed on this host's cores, on a bounded sample."""
    import numpy as np
    import torch
    from oracle import decode_ref as D
    from oracle import model_ref as M
    threads = min(args.cpu_threads, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    h, _ = D.orientation_histogram(12, False)
    bs, nb = args.cpu_batch, args.cpu_batches
    fr = synth_frames(bs, args.size, args.size, 10_000)
    x = M.u8_nhwc_to_nchw_f32(fr)
    o, p = M.forward(x[:2], sd)                                        # warm-up
    t0 = time.perf_counter()
    for _ in range(nb):
        o, p = M.forward(x, sd)
        D.decode_orientation_batch(D.softmax_f32(o.numpy()), h)
    dt = time.perf_counter() - t0
    base = {'value': round(bs * nb / dt, 3), 'unit': 'images/sec', 'cores': threads, 'kind': 'port',
            'sample': f'{nb} batches x {bs} synthetic {args.size}x{args.size} frames, FP32 torch CPU forward + '
                      f'NumPy softmax/Markley decode (oracle/, pinned to the reference by tests/golden), '
                      f'{threads} threads, {dt:.1f} s'}
    q = D.decode_orientation_batch(D.softmax_f32(o.numpy()), h)
    return base, (fr, o.numpy(), p.numpy(), q)


def pose_error(eng, dev, fr, o_ref, p_ref, q_ref):
    """'pose err vs fp32 ref' half of the metric: the GPU path (uint8 NHWC frames, as timed) on the CPU
    baseline's own frames, against the FP32 oracle's logits and decoded pose."""
    import numpy as np
    import torch
    from oracle import decode_ref as D
    xg = torch.from_numpy(fr).to(dev)
    o, p = eng.forward(xg)
    dec = eng.decode(1, 0, o, p, want_soft=True)
    ang = D.angle_deg_stable(dec['ori'].cpu().numpy().astype(np.float64), q_ref)
    torch.cuda.synchronize(dev)
    return {'frames': int(fr.shape[0]), 'ori_logit_max_abs': float(np.abs(o.cpu().numpy() - o_ref).max()),
            'pos_max_abs_m': float(np.abs(p.cpu().numpy() - p_ref).max()), 'ori_max_deg': float(ang.max()),
            'tolerance': 'logits 1e-3, pose 0.1 deg / 1 mm (BASELINE.json north_star)'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=100)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--size', type=int, default=512)
    ap.add_argument('--dtype', default='fp16', choices=['fp16', 'bf16', 'int8'],
                    help='int8 = the Brevitas-mirroring C5 path (calibrated activation scales)')
    ap.add_argument('--inflight', type=int, default=3,
                    help='batches in flight: consecutive steps alternate over this many HIP streams (spef_amd.pipeline)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-threads', type=int, default=16)
    ap.add_argument('--cpu-batch', type=int, default=64)
    ap.add_argument('--cpu-batches', type=int, default=3)
    ap.add_argument('--traffic', default=None,
                    help='committed rocprofv3 FETCH/WRITE summary used for roofline.traffic (default: '
                         'profiles/r01_pmc_traffic.json, r01_int8_pmc_traffic.json for --dtype int8)')
    args = ap.parse_args()
    if args.traffic is None:
        args.traffic = os.path.join(ROOT, 'profiles', 'r01_int8_pmc_traffic.json' if args.dtype == 'int8'
                                    else 'r01_pmc_traffic.json')

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', rank=rank, world_size=world, device_id=torch.device(f'cuda:{local}'))
    dev = torch.device(f'cuda:{local}')
    torch.cuda.set_device(dev)

    from spef_amd import blob as Bl
    from spef_amd.arch import flops_per_image, mobilenet_v2
    from spef_amd import _lib as L
    from spef_amd.pipeline import StreamPipeline
    from spef_amd.shard import broadcast_blob, max_over_ranks, shard_range
    from spef_amd.spe.spe_utils import SPEUtils
    from spef_amd.weights import synthetic_state_dict

    sd = None
    blob = None
    if rank == 0:
        sd = synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=1001)
        if args.dtype == 'int8':
            from spef_amd.blob_q8 import pack_int8
            from spef_amd.quant import calibrate
            blob = pack_int8(sd, calibrate(sd, synth_frames(4, 128, 128, 900)))
        else:
            blob = Bl.pack(sd, dtype=args.dtype)
    dblob = broadcast_blob(blob, dev)                 # RCCL over xGMI
    su = SPEUtils(None, 'classification', 12, 3, False, 'regression')
    pipe = StreamPipeline(dblob, dev, depth=max(1, args.inflight), ori_bins=su.orientation.histogram)
    eng = pipe.engine

    B, S = args.batch, args.size
    first, stop = shard_range(B * world, rank, world)          # this rank's global frame indices
    frames = torch.from_numpy(synth_frames(stop - first, S, S, first)).to(dev)
    pipe.reserve(B, S, S)
    ori = torch.empty((B, eng.n_out0), dtype=torch.float32, device=dev)
    pos = torch.empty((B, eng.n_out1), dtype=torch.float32, device=dev)

    def step():   # one batch: forward + decode, on the next of --inflight streams
        return pipe.submit(frames, L.CLASSIFICATION, L.REGRESSION, want_soft=True)

    def step_single():   # the same work on one stream (the per-kernel HIP-event leg)
        eng.forward(frames, ori, pos)
        return eng.decode(1, 0, ori, pos, want_soft=True)

    for _ in range(args.warmup):
        step()
    pipe.synchronize()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    pipe.synchronize()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, dev)
    assert not out['status'].any().item(), 'decode reported NaN'

    # roofline leg: per-kernel HIP events on the engine's stream, K more steps
    eng.profile_begin()
    for _ in range(args.steps):
        step_single()
    prof = eng.profile_end()

    if rank == 0:
        total_img = B * args.steps * world
        value = total_img / elapsed
        dom_key = max(prof, key=lambda k: prof[k][1])
        n, ms, byts, fl = prof[dom_key]
        avg_s = ms / n / 1e3
        ach_gbs = byts / n / avg_s / 1e9
        ach_tfl = fl / n / avg_s / 1e12
        fpi = flops_per_image(S, S)
        step_ms = elapsed / args.steps * 1e3
        traffic = pmc_traffic(dom_key, args.traffic)
        if traffic is not None:
            traffic *= B / 64.0     # the PMC passes ran batch 64 (tools/pmc.sh); bytes scale with the batch
        rec = {
            'metric': 'images/sec at 512\u00d7512 batch 64, 1/2/4/8 MI355X; pose err vs fp32 ref',
            'value': round(value, 2),
            'unit': 'images/sec',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(step_ms, 4),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': args.dtype,
            'data': 'synthetic SPEED-style uint8 frames resident in HBM; seeded random weights (BN-calibrated)',
            'config': {'workload': (f'C5: INT8 (Brevitas-mirroring, calibrated scales) full net + decode, {S}x{S}, '
                                    f'batch {B} per GPU' if args.dtype == 'int8' else
                                    f'C3: full net + decode, {S}x{S}, batch {B} per GPU'), 'global_batch': B * world,
                       'image_size': S, 'parallelism': f'frame-parallel x{world} (RCCL weight bcast)',
                       'inflight_batches': max(1, args.inflight)},
            'roofline': {'bound': 'hbm', 'kernel': dom_key, 'achieved': round(ach_gbs, 1), 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': round(ach_gbs / HBM_PEAK_GBS, 4),
                         'traffic': None if traffic is None else round(traffic),
                         'traffic_source': os.path.relpath(args.traffic, ROOT) if traffic is not None else None,
                         'algorithmic_bytes_per_launch': round(byts / n),
                         'avg_launch_us': round(avg_s * 1e6, 2), 'launches_per_step': n / args.steps,
                         'kernel_mfma_tflops': round(ach_tfl, 2)},
            'mfma_utilisation_whole_net': round(fpi * value / world / 1e12 /
                                                (2 * MFMA_PEAK_TFLOPS if args.dtype == 'int8' else MFMA_PEAK_TFLOPS), 5),
            'kernels': {k: {'launches_per_step': v[0] / args.steps, 'ms_per_step': round(v[1] / args.steps, 4),
                            'GB/s': round(v[2] / (v[1] / 1e3) / 1e9, 1) if v[1] > 0 else None}
                        for k, v in sorted(prof.items(), key=lambda kv: -kv[1][1])},
        }
        if world == 1 and not args.no_cpu_baseline:
            rec['cpu_baseline'], ref = cpu_baseline(args, sd)
            rec['pose_err_vs_fp32'] = pose_error(eng, dev, *ref)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
