"""SPEF MI355X benchmark: images/sec at 512x512, batch 64 per GPU (BASELINE.json metric).

A "step" = one pass of the hot path over one batch: uint8 NHWC frames already resident in HBM ->
MobileNet-V2 backbone -> URSONet head -> on-device decode (softmax + Markley orientation average, position
regression), i.e. SPEMi355x.predict minus the host copies. Weights: seeded synthetic (spef_amd.weights),
BN folded. Headline schedule: fp16mx (blob dtype 6) -- every matrix product on the fp16 MFMA with hi + lo split
operands and fp32 accumulation, fp32 depthwise, fp32 activations except the block outputs of blocks 1-6 (fp16): within
the north star's 1e-3 logit bound at trained head scales; the fp16 schedule (fast, not within
that bound at sharp heads), fp16x2 (all activations fp32) and int8 (C5) are sub-records. Frames: synthetic SPEED-style (dark background + noise + bright
target), generated per rank from (seed, global frame index); the timed steps rotate over --frame-buffers distinct
device batches (6 x 50 MB by default, more than the 256 MB Infinity Cache), so every step streams its input from
HBM. Consecutive steps alternate over --inflight HIP streams (spef_amd.pipeline.StreamPipeline, default 3 batches
in flight): every step is still the complete forward + decode of its batch, but one batch's low-occupancy tail
overlaps the next batch's front kernels.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process per GPU. Rank 0
packs the weight blob; the library's own RCCL communicator (C ABI spef_comm_init, id shipped over the
torch.distributed group) broadcasts it over xGMI into every rank's contexts (spef_bcast_weights); every rank then
runs independent batches of 64 (frame-parallel, weak scaling, no data-path collective). Timing: barrier + device
sync on both sides of exactly K steps, max over ranks; value = all ranks' images / that time.
``--dry-run`` runs the same control flow on CPU with gloo (no device work; tests/test_bench_dist.py).

Rank 0 prints ONE JSON line, the last line of stdout, kept to a few KB (``compact_record``: contract fields, roofline,
cpu_baseline, pose errors, one summary per sub-record); the full record with the per-kernel tables and every sub-record
goes to ``--detail-out`` (default gpurun_out/bench_detail.json). Fields: DESIGN.md section 9.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd'))
sys.path.insert(0, ROOT)

from spef_amd.data.synthetic import synth_frames  # noqa: E402  (SPEED-style frames)
from spef_amd.measure import ClockProbe, measure_peaks  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_PEAK_TFLOPS = 2500.0      # dense fp16/bf16 MFMA, no sparsity (int8: 2x)
METRIC = 'images/sec at 512×512 batch 64, 1/2/4/8 MI355X; pose err vs fp32 ref'
INT8_TOLERANCE = ('int8 contract: bit-exact vs the integer oracle (oracle/int8_ref.py, tests/test_gpu_int8.py); '
                  'accuracy vs FP32 is set by the quantisation scales (PTQ-calibrated here, QAT-learned in the '
                  'reference), not by the kernels: its own bound is logits 0.05, pose 0.25 deg / 30 mm (DESIGN.md '
                  'section 5), not the fp16 1e-3 / 0.1 deg / 1 mm')
INT8_BOUND = (0.05, 0.030, 0.25)   # logits, position (m), orientation (deg)
# committed rocprofv3 FETCH_SIZE / WRITE_SIZE summaries, newest first (profiles/)
FP16_TRAFFIC = ['r04_pmc_traffic.json', 'r03f_pmc_traffic.json']
MX_TRAFFIC = ['r06_mx_pmc_traffic.json', 'r05_mx_pmc_traffic.json']
INT8_TRAFFIC = ['r03_int8_pmc_traffic.json']
X2_TRAFFIC = ['r06_x2_pmc_traffic.json', 'r05_x2_pmc_traffic.json', 'r04_x2_pmc_traffic.json']
TRAFFIC = {'fp16': FP16_TRAFFIC, 'bf16': FP16_TRAFFIC, 'int8': INT8_TRAFFIC, 'fp16x2': X2_TRAFFIC, 'fp16mx': MX_TRAFFIC}
ARITH = {'fp16': 'fp16 storage, fp16 MFMA operands, fp32 accumulate (packed-fp16 depthwise in blocks 2-7)',
         'bf16': 'bf16 storage, bf16 MFMA operands, fp32 accumulate',
         'int8': 'int8 MFMA, exact int32 accumulate, fixed-point requant',
         'fp16x2': 'fp32 activations; hi + lo fp16 MFMA operands (3 MFMAs per product), fp32 accumulate, fp32 depthwise',
         'fp16mx': 'hi + lo fp16 MFMA operands, fp32 accumulate, fp32 depthwise; fp32 activations except fp16 storage '
                   'of the stem map, the block outputs of blocks 1-3 and the hidden tensors of blocks 2-4'}


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
    m = re.fullmatch(r'(x2_ir[bwp]_kernel|mx_irb_kernel|ir[bwp]_kernel)<(\d+),(\d+),(\d+),s(\d+)>', kernel_key)
    if m:   # fused block key -> the one template instantiation profiled for that geometry (fp16x2: slab, role-split or
        # three-stage; the key names the kernel the library launched)
        geo = ','.join(m.groups()[1:]) + ','
        kind = {'x2_irb_kernel': r'x2_ir[bwp]_kernel<', 'x2_irw_kernel': r'x2_irw_kernel<',
                'x2_irp_kernel': r'x2_irp_kernel<', 'mx_irb_kernel': r'mx_irb_kernel<'}.get(m.group(1),
                                                                                         m.group(1) + r'<B?F16,')
        hits = [v for k, v in kernels.items() if re.match(kind + re.escape(geo), k)]
    else:   # e.g. front_kernel<stem+block1> -> front_kernel<...> or its fp16 form front_vp_kernel<...>
        base = kernel_key.split('<')[0]
        prefixes = (base + '<', base.replace('_kernel', '_vp_kernel') + '<')
        if base == 'mx_front_kernel':   # the fp16mx front kernel's symbol
            prefixes = ('front_mx_kernel<',)
        elif base == 'x2_pw_kernel' and kernel_key.endswith('<pool>'):   # the staged last conv + mean
            prefixes = ('x2_pws_kernel<',)
        hits = [v for k, v in kernels.items() if k.startswith(prefixes)]
    return hits[0]['hbm_bytes_per_launch'] if len(hits) == 1 else None


def cpu_info() -> dict:
    """CPU model, physical cores per socket (lscpu), the cgroup CPU quota and the affinity mask of this process."""
    info = {'model': None, 'sockets': None, 'cores_per_socket': None, 'cpu_quota': None,
            'affinity': len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else os.cpu_count()}
    try:
        import subprocess
        out = subprocess.run(['lscpu'], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(':')
            k, v = k.strip(), v.strip()
            if k == 'Model name':
                info['model'] = v
            elif k == 'Socket(s)':
                info['sockets'] = int(v)
            elif k == 'Core(s) per socket':
                info['cores_per_socket'] = int(v)
    except (OSError, ValueError):
        pass
    try:
        q, p = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            info['cpu_quota'] = int(q) / int(p)
    except (OSError, ValueError):
        pass
    return info


def cpu_baseline(args, sd):
    """The CPU oracle (FP32 PyTorch restatement of the reference eval path: forward + softmax + Markley decode,
    pinned to the reference by tests/golden) timed on this host's cores, BASELINE.md section 3 protocol: threads =
    one socket's physical cores (capped by this container's CPU quota and affinity), C3 B=64: one warm-up batch,
    median of 3; C1 B=1: one warm-up, median of 5."""
    import numpy as np
    import torch
    from oracle import decode_ref as D
    from oracle import model_ref as M
    ci = cpu_info()
    cap = [c for c in (ci['cores_per_socket'], ci['cpu_quota'] and int(ci['cpu_quota']), ci['affinity']) if c]
    threads = args.cpu_threads or max(1, min(cap) if cap else (os.cpu_count() or 1))
    torch.set_num_threads(threads)
    h, _ = D.orientation_histogram(12, False)
    bs = args.cpu_batch
    fr = synth_frames(bs, args.size, args.size, 10_000)
    x = M.u8_nhwc_to_nchw_f32(fr)

    def predict(xb):
        o, p = M.forward(xb, sd)
        q = D.decode_orientation_batch(D.softmax_f32(o.numpy()), h)
        return o, p, q

    def timed(xb, n):
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            out = predict(xb)
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts), out

    t0 = time.perf_counter()
    predict(x)                                                          # warm-up at the timed batch size
    t_b, (o, p, q) = timed(x, 3)
    predict(x[:1])
    t_1, _ = timed(x[:1], 5)
    total = time.perf_counter() - t0
    base = {'value': round(bs / t_b, 3), 'unit': 'images/sec', 'cores': threads, 'kind': 'port',
            'sample': f'C3: {bs} synthetic {args.size}x{args.size} frames per batch, FP32 torch CPU forward + NumPy '
                      f'softmax/Markley decode (oracle/, pinned to the reference by tests/golden); 1 warm-up batch, '
                      f'median of 3; {threads} threads; {total:.1f} s for C3 + C1 together',
            'cpu_model': ci['model'], 'sockets': ci['sockets'], 'socket_physical_cores': ci['cores_per_socket'],
            'cpu_quota': ci['cpu_quota'], 'affinity_cpus': ci['affinity'],
            'c1_b1': {'images_per_sec': round(1.0 / t_1, 3), 'latency_ms': round(t_1 * 1e3, 2),
                      'protocol': 'B=1, 1 warm-up, median of 5, same threads'}}
    return base, (fr, o.numpy(), p.numpy(), q)


def pose_error(eng, dev, fr, o_ref, p_ref, q_ref, tolerance):
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
    rec = {'frames': int(fr.shape[0]), 'ori_logit_max_abs': float(np.abs(o.cpu().numpy() - o_ref).max()),
           'pos_max_abs_m': float(np.abs(p.cpu().numpy() - p_ref).max()), 'ori_max_deg': float(ang.max()),
           'tolerance': tolerance}
    if tolerance.startswith('logits'):
        rec['within_tolerance'] = bool(rec['ori_logit_max_abs'] < 1e-3 and rec['pos_max_abs_m'] < 1e-3 and
                                       rec['ori_max_deg'] < 0.1)
    else:
        rec['within_fp32_tolerance'] = bool(rec['ori_logit_max_abs'] < 1e-3 and rec['pos_max_abs_m'] < 1e-3 and
                                            rec['ori_max_deg'] < 0.1)
        rec['within_int8_tolerance'] = bool(rec['ori_logit_max_abs'] < INT8_BOUND[0] and
                                            rec['pos_max_abs_m'] < INT8_BOUND[1] and rec['ori_max_deg'] < INT8_BOUND[2])
    return rec


def device_batches(B, S, first, n_buf, dev):
    """n_buf distinct device batches: synthetic frames (seed, global index), each further buffer a spatially
    rolled copy (distinct bytes, same statistics) made on the device."""
    import torch
    base = torch.from_numpy(synth_frames(B, S, S, first)).to(dev)
    return [base] + [torch.roll(base, shifts=(37 * k, 53 * k), dims=(1, 2)).contiguous() for k in range(1, n_buf)]


def time_steps(step, n_warm, n_steps, sync, barrier, probe=None, settle_s=0.0, keep=None):
    """W warm-up steps, then exactly K timed steps bracketed by barrier + device sync on both sides. ``probe``
    (measure.ClockProbe) stamps the shader clock just outside the bracket (its kernels are synchronised before t0
    and launched after t1). ``settle_s``: before the W warm-up steps, the same steps run untimed for at least this
    long (synchronised every 8 steps), so the timed region sees the shader clock the GPU holds under this load
    rather than its ramp out of idle: measured on MI355X, 20 steps right after 5 warm-up steps ran at 2,030-2,090 MHz
    and 80.0-82.2k img/s, 100 steps at 2,290 MHz and 92.1k img/s (same box, same build).
    ``keep``: called with every timed step's output (e.g. to collect each step's decode status)."""
    i = 0
    t = time.perf_counter()
    while time.perf_counter() - t < settle_s:
        for _ in range(8):
            step(i)
            i += 1
        sync()
    for i in range(n_warm):
        step(i)
    sync()
    barrier()
    if probe is not None:
        probe.start()
    sync()
    t0 = time.perf_counter()
    out = None
    for i in range(n_steps):
        out = step(i)
        if keep is not None:
            keep(out)
    sync()
    barrier()
    sync()
    el = time.perf_counter() - t0
    if probe is not None:
        probe.stop()
    return el, out


def roofline(prof, steps, B, traffic_path, peaks=None, int8=False):
    """Dominant kernel (longest per step): MFMA bound (SURVEY §8d headline) with the HBM figure beside it; ``frac``
    against the nominal peak, ``frac_measured`` against the peak measured on this box (measure.measure_peaks)."""
    dom_key = max(prof, key=lambda k: prof[k][1])
    n, ms, byts, fl = prof[dom_key]
    avg_s = ms / n / 1e3
    ach_gbs = byts / n / avg_s / 1e9
    ach_tfl = fl / n / avg_s / 1e12
    traffic = pmc_traffic(dom_key, traffic_path)
    if traffic is not None:
        traffic *= B / 64.0     # the PMC passes ran batch 64 (tools/pmc.sh); bytes scale with the batch
    rec = {'bound': 'mfma', 'kernel': dom_key, 'achieved': round(ach_tfl, 2), 'peak': MFMA_PEAK_TFLOPS,
            'unit': 'TFLOP/s', 'frac': round(ach_tfl / MFMA_PEAK_TFLOPS, 4),
            'traffic': None if traffic is None else round(traffic),
            'traffic_source': os.path.relpath(traffic_path, ROOT) if traffic is not None else None,
            'traffic_over_algorithmic': None if traffic is None or not byts else round(traffic / (byts / n), 3),
            'algorithmic_flops_per_launch': round(fl / n), 'algorithmic_bytes_per_launch': round(byts / n),
            'avg_launch_us': round(avg_s * 1e6, 2), 'launches_per_step': n / steps,
            'hbm': {'achieved': round(ach_gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                    'frac': round(ach_gbs / HBM_PEAK_GBS, 4)}}
    if int8:
        rec['peak'], rec['unit'] = 2 * MFMA_PEAK_TFLOPS, 'TOP/s'
        rec['frac'] = round(ach_tfl / rec['peak'], 4)
    if peaks:
        pm = peaks['int8_mfma_tops' if int8 else 'fp16_mfma_tflops']
        rec['peak_measured'], rec['frac_measured'] = pm, round(ach_tfl / pm, 4) if pm else None
        hm = peaks['hbm_read_gbs']
        rec['hbm']['peak_measured'], rec['hbm']['frac_measured'] = hm, round(ach_gbs / hm, 4) if hm else None
    return rec


HEADLINE_MAX_BYTES = 6000   # the driver parses the LAST stdout line from an 8 KB tail (BENCH_r05: a 22.5 KB line failed)


def _clock(c):
    return None if not isinstance(c, dict) else {k: c[k] for k in ('sclk_mhz', 'spread_mhz') if k in c}


def compact_record(full: dict, detail_path=None) -> dict:
    """The headline JSON line: the contract fields, ``roofline``, ``cpu_baseline``, ``peak_measured``, the pose errors
    and a one-line summary of every sub-record (img/s + tolerance flag). Per-kernel tables and the sub-records
    themselves stay in ``full`` (written to the sidecar ``detail_path``), so the line stays a few KB."""
    keep = ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better', 'scaling',
            'vs_baseline', 'dtype', 'arith', 'data', 'config', 'clock_settle_s', 'graphs', 'dry_run',
            'mfma_utilisation_whole_net', 'mfma_utilisation_whole_net_measured_peak', 'cpu_baseline',
            'pose_err_vs_fp32', 'within_north_star')
    rec = {k: full[k] for k in keep if k in full}
    if 'sclk_timed_region' in full:
        rec['sclk_timed_region'] = _clock(full['sclk_timed_region'])
    if isinstance(full.get('peak_measured'), dict):
        rec['peak_measured'] = {k: v for k, v in full['peak_measured'].items() if not isinstance(v, (dict, str))}
    if isinstance(full.get('roofline'), dict):
        rf = dict(full['roofline'])
        rf.pop('sclk_leg', None)
        rec['roofline'] = rf
    sh = full.get('pose_err_vs_fp32_sharp_head')
    if isinstance(sh, dict):
        rec['pose_err_vs_fp32_sharp_head'] = {
            'frames': sh.get('frames'), 'head': sh.get('head'),
            **({full['dtype']: sh[full['dtype']]} if full.get('dtype') in sh else {}),
            'within_tolerance_by_dtype': {k: v['within_tolerance'] for k, v in sh.items()
                                          if isinstance(v, dict) and 'within_tolerance' in v}}
    subs = {}
    for k in ('c5', 'fp16x2', 'fp16'):
        s = full.get(k)
        if isinstance(s, dict):
            pe = s.get('pose_err_vs_fp32', {})
            subs[k] = {'value': s.get('value'), 'dtype': s.get('dtype'),
                       'roofline_frac': s.get('roofline_kernel', {}).get('frac'),
                       **{f: pe[f] for f in ('ori_logit_max_abs', 'within_tolerance', 'within_int8_tolerance')
                          if f in pe}}
    kp = full.get('keypoint_mode')
    if isinstance(kp, dict):
        subs['keypoint_mode'] = {dt: {'value': kp[dt].get('value'),
                                      'within_tolerance': kp[dt].get('pose_err_vs_fp32', {}).get('within_tolerance'),
                                      'pos_max_m': kp[dt].get('pose_err_vs_fp32', {}).get('pos_max_m')}
                                 for dt in ('fp32', 'fp16x2', 'fp16') if isinstance(kp.get(dt), dict)}
        if isinstance(kp.get('epnp'), dict):
            subs['epnp'] = {k: kp['epnp'].get(k) for k in ('value', 'unit', 'latency_b64_us', 'kat_max_ori_deg')}
    if subs:
        rec['sub_records'] = subs
    if detail_path:
        rec['detail'] = detail_path
    return rec


def kernel_table(prof, steps):
    return {k: {'launches_per_step': v[0] / steps, 'ms_per_step': round(v[1] / steps, 4),
                'GB/s': round(v[2] / (v[1] / 1e3) / 1e9, 1) if v[1] > 0 else None,
                'TFLOP/s': round(v[3] / (v[1] / 1e3) / 1e12, 2) if v[1] > 0 else None}
            for k, v in sorted(prof.items(), key=lambda kv: -kv[1][1])}


def newest_profile(names):
    """The first of the committed profiles/ summaries (newest first) that exists; the last name otherwise."""
    paths = [os.path.join(ROOT, 'profiles', n) for n in names]
    return next((p for p in paths if os.path.exists(p)), paths[-1])


def run_int8(args, sd, dev, frames, ref, peaks=None):
    """C5 sub-record: the INT8 (Brevitas-mirroring) path at the same workload, same timing protocol (N=1)."""
    from spef_amd.blob_q8 import pack_int8
    from spef_amd.quant import calibrate
    blob = pack_int8(sd, calibrate(sd, synth_frames(4, 128, 128, 900)))
    return run_variant(args, blob, 'int8', dev, frames, ref, peaks)


def set_wavespec(pipe, args) -> None:
    """--wavespec / --q8-rolesplit: the late-block schedule of every engine in the pipeline (A/B aids)."""
    from spef_amd import _lib as L
    extra = [tuple(int(v) for v in o.split('=')) for o in args.set_option]
    if getattr(args, 'graphs', False):
        pipe.use_graphs()
    for opt, val in [(L.OPT_WAVESPEC, args.wavespec), (L.OPT_Q8_ROLESPLIT, args.q8_rolesplit)] + extra:
        if val is not None:
            for e in pipe.engines:
                e.set_option(opt, val)


def run_variant(args, blob, dtype, dev, frames, ref, peaks=None):
    """A precision variant's sub-record at the headline workload and timing protocol (N=1): int8 (C5) or fp16x2
    (the fp32-accurate split-fp16 schedule)."""
    import torch
    from spef_amd import _lib as L
    from spef_amd.pipeline import StreamPipeline
    from spef_amd.spe.spe_utils import SPEUtils
    su = SPEUtils(None, 'classification', 12, 3, False, 'regression')
    pipe = StreamPipeline(blob, dev, depth=max(1, args.inflight), ori_bins=su.orientation.histogram)
    set_wavespec(pipe, args)
    B, S = args.batch, args.size
    pipe.reserve(B, S, S)

    def step(i):
        return pipe.submit(frames[i % len(frames)], L.CLASSIFICATION, L.REGRESSION, want_soft=True)
    sync = lambda: (pipe.synchronize(), torch.cuda.synchronize(dev))   # noqa: E731
    probe = ClockProbe(dev)
    el, _ = time_steps(step, args.warmup, args.steps, sync, lambda: None, probe, args.settle)
    eng = pipe.engine
    eng.profile_begin()
    for i in range(args.steps):
        o, p = eng.forward(frames[i % len(frames)])
        eng.decode(1, 0, o, p, want_soft=True)
    prof = eng.profile_end()
    int8 = dtype == 'int8'
    rec = {'workload': (f'C5: INT8 (Brevitas-mirroring, PTQ-calibrated scales) full net + decode, {S}x{S}, batch {B}'
                        if int8 else f'C3 {dtype}: full net + decode, {S}x{S}, batch {B} ({ARITH[dtype]})'),
           'value': round(B * args.steps / el, 2), 'unit': 'images/sec', 'ms_per_step': round(el / args.steps * 1e3, 4),
           'dtype': dtype, 'sclk_timed_region': probe.mhz(),
           'roofline_kernel': roofline(prof, args.steps, B, newest_profile(TRAFFIC[dtype]), peaks, int8=int8),
           'kernels': kernel_table(prof, args.steps)}
    if ref is not None:
        rec['pose_err_vs_fp32'] = pose_error(eng, dev, *ref, tolerance=INT8_TOLERANCE if int8 else
                                             'logits 1e-3, pose 0.1 deg / 1 mm (BASELINE.json north_star)')
    pipe.close()
    return rec


def sharp_head(args, dev, fr):
    """'pose err vs fp32 ref' with a sharp orientation head: the bench's backbone weights with the
    orientation Linear at std 0.3 (logits up to ~20, peaked histograms; the reference-generated predict fixtures' scale,
    tests/golden/cases.py) and a SPEED-range position bias, on the CPU baseline's frames, for the fp16mx headline, the
    fp16 schedule and the fp16x2 parity variant, against the FP32 oracle at the north star's absolute bounds."""
    import numpy as np
    import torch
    from oracle import decode_ref as D
    from oracle import model_ref as M
    from spef_amd import blob as Bl
    from spef_amd.arch import mobilenet_v2
    from spef_amd.engine import Engine
    from spef_amd.weights import synthetic_state_dict
    n = min(args.sharp_frames, fr.shape[0])
    fr = fr[:n]
    sd = synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=1001, head_std=0.3, pos_std=0.01,
                              pos_bias=(0.3, -0.2, 12.0))
    ro, rp = M.forward(M.u8_nhwc_to_nchw_f32(fr), sd)
    ro, rp = ro.numpy(), rp.numpy()
    h, _ = D.orientation_histogram(12, False)
    rq = D.decode_orientation_batch(D.softmax_f32(ro), h)
    out = {'frames': n, 'head': 'ori Linear std 0.3 (logit max |%.1f|), pos std 0.01 + bias (0.3, -0.2, 12.0) m'
                                % float(np.abs(ro).max())}
    for dt in ('fp16mx', 'fp16', 'fp16x2'):
        e = Engine(Bl.pack(sd, dtype=dt), dev)
        e.set_decode_tables(h, None)
        o, p = e.forward(torch.from_numpy(fr).to(dev))
        dec = e.decode(1, 0, o, p)
        ang = D.angle_deg_stable(dec['ori'].cpu().numpy().astype(np.float64), rq)
        r = {'ori_logit_max_abs': float(np.abs(o.cpu().numpy() - ro).max()),
             'pos_max_abs_m': float(np.abs(p.cpu().numpy() - rp).max()), 'ori_max_deg': float(ang.max())}
        r['within_tolerance'] = bool(r['ori_logit_max_abs'] < 1e-3 and r['pos_max_abs_m'] < 1e-3 and
                                     r['ori_max_deg'] < 0.1)
        out[dt] = r
        e.close()
    return out


def run_keypoint(args, dev, with_ref: bool):
    """Keypoint mode of C3: KeypointRegressionHead (only defined at 240x384, keypoints.py:20) +
    sigmoid + batched EPnP, batch ``args.batch``; the fp32 blob (the parity variant, build_mi355x's keypoint
    default) and the fp16 fast variant, each with img/s and pose error against the FP32 oracle (forward + EPnP
    restatement) on the same frames. Plus EPnP alone at 512 problems per launch (problems/s, kernel time from HIP
    events) on the reference's own projections of valid.json poses (tests/golden/keypoints.npz)."""
    import numpy as np
    import torch
    from spef_amd import blob as Bl
    from spef_amd.arch import mobilenet_v2
    from spef_amd.engine import Engine
    from spef_amd.weights import plant_keypoint_head, synthetic_state_dict
    g = np.load(os.path.join(ROOT, 'tests', 'golden', 'keypoints.npz'))
    kp3d, K, nu, nv = g['kp3d'], g['K'], float(g['nu']), float(g['nv'])
    arch = mobilenet_v2('keypoints')
    # the head outputs real keypoints (bias = logit of the reference projection of the valid.json pose at the median
    # distance, small weights): a random head clusters the keypoints and makes EPnP ill-conditioned
    ip = int(np.argmin(np.abs(g['t'][:, 2] - np.median(g['t'][:, 2]))))
    sd = plant_keypoint_head(synthetic_state_dict(arch, seed=1001, head_std=2e-4), g['kp2d'][ip])
    B, H, W = args.batch, 240, 384
    fr = synth_frames(B, H, W, 20_000)
    xg = torch.from_numpy(fr).to(dev)
    rec = {'workload': f'C3 keypoint mode: MobileNetV2 + KeypointRegressionHead + sigmoid + batched EPnP, {H}x{W}, '
                       f'batch {B} (uint8 frames resident in HBM, {max(1, args.inflight)} batches in flight as the '
                       f'headline); head bias planted at the reference projection of valid.json pose {ip}'}
    ref = None
    if with_ref:
        from oracle import decode_ref as D
        from oracle import epnp_ref as E
        from oracle import model_ref as M
        raw_ref = M.forward(M.u8_nhwc_to_nchw_f32(fr), sd, head='keypoints').numpy()
        rq, rt = E.decode_batch(D.sigmoid_f32(raw_ref), kp3d, K)
        ref = (raw_ref, rq, rt, D)
    from spef_amd.pipeline import StreamPipeline
    for dtype in ('fp32', 'fp16x2', 'fp16'):
        # timed as the headline: --inflight batches on separate streams (batch k's EPnP and late blocks overlap batch
        # k+1's early blocks), every step the complete forward + sigmoid + EPnP of one batch
        pipe = StreamPipeline(Bl.pack(sd, arch, dtype=dtype), dev, depth=max(1, args.inflight))
        set_wavespec(pipe, args)
        pipe.set_keypoints(kp3d, K, nu, nv)
        pipe.reserve(B, H, W)
        statuses = []
        sync = lambda: (pipe.synchronize(), torch.cuda.synchronize(dev))   # noqa: E731
        n = max(5, args.steps // 4)
        el, _ = time_steps(lambda i: pipe.submit_keypoints(xg), max(2, args.warmup // 2), n, sync, lambda: None,
                           settle_s=args.settle, keep=lambda o: statuses.append(o['status']))
        bad = int(sum(int((st != 0).sum().item()) for st in statuses))
        r = {'value': round(B * n / el, 2), 'unit': 'images/sec', 'ms_per_step': round(el / n * 1e3, 4), 'steps': n,
             'inflight': pipe.depth, 'epnp_failed_problems': bad}
        eng = pipe.engine   # single-stream leg: the per-kernel table and the pose error

        def step(i):
            raw, _ = eng.forward(xg)
            return raw, eng.decode_keypoints(raw)
        raw, out = step(0)
        torch.cuda.synchronize(dev)
        eng.profile_begin()
        for _ in range(n):
            step(0)
        r['kernels'] = kernel_table(eng.profile_end(), n)
        if ref is not None:
            raw_ref, rq, rt, D = ref
            ang = D.angle_deg_stable(out['ori'].cpu().numpy().astype(np.float64), rq)
            dt = np.linalg.norm(out['pos'].cpu().numpy().astype(np.float64) - rt, axis=1)
            r['pose_err_vs_fp32'] = {'raw_max_abs': float(np.abs(raw.cpu().numpy() - raw_ref).max()),
                                     'ori_max_deg': float(ang.max()), 'ori_median_deg': float(np.median(ang)),
                                     'pos_max_m': float(dt.max()), 'pos_median_m': float(np.median(dt))}
            r['pose_err_vs_fp32']['within_tolerance'] = bool(r['pose_err_vs_fp32']['raw_max_abs'] < 1e-3 and
                                                             ang.max() < 0.1 and dt.max() < 1e-3)
        rec[dtype] = r
        if dtype == 'fp32':   # EPnP alone: B = 64 (the keypoint step's launch), 512, and all 1,800 reference poses
            from spef_amd.quaternion import angle_deg
            by_p = {}
            for P in (64, 512, len(g['kp2d'])):
                kp = torch.from_numpy(np.ascontiguousarray(g['kp2d'][:P], np.float32)).to(dev)
                o = eng.decode_keypoints(kp, apply_sigmoid=False)
                torch.cuda.synchronize(dev)
                kat_deg = float(np.max(angle_deg(o['ori'].cpu().numpy(), g['q'][:P])))
                n_l = 100
                eng.profile_begin()
                t0 = time.perf_counter()
                for _ in range(n_l):
                    eng.decode_keypoints(kp, apply_sigmoid=False)
                torch.cuda.synchronize(dev)
                wall = time.perf_counter() - t0
                prof = eng.profile_end()
                kn, kms = prof['epnp_kernel'][0], prof['epnp_kernel'][1]
                by_p[P] = {'problems_per_launch': P, 'launches': n_l, 'value': round(P * kn / (kms / 1e3), 1),
                           'kernel_us_per_launch': round(kms / kn * 1e3, 2), 'value_wall': round(P * n_l / wall, 1),
                           'kat_max_ori_deg': kat_deg,
                           'kat_max_pos_m': float(np.linalg.norm(o['pos'].cpu().numpy() - g['t'][:P], axis=1).max())}
            # value: the full reference set per launch (1,800 workgroups: the GPU's throughput); the B = 64 launch of a
            # keypoint step (one problem per workgroup on 64 CUs) is the latency figure
            rec['epnp'] = dict(by_p[len(g['kp2d'])], unit='problems/sec',
                               latency_b64_us=by_p[64]['kernel_us_per_launch'],
                               by_problems={str(k): v for k, v in by_p.items()},
                               sample='noise-free reference projections of the valid.json poses '
                                      '(tests/golden/keypoints.npz, KeyPoints.project of the reference)')
        pipe.close()
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=100)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--settle', type=float, default=0.5,
                    help='seconds of untimed steps before the warm-up steps (shader clock out of idle; 0 = off)')
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--size', type=int, default=512)
    ap.add_argument('--dtype', default='fp16mx', choices=['fp16mx', 'fp16', 'fp16x2', 'bf16', 'int8'],
                    help='headline schedule: fp16mx (default; within 1e-3 at trained head scales), fp16 (fast; misses '
                         '1e-3 at sharp heads), fp16x2 (fp32 activations), bf16, int8 (the Brevitas-mirroring C5 path)')
    ap.add_argument('--wavespec', type=int, default=None,
                    help='late-block schedule (SPEF_OPT_WAVESPEC): 0 slab kernels, 1 wave-specialised, 2 three-stage '
                         '(fp16 blocks 14-17; A/B aid; default: the library\'s)')
    ap.add_argument('--set-option', action='append', default=[], metavar='OPT=VALUE',
                    help='spef_set_option(OPT, VALUE) on every engine (schedule / tuning A/B aid; include/spef.h, '
                         'csrc/spef_tuning.hpp)')
    ap.add_argument('--q8-rolesplit', type=int, default=None,
                    help='int8 blocks 8-17 as role-split kernels (SPEF_OPT_Q8_ROLESPLIT 1) or slab kernels (0, the '
                         'library default)')
    ap.add_argument('--inflight', type=int, default=3,
                    help='batches in flight: consecutive steps alternate over this many HIP streams (spef_amd.pipeline)')
    ap.add_argument('--graphs', action='store_true',
                    help='replay each (stream, input batch) forward + decode as a recorded HIP graph (StreamPipeline.use_graphs)')
    ap.add_argument('--frame-buffers', type=int, default=6,
                    help='distinct device batches the timed steps rotate over (6 x 50 MB > 256 MB Infinity Cache)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-int8', action='store_true', help='skip the C5 (int8) sub-record')
    ap.add_argument('--no-keypoint', action='store_true', help='skip the keypoint-mode / EPnP sub-record')
    ap.add_argument('--no-x2', action='store_true', help='skip the fp16x2 (fp32-accurate) sub-record')
    ap.add_argument('--no-fp16', action='store_true', help='skip the fp16 (fast schedule) sub-record')
    ap.add_argument('--sharp-frames', type=int, default=16,
                    help='frames of the sharp-head pose-error check (FP32 oracle on the CPU: ~0.1 s per frame)')
    ap.add_argument('--no-peaks', action='store_true', help='skip the on-box peak microbenchmark')
    ap.add_argument('--cpu-threads', type=int, default=0, help='0 = one socket\'s physical cores (capped by quota)')
    ap.add_argument('--cpu-batch', type=int, default=64)
    ap.add_argument('--traffic', default=None,
                    help='committed rocprofv3 FETCH/WRITE summary used for roofline.traffic (default: the newest '
                         'committed profiles/*_pmc_traffic.json of the path)')
    ap.add_argument('--detail-out', default=os.path.join('gpurun_out', 'bench_detail.json'),
                    help='sidecar file for the full record (per-kernel tables, every sub-record); \'\' = none')
    ap.add_argument('--dry-run', action='store_true',
                    help='CPU + gloo: the distributed control flow (weight distribution, timing, max over ranks, '
                         'JSON) without device work')
    args = ap.parse_args()
    if args.graphs:   # every (stream, frame buffer) key recorded before timing starts (recording is not timed work)
        import math
        args.warmup = max(args.warmup, math.lcm(max(1, args.inflight), args.frame_buffers))
    if args.traffic is None:   # the newest committed FETCH/WRITE summary of this path
        args.traffic = newest_profile(TRAFFIC[args.dtype])

    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.dry_run:
        dev = torch.device('cpu')
        if world > 1:
            os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
            dist.init_process_group('gloo', rank=rank, world_size=world)
    else:
        dev = torch.device(f'cuda:{local}')
        torch.cuda.set_device(dev)
        if world > 1:
            os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
            dist.init_process_group('nccl', rank=rank, world_size=world, device_id=dev)

    from spef_amd import blob as Bl
    from spef_amd.arch import flops_per_image, mobilenet_v2
    from spef_amd.shard import broadcast_blob, max_over_ranks, shard_range
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
    B, S = args.batch, args.size
    first, stop = shard_range(B * world, rank, world)          # this rank's global frame indices
    barrier = (lambda: dist.barrier()) if world > 1 else (lambda: None)

    if args.dry_run:
        # weights travel over the process group (gloo) and every rank validates what it received (host C ABI)
        import ctypes as C
        from spef_amd import _lib as L
        got = broadcast_blob(blob, dev).numpy().tobytes()
        L.check(L.load().spef_validate_blob(C.create_string_buffer(got, len(got)), len(got), None, None, None, None))
        frames = [synth_frames(stop - first, 32, 32, first)]
        step = lambda i: {'status': torch.zeros(1, dtype=torch.int32)}   # noqa: E731
        sync = lambda: None                                                # noqa: E731
        prof = None
    else:
        from spef_amd import _lib as L
        from spef_amd.pipeline import StreamPipeline
        from spef_amd.spe.spe_utils import SPEUtils
        comm = None
        if world > 1:   # the library's RCCL communicator carries the weights over xGMI (spef_bcast_weights)
            from spef_amd.shard import RcclComm
            comm = RcclComm(dev)
        su = SPEUtils(None, 'classification', 12, 3, False, 'regression')
        pipe = StreamPipeline(blob, dev, depth=max(1, args.inflight), ori_bins=su.orientation.histogram, comm=comm)
        set_wavespec(pipe, args)
        eng = pipe.engine
        frames = device_batches(stop - first, S, first, max(1, args.frame_buffers), dev)
        pipe.reserve(B, S, S)

        def step(i):   # one batch: forward + decode, on the next of --inflight streams
            return pipe.submit(frames[i % len(frames)], L.CLASSIFICATION, L.REGRESSION, want_soft=True)

        def sync():
            pipe.synchronize()
            torch.cuda.synchronize(dev)

    peaks = None
    probe = None
    if not args.dry_run:
        if rank == 0 and not args.no_peaks:
            peaks = measure_peaks(local)                   # < 1 s, before the warm-up
        probe = ClockProbe(dev)
        barrier()
    statuses = []
    elapsed, out = time_steps(step, args.warmup, args.steps, sync, barrier, probe,
                              0.0 if args.dry_run else args.settle, keep=lambda o: statuses.append(o['status']))
    elapsed = max_over_ranks(elapsed, dev)
    assert len(statuses) == args.steps and not torch.stack(statuses).any().item(), 'decode reported NaN in a timed step'

    leg_probe = None
    if not args.dry_run:
        # roofline leg: per-kernel HIP events on the engine's stream, K more steps on one stream, with the shader
        # clock of the leg stamped around it (the roofline's achieved rate is priced at this clock)
        leg_probe = ClockProbe(dev)
        leg_probe.start()
        eng.profile_begin()
        for i in range(args.steps):
            o, p = eng.forward(frames[i % len(frames)])
            eng.decode(1, 0, o, p, want_soft=True)
        prof = eng.profile_end()
        leg_probe.stop()

    if rank == 0:
        total_img = B * args.steps * world
        value = total_img / elapsed
        fpi = flops_per_image(S, S)
        peak = 2 * MFMA_PEAK_TFLOPS if args.dtype == 'int8' else MFMA_PEAK_TFLOPS
        rec = {
            'metric': METRIC,
            'value': round(value, 2),
            'unit': 'images/sec',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'clock_settle_s': 0.0 if args.dry_run else args.settle,
            **({'graphs': 'replayed HIP graphs: each replay reuses its key\'s graph-owned outputs, so the per-step '
                          'decode-status check sees the last replay of every (stream, frame buffer) key'}
               if args.graphs else {}),
            'ms_per_step': round(elapsed / args.steps * 1e3, 4),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': args.dtype,
            'arith': ARITH[args.dtype],
            'data': f'synthetic SPEED-style uint8 frames resident in HBM, {max(1, args.frame_buffers)} distinct '
                    f'batches rotated; seeded random weights (BN-calibrated)',
            'config': {'workload': (f'C5: INT8 (Brevitas-mirroring, calibrated scales) full net + decode, {S}x{S}, '
                                    f'batch {B} per GPU' if args.dtype == 'int8' else
                                    f'C3: full net + decode, {S}x{S}, batch {B} per GPU, {args.dtype} schedule'),
                       'global_batch': B * world,
                       'image_size': S, 'parallelism': f'frame-parallel x{world} (RCCL weight bcast)',
                       'inflight_batches': max(1, args.inflight), 'frame_buffers': max(1, args.frame_buffers)},
            'mfma_utilisation_whole_net': round(fpi * value / world / 1e12 / peak, 5),
        }
        if peaks:
            pm = peaks['int8_mfma_tops' if args.dtype == 'int8' else 'fp16_mfma_tflops']
            rec['mfma_utilisation_whole_net_measured_peak'] = round(fpi * value / world / 1e12 / pm, 5)
            rec['peak_measured'] = peaks
        if probe is not None:
            rec['sclk_timed_region'] = probe.mhz()
        if args.dry_run:
            rec['dry_run'] = True
        else:
            rec['roofline'] = roofline(prof, args.steps, B, args.traffic, peaks, int8=args.dtype == 'int8')
            leg_clk = leg_probe.mhz()
            rec['roofline']['sclk_mhz'] = leg_clk['sclk_mhz'] if leg_clk else None
            rec['roofline']['sclk_leg'] = leg_clk
            rec['kernels'] = kernel_table(prof, args.steps)
            ref = None
            if world == 1 and not args.no_cpu_baseline:
                rec['cpu_baseline'], ref = cpu_baseline(args, sd)
                rec['pose_err_vs_fp32'] = pose_error(
                    eng, dev, *ref, tolerance='logits 1e-3, pose 0.1 deg / 1 mm (BASELINE.json north_star)')
            if world == 1 and args.dtype != 'int8' and not args.no_int8:
                rec['c5'] = run_int8(args, sd, dev, frames, ref, peaks)
            if world == 1 and args.dtype != 'fp16x2' and not args.no_x2:
                rec['fp16x2'] = run_variant(args, Bl.pack(sd, dtype='fp16x2'), 'fp16x2', dev, frames, ref, peaks)
            if world == 1 and args.dtype != 'fp16' and not args.no_fp16:
                rec['fp16'] = run_variant(args, Bl.pack(sd, dtype='fp16'), 'fp16', dev, frames, ref, peaks)
            if world == 1 and ref is not None and args.sharp_frames > 0:
                sh = sharp_head(args, dev, ref[0])
                rec['pose_err_vs_fp32_sharp_head'] = sh
                for k in ('fp16', 'fp16x2'):   # each sub-record carries its own sharp-head result too
                    if isinstance(rec.get(k), dict) and k in sh:
                        rec[k]['pose_err_vs_fp32_sharp_head'] = sh[k]
                if args.dtype in sh:
                    rec['within_north_star'] = bool(sh[args.dtype]['within_tolerance'] and
                                                    rec['pose_err_vs_fp32']['within_tolerance'])
            if world == 1 and not args.no_keypoint:
                rec['keypoint_mode'] = run_keypoint(args, dev, with_ref=not args.no_cpu_baseline)
        # full record (per-kernel tables, every sub-record) to the sidecar; the LAST stdout line is the compact headline
        detail = args.detail_out or None
        if detail:
            try:
                os.makedirs(os.path.dirname(os.path.abspath(detail)), exist_ok=True)
                with open(detail, 'w') as f:
                    json.dump(rec, f)
            except OSError as e:
                print(f'bench: could not write {detail}: {e}', file=sys.stderr)
                detail = None
        line = json.dumps(compact_record(rec, detail))
        if len(line) > HEADLINE_MAX_BYTES:
            print(f'bench: headline line {len(line)} B exceeds {HEADLINE_MAX_BYTES} B', file=sys.stderr)
        sys.stderr.flush()
        print(line, flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
