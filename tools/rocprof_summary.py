"""Turn rocprofv3 outputs (gpurun_out/) into the committed summaries under profiles/.

  python tools/rocprof_summary.py --tag r01 --stats gpurun_out/prof_r1 \
      --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write

Writes profiles/<tag>_kernel_stats.csv (copy of rocprofv3 --stats) and profiles/<tag>_pmc_traffic.json:
per kernel symbol, the mean HBM bytes per dispatch from separate FETCH_SIZE / WRITE_SIZE passes, corrected as
MI355X_MICROARCH.md §HBM prescribes: bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (FETCH_SIZE is KB and on
gfx950 reads half the bytes of a wide coalesced stream). Keys are short kernel names matching bench.py's keys.
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _demangle_spef(full: str) -> str:
    """Mangled symbols the profiler left as-is, e.g. '_ZN4spef15front_vp_kernelILi16ELi16ELi8EEEv...' ->
    'front_vp_kernel<16,16,8>' (integer and bool template arguments only; anything else is returned unchanged)."""
    m = re.match(r'_ZN4spef(\d+)', full)
    if not m:
        return full
    ln = int(m.group(1))
    name = full[m.end():m.end() + ln]
    rest = full[m.end() + ln:]
    if not rest.startswith('I'):
        return name
    args = re.findall(r'L[ib](\d+)E', rest[1:rest.find('EEE') + 1] if 'EEE' in rest else rest[1:])
    return f"{name}<{','.join(args)}>"


def short_name(full: str) -> str:
    """'void spef::pw_kernel<spef::F16, 6, 2, 1>(...)' -> 'pw_kernel<F16,6,2,1>' (bench.py key form)."""
    if full.startswith('_Z'):
        full = _demangle_spef(full)
    n = full.replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '').replace('spef::', '').strip()
    n = re.sub(r'\s+', '', n)
    n = n.replace('stem_kernel<F16,0>', 'stem_kernel<u8>').replace('stem_kernel<F16,1>', 'stem_kernel<f32>')
    n = n.replace('stem_kernel<BF16,0>', 'stem_kernel<u8>').replace('stem_kernel<BF16,1>', 'stem_kernel<f32>')
    n = re.sub(r'dw_kernel<B?F16,(\d)>', r'dw_kernel<\1>', n)
    n = re.sub(r'pw_pool_kernel<B?F16,(\d)>', r'pw_pool_kernel<\1>', n)
    n = re.sub(r'^q_irb_kernel<(\d+),(\d+),(\d+),(\d+),.*>$', r'q_irb_kernel<\1,\2,\3,s\4>', n)   # int8 path
    n = re.sub(r'^q_stem(_rows)?_kernel<false>$', 'q_stem_kernel<u8>', n)
    n = re.sub(r'^q_stem(_rows)?_kernel<true>$', 'q_stem_kernel<f32>', n)
    return n


def per_kernel(counter_dir: str, counter: str):
    f = glob.glob(os.path.join(counter_dir, '*counter_collection.csv'))[0]
    acc = defaultdict(list)
    for row in csv.DictReader(open(f)):
        if row['Counter_Name'] == counter:
            acc[short_name(row['Kernel_Name'])].append(float(row['Counter_Value']))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tag', required=True)
    ap.add_argument('--stats', required=True)
    ap.add_argument('--fetch')
    ap.add_argument('--write')
    ap.add_argument('--leg', type=int, default=0,
                    help="bench.py's single-stream HIP-event leg = the last LEG steps of the traced run")
    ap.add_argument('--total', type=int, default=0, help='all steps of the traced run (warmup + steps + leg)')
    ap.add_argument('--per-step', default='',
                    help='a kernel launched once per step (e.g. front_vp_kernel): the leg of every kernel is then its '
                         'last LEG x (its dispatches / this kernel\'s dispatches), whatever the number of steps '
                         '(bench.py\'s time-based settle phase makes --total unknown)')
    a = ap.parse_args()
    out = os.path.join(ROOT, 'profiles')
    os.makedirs(out, exist_ok=True)
    st = glob.glob(os.path.join(a.stats, '*kernel_stats.csv'))[0]
    shutil.copy(st, os.path.join(out, f'{a.tag}_kernel_stats.csv'))
    if a.leg and (a.total or a.per_step):
        # Per kernel, the dispatches of bench.py's roofline leg (one stream, no overlap with other batches): the
        # durations bench.py's HIP events measure. The pipelined steps before it overlap up to --inflight batches,
        # which stretches their individual kernel durations in the --stats average.
        tr = glob.glob(os.path.join(a.stats, '*kernel_trace.csv'))[0]
        by = defaultdict(list)
        for r in csv.DictReader(open(tr)):
            by[short_name(r['Kernel_Name'])].append((int(r['Start_Timestamp']), int(r['End_Timestamp'])))
        with open(os.path.join(out, f'{a.tag}_kernel_stats_leg.csv'), 'w', newline='') as f:
            w = csv.writer(f)
            w.writerow(['Name', 'LegCalls', 'AverageNs', 'MinNs', 'MaxNs', 'AllCalls', 'AllAverageNs'])
            for k, v in sorted(by.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
                v.sort()
                if a.per_step:
                    ref = next(len(x) for kk, x in by.items() if kk.startswith(a.per_step))
                    n = max(1, min(len(v), round(a.leg * len(v) / ref)))
                else:
                    n = max(1, round(len(v) * a.leg / a.total))
                d = [e - s for s, e in v[-n:]]
                alld = [e - s for s, e in v]
                w.writerow([k, n, round(sum(d) / n, 1), min(d), max(d), len(v), round(sum(alld) / len(alld), 1)])
    if a.fetch and a.write:
        fe, n = per_kernel(a.fetch, 'FETCH_SIZE')
        wr, _ = per_kernel(a.write, 'WRITE_SIZE')
        res = {k: {'hbm_bytes_per_launch': (2 * fe[k] + wr.get(k, 0.0)) * 1024, 'fetch_kb': fe[k],
                   'write_kb': wr.get(k, 0.0), 'dispatches': n[k]} for k in fe}
        json.dump({'correction': 'bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md HBM)',
                   'kernels': res}, open(os.path.join(out, f'{a.tag}_pmc_traffic.json'), 'w'), indent=1)
    print('wrote profiles for', a.tag)


if __name__ == '__main__':
    main()
