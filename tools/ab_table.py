"""Per-kernel us/step from r6_ab.sh's bench records (gpurun_out/ab_<variant><pass>.json): python tools/ab_table.py a b"""
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
names = sys.argv[1:]
acc = {n: defaultdict(list) for n in names}
val = {n: [] for n in names}
for n in names:
    for r in range(1, 20):
        p = os.path.join(ROOT, 'gpurun_out', f'ab_{n}{r}.json')
        if not os.path.exists(p):
            continue
        d = json.load(open(p))
        val[n].append(d['value'])
        for k, v in d['kernels'].items():
            acc[n][k].append(v['ms_per_step'] * 1e3)
mean = lambda v: sum(v) / len(v) if v else float('nan')  # noqa: E731
print(' '.join(f'{n}: {mean(val[n]):.0f} img/s ({len(val[n])})' for n in names))
keys = sorted(acc[names[0]], key=lambda k: -mean(acc[names[0]][k]))
print(f'{"kernel":40s}' + ''.join(f'{n:>10s}' for n in names))
for k in keys:
    print(f'{k:40s}' + ''.join(f'{mean(acc[n][k]):10.1f}' for n in names))
print(f'{"(sum)":40s}' + ''.join(f'{sum(mean(v) for v in acc[n].values()):10.1f}' for n in names))
