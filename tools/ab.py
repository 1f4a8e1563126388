"""A/B per-kernel timing of two builds of the HIP library on the GPU box (same box, interleaved runs, so box-to-box
clock differences cancel): python tools/ab.py ab/old.so [new.so] [rounds]. Prints per-kernel us/step for each build
(mean over rounds) and the difference. The second build defaults to the in-tree library."""
import os
import re
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(lib):
    env = dict(os.environ, SWEEP='0')
    if lib:
        env['SPEF_LIB'] = lib
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'explore.py')], env=env, capture_output=True,
                         text=True, timeout=300).stdout
    res = {}
    for line in out.splitlines():
        m = re.match(r'\s+([\d.]+) us\s+x\s*[\d.]+\s+\d+ GB/s\s+[\d.]+ TF/s\s+(\S.*)$', line)
        if m:
            res[m.group(2)] = float(m.group(1))
        m = re.search(r'kernel sum ([\d.]+) ms/step', line)
        if m:
            res['(kernel sum)'] = float(m.group(1)) * 1e3
    return res


def main():
    a = sys.argv[1]
    b = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].isdigit() else ''
    rounds = int(sys.argv[-1]) if sys.argv[-1].isdigit() else 2
    acc = {'A': defaultdict(list), 'B': defaultdict(list)}
    for r in range(rounds):   # alternate the order (A B, B A, ...): the second run of a pair is systematically slower
        for tag, lib in ((('A', a), ('B', b)) if r % 2 == 0 else (('B', b), ('A', a))):
            for k, v in run(lib).items():
                acc[tag][k].append(v)
    mean = lambda v: sum(v) / len(v) if v else float('nan')  # noqa: E731
    keys = sorted(set(acc['A']) | set(acc['B']), key=lambda k: -max(mean(acc['A'].get(k)), mean(acc['B'].get(k)),
                                                                 key=lambda x: x if x == x else -1))
    print(f'{"A us":>9} {"B us":>9} {"B-A":>8}  kernel   (A={a}, B={b or "in-tree"}, {rounds} rounds)')
    for k in keys:
        ma, mb = mean(acc['A'].get(k)), mean(acc['B'].get(k))
        print(f'{ma:9.1f} {mb:9.1f} {mb - ma:+8.1f}  {k}')


if __name__ == '__main__':
    main()
