"""Mean per-kernel us/step per build from tools/ktime.sh's gpurun_out/kt.txt (lines '<name> {json}')."""
import json
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
order = []
for line in open(sys.argv[1]):
    name, _, js = line.partition(' ')
    if not js.strip():
        continue
    if name not in order:
        order.append(name)
    for k, v in json.loads(js).items():
        acc[name][k].append(v)
mean = lambda v: sum(v) / len(v)  # noqa: E731
keys = sorted(acc[order[0]], key=lambda k: -mean(acc[order[0]][k]))
print(f'{"kernel":36s}' + ''.join(f'{n:>9s}' for n in order))
for k in keys:
    print(f'{k[:36]:36s}' + ''.join(f'{mean(acc[n][k]):9.1f}' if k in acc[n] else '        -' for n in order))
print(f'{"(sum)":36s}' + ''.join(f'{sum(mean(v) for v in acc[n].values()):9.1f}' for n in order))
