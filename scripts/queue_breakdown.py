"""Per-queue, per-kernel time per step from a rocprofv3 kernel_trace.csv of bench.py (steps are
delimited by the first kernel of the step's marker, default the SA1 FPS / the first kNN)."""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
marker = sys.argv[2] if len(sys.argv) > 2 else None
if marker is None:
    marker = 'fps_kernel<512' if any('fps_kernel<512' in r['Kernel_Name'] for r in rows) else 'knn_wave_kernel<3'
idx = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
agg = defaultdict(lambda: defaultdict(lambda: [0, 0.0]))
steps = list(range(max(0, len(idx) - 8), len(idx) - 1))
spans = []
for k in steps:
    seg = rows[idx[k]:idx[k + 1]]
    spans.append((int(seg[-1]['End_Timestamp']) - int(seg[0]['Start_Timestamp'])) / 1e3)
    for r in seg:
        name = re.sub(r'\(.*', '', r['Kernel_Name']).replace('void ', '')[:80]
        a = agg[r['Queue_Id']][name]
        a[0] += 1
        a[1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
n = len(steps)
print(f'{n} steps, span (first marker to next) {sum(spans) / max(n, 1):.1f} us/step')
for q in sorted(agg):
    items = sorted(agg[q].items(), key=lambda kv: -kv[1][1])
    print(f'== queue {q}: {sum(v[1] for _, v in items) / n:.0f} us/step of kernels')
    for name, (c, t) in items[:int(__import__("os").environ.get("QB_TOP", "40"))]:
        print(f'  {t / n:8.1f} us/step {c / n:5.1f}x {t / c:8.1f} us  {name}')
