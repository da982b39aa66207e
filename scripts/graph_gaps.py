"""Device idle time of a bench step from a rocprofv3 kernel trace: the union of all kernel intervals
per step (steps delimited by the SA1 FPS), the whole-GPU idle gaps between them (every queue idle),
and how the kernels spread over hardware queues.  Used to compare the eager step with the
HIP-graph replay (scripts/gpu_r04_graph.sh)."""
import csv, sys
from collections import Counter

def load(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    return rows

for path in sys.argv[1:]:
    rows = load(path)
    idx = [i for i, r in enumerate(rows) if 'fps_kernel<512' in r['Kernel_Name']]
    steps = list(range(max(0, len(idx) - 6), len(idx) - 1))
    tot_span = tot_busy = 0.0
    gaps = Counter()
    qs = Counter()
    big = []
    for k in steps:
        seg = rows[idx[k]:idx[k + 1]]
        t0 = int(seg[0]['Start_Timestamp'])
        t1 = int(rows[idx[k + 1]]['Start_Timestamp'])
        busy, cur_s, cur_e = 0, None, None
        for r in seg:
            s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
            qs[r['Queue_Id']] += 1
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    g = (s - cur_e) / 1e3
                    gaps['<5us' if g < 5 else ('5-20us' if g < 20 else '>=20us')] += 1
                    if g >= 20:
                        big.append((g, r['Kernel_Name'][:60]))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        tot_span += (t1 - t0) / 1e3
        tot_busy += busy / 1e3
    n = len(steps)
    print(f'{path}: {n} steps, span {tot_span / n:.0f} us/step, GPU busy (union) {tot_busy / n:.0f} us, '
          f'all-idle {(tot_span - tot_busy) / n:.0f} us/step')
    print('  all-idle gaps per step:', {k: round(v / n, 1) for k, v in sorted(gaps.items())})
    print('  kernels per queue per step:', {q: round(c / n, 1) for q, c in sorted(qs.items())})
    big.sort(reverse=True)
    for g, name in big[:8]:
        print(f'  gap {g:6.1f} us before {name}')
