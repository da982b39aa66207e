"""Split a rocprofv3 kernel trace of `bench.py` into the roofline's probed in-step launches
(the step enqueued behind pcs::spin_kernel, which bench.py times with HIP events) and the
rest, for one kernel: the average in-step duration is what the bench line's
roofline.avg_launch_us reports.

usage: instep_split.py run_kernel_trace.csv 'kernel substring' [window_ms]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
name = sys.argv[2]
win = float(sys.argv[3]) if len(sys.argv) > 3 else 30.0
rows.sort(key=lambda r: int(r['Start_Timestamp']))
spins = [int(r['End_Timestamp']) for r in rows if 'spin_kernel' in r['Kernel_Name']]
inside, outside = [], []
for r in rows:
    if name not in r['Kernel_Name']:
        continue
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    probed = any(0 <= s - t <= win * 1e6 for t in spins)
    (inside if probed else outside).append((e - s) / 1e3)
for label, v in (('in-step (probed, behind the spin)', inside), ('other launches', outside)):
    if v:
        print(f'{label:36s} n={len(v):4d}  avg {sum(v) / len(v):9.2f} us  min {min(v):8.2f}  max {max(v):8.2f}')
