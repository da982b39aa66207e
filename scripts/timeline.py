"""Print the kernel timeline of one step from a rocprofv3 kernel_trace.csv.

usage: timeline.py trace.csv [step_index_from_end] [marker_substring]
A step starts at each dispatch whose name contains the marker (default: Adam's
multi_tensor_apply is the end of a step, so we split on the first kernel after it).
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
which = int(sys.argv[2]) if len(sys.argv) > 2 else 2
marker = sys.argv[3] if len(sys.argv) > 3 else 'fps_kernel<512'
rows.sort(key=lambda r: int(r['Start_Timestamp']))
starts = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
a = starts[-which]
b = starts[-which + 1] if which > 1 else len(rows)
seg = rows[a:b]
t0 = int(seg[0]['Start_Timestamp'])
busy_end = t0
busy = 0
for r in seg:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    if e > busy_end:
        busy += e - max(s, busy_end)
        busy_end = e
span = int(seg[-1]['End_Timestamp']) - t0
print(f'{len(seg)} kernels, span {span/1e3:.1f} us, union busy {busy/1e3:.1f} us')
for r in seg:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{(s-t0)/1e3:9.1f} {(e-s)/1e3:8.1f} q{r['Queue_Id']} s{r['Stream_Id']} g{r['Grid_Size_X']}x{r['Grid_Size_Y']} {r['Kernel_Name'][:90]}")
