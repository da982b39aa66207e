"""Split one kernel's rocprofv3 kernel-trace durations into the in-step launches and the
trailing back-to-back replays bench.py issues for its roofline (pcs_probe_replay).

usage: replay_split.py kernel_trace.csv KERNEL_PREFIX N_REPLAYS
"""
import csv
import sys

path, name, nrep = sys.argv[1], sys.argv[2], int(sys.argv[3])
rows = [r for r in csv.DictReader(open(path)) if r['Kernel_Name'].startswith(name)]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows]
rep, ins = d[-nrep:], d[:-nrep]
print(f'{name}: {len(d)} dispatches')
print(f'  replayed back to back (last {len(rep)}): avg {sum(rep) / len(rep):.2f} us   <- compare bench.py roofline.avg_launch_us')
if ins:
    print(f'  in-step ({len(ins)}, concurrent with the side-stream wgrad/geometry): avg {sum(ins) / len(ins):.2f} us')
