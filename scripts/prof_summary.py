"""Summarise a rocprofv3 --stats kernel csv: per-step ms of the top kernels."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 7.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f'kernel time total {tot/1e6:.2f} ms = {tot/steps/1e6:.3f} ms/step over {steps:g} steps, {len(rows)} kernels')
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:top]:
    print(f"{float(r['TotalDurationNs'])/steps/1e6:8.3f} ms/step {int(r['Calls'])/steps:6.1f}/step "
          f"{float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:96]}")
