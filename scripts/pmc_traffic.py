"""Per-kernel HBM bytes per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

usage: pmc_traffic.py FETCH_DIR WRITE_DIR [--json OUT]
FETCH_SIZE/WRITE_SIZE are in KB per dispatch.  gfx950 correction (MI355X_MICROARCH.md,
"HBM"): FETCH_SIZE reports half the bytes of wide coalesced reads, so it is doubled;
WRITE_SIZE is taken as is.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    if not files:
        raise SystemExit(f'no counter_collection.csv under {d}')
    per = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get('Counter_Name') != counter:
                continue
            per[r['Kernel_Name']].append(float(r['Counter_Value']) * 1024.0)   # KB -> bytes
    return per


def main():
    fetch = load(sys.argv[1], 'FETCH_SIZE')
    write = load(sys.argv[2], 'WRITE_SIZE')
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        fb = 2.0 * sum(f) / len(f) if f else None
        wb = sum(w) / len(w) if w else None
        out[k] = {'launches_fetch': len(f), 'launches_write': len(w),
                  'fetch_bytes_per_launch_x2': fb, 'write_bytes_per_launch': wb,
                  'hbm_bytes_per_launch': (fb or 0.0) + (wb or 0.0)}
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]['hbm_bytes_per_launch'] *
                       max(kv[1]['launches_fetch'], 1))[:40]:
        print(f"{v['hbm_bytes_per_launch'] / 1e6:10.2f} MB/launch  fetch*2 {(v['fetch_bytes_per_launch_x2'] or 0) / 1e6:9.2f}"
              f"  write {(v['write_bytes_per_launch'] or 0) / 1e6:9.2f}  n={v['launches_fetch']:4d}  {k[:90]}")
    if '--json' in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index('--json') + 1], 'w'), indent=1)


if __name__ == '__main__':
    main()
