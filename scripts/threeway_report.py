"""Condense a `pytest -s` log of the three-way model parity tests (scripts/gpu_r04_parity.sh) into
the margins report committed under profiles/: per test, how many tensors passed by which clause,
the worst weight line the test printed, and the five weight gradients closest to the 1e-3 limit
(gpu/truth relative error, with the reference fp32's own error beside it).

usage: python scripts/threeway_report.py gpurun_out/<tag>/threeway.log > profiles/<round>_threeway_report.txt
"""
import re
import sys
from collections import Counter


def main(path: str) -> None:
    lines = open(path, errors='replace').read().splitlines()
    sections, cur = [], None
    for ln in lines:
        m = re.match(r'^-- three-way clauses (.*)$', ln)
        if m:
            cur = {'tag': m.group(1), 'rows': [], 'worst': ''}
            sections.append(cur)
            continue
        if cur is None:
            continue
        m = re.match(r'^(\S+)\s+gpu/truth\s+(\S+)\s+cpu32/truth\s+(\S+)\s+(\S+)$', ln)
        if m:
            cur['rows'].append((m.group(1), float(m.group(2)), float(m.group(3)), m.group(4)))
        elif ln.startswith('worst weight'):
            cur['worst'] = ln
            cur = None
    print('three-way parity margins (GPU fp32 vs CPU fp32 reference algorithm vs CPU fp64 truth, same indices)')
    print(f'source: {path}')
    print('clauses (tests/fp64_check.py): rel = within 1e-3 of the fp64 truth; ref-noise = within 10x the')
    print('reference fp32 error, and for every WEIGHT (conv / linear / BN gamma) within 3x; floor = module floor')
    print('(never for weights).  Weight rows: the five closest to the 1e-3 limit, and gpu/cpu32 = the ratio the')
    print('3x clause bounds.')
    for s in sections:
        print(f"\n== {s['tag']}")
        print('   clauses: ' + ', '.join(f'{k} {v}' for k, v in sorted(Counter(r[0] for r in s['rows']).items())))
        print('   ' + s['worst'])
        w = [r for r in s['rows'] if r[3].endswith('weight') and 'running' not in r[3]]
        w.sort(key=lambda r: -r[1])
        for cl, g, c, name in w[:5]:
            print(f'   {name:46s} gpu/truth {g:.2e} ({g / 1e-3:4.2f} of 1e-3)  cpu32/truth {c:.2e}'
                  f'  gpu/cpu32 {g / c if c else 0.0:4.2f} (limit 3)  [{cl}]')
    traj = [ln for ln in lines if re.match(r'^(tests/\S+ )?step \d+: fp64', ln)]
    if traj:
        print('\n== harness-A loop (torch.optim.Adam, teacher-forced weights): loss per step')
        for ln in traj:
            print('   ' + re.sub(r'^tests/\S+ ', '', ln))


if __name__ == '__main__':
    main(sys.argv[1])
