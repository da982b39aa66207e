"""bench.py's final stdout line stays a compact JSON object the driver can parse (round 5's
32 KB line overflowed the driver's ~10 KB stdout tail): built from a canned full record (the
round-5 default run's, profiles/r05_bench_default.json), it is under 4096 bytes, is the last
stdout line, carries the contract's keys plus the compact roofline and CPU baseline of both
halves of the metric, and names the detail file that holds the rest."""
import json
import os
import sys

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402

CANNED = os.path.join(REPO, 'profiles', 'r05_bench_default.json')


def _canned():
    full = json.load(open(CANNED))
    for r in [full, full['secondary']] + list(full['other_configs'].values()):
        r['config'].setdefault('rccl_world', 1)
        roof = r['roofline']
        roof['committed_profile_avg_us'] = roof.pop('rocprof_avg_launch_us', None)
    return full


def test_line_is_compact_last_and_complete(tmp_path, capsys):
    full = _canned()
    det = tmp_path / 'bench_detail.json'
    line = bench.emit_line(full, str(det))
    out = capsys.readouterr().out
    assert out.rstrip('\n').splitlines()[-1] == line
    assert len(line.encode()) <= 4096, len(line)
    rec = json.loads(line)
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better',
              'scaling', 'vs_baseline', 'dtype', 'data', 'config'):
        assert k in rec, k
    assert rec['metric'] == bench.METRIC and rec['value'] == full['value']
    assert 'workload' in rec['config']
    for blk in (rec, rec['secondary']):
        roof = blk['roofline']
        for k in ('kernel', 'bound', 'achieved', 'peak', 'unit', 'frac', 'traffic', 'avg_launch_us'):
            assert k in roof, k
        assert abs(roof['frac'] - roof['achieved'] / roof['peak']) < 1e-3
        assert blk['cpu_baseline']['value'] > 0 and blk['cpu_baseline']['cores'] > 0
    assert rec['secondary']['ms_per_step'] == full['secondary']['ms_per_step']
    assert set(rec['other_configs']) == {'pointnetpp_msg', 'pointnext'}
    for v in rec['other_configs'].values():
        assert set(v) == {'value', 'ms_per_step', 'frac', 'drop_in_ms'}
    # the detail file holds the full record
    assert json.load(open(det))['roofline']['top_kernels'] == full['roofline']['top_kernels']
    assert rec['detail'] == os.path.relpath(str(det), REPO)


def test_line_trims_when_strings_grow():
    full = _canned()
    full['cpu_baseline']['sample'] = 'x' * 5000
    full['secondary']['config']['workload'] = 'y' * 1500
    line = json.dumps(bench.compact_line(full, None), separators=(',', ':'))
    assert len(line.encode()) <= 4096
    json.loads(line)
