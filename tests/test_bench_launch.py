"""bench.py's multi-rank launch path on the CPU (no GPU is touched): `--gpus N` without an
external launcher spawns N rank processes with torchrun's env (RANK, LOCAL_RANK,
WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), each joins one process group of size N;
a launcher whose WORLD_SIZE disagrees with --gpus is refused; the CPU-baseline worker
emits the cpu_baseline record."""
import json
import os
import subprocess
import sys

from conftest import REPO

BENCH = os.path.join(REPO, 'bench.py')


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')}
    env.update(HIP_VISIBLE_DEVICES='', CUDA_VISIBLE_DEVICES='', **kw)
    return env


def test_gpus_n_spawns_n_ranks_with_torchrun_env():
    out = subprocess.run([sys.executable, BENCH, '--gpus', '3', '--check-launch'], env=_env(), capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    recs = [json.loads(l) for l in out.stdout.splitlines() if l.startswith('{')]
    assert sorted(r['rank'] for r in recs) == [0, 1, 2]
    assert all(r['world'] == 3 and r['local_rank'] == r['rank'] for r in recs)
    assert len({r['master'] for r in recs}) == 1 and recs[0]['master'].startswith('127.0.0.1:')


def test_external_launcher_world_must_match_gpus():
    out = subprocess.run([sys.executable, BENCH, '--gpus', '1', '--check-launch'],
                         env=_env(WORLD_SIZE='2', RANK='0', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1',
                                  MASTER_PORT='29999'), capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and 'WORLD_SIZE=2' in (out.stderr + out.stdout)


def test_cpu_baseline_worker_record():
    out = subprocess.run([sys.executable, BENCH, '--cpu-baseline-worker', '--model', 'pointnetpp', '--npoints',
                          '512', '--cpu-batch', '1', '--cpu-steps', '2', '--cpu-threads', '2', '--cpu-budget', '0.1'],
                         env=_env(), capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec['value'] > 0 and rec['cores'] == 2 and rec['kind'] == 'port' and 'median' in rec['sample']
