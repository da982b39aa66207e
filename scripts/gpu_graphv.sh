# graph variants vs eager, default bench line, host profile
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-gv}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
run() { # name, args...
  local nm=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --secondary none "$@" > $out/bench_$nm.log 2>&1; local rc=$?
  [ $rc -eq 0 ] || { echo "$nm rc=$rc"; tail -3 $out/bench_$nm.log; return $rc; }
  tail -1 $out/bench_$nm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$nm', d['ms_per_step'], d['host_enqueue_ms_per_step'])"
}
run eager && run graph --graph && run graph_geo_eager --graph --graph-geometry eager || exit 1
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $out/bench_default.log 2>&1; rc=$?; echo "bench default rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/bench_default.log; exit $rc; }
tail -1 $out/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['ms_per_step'], r['kernel'], r['frac'], [ (t['kernel'][:40], t['in_step_ms']) for t in r['top_kernels']]); print(d['secondary']['ms_per_step'], d['secondary']['step_roofline'])"
timeout -k 10 300 python -u scripts/host_profile.py > $out/host_profile.log 2>&1; echo "hostprof rc=$?"
