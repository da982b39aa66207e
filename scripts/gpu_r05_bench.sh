# Round 5: the named GPU tests, then the default bench line without the CPU baseline (PointNet++ value,
# DGCNN secondary, MSG + PointNeXt-B other_configs, drop-in lines), then the drop-in host profile.
# usage: scripts/gpu_r05_bench.sh <tag> "<pytest selection>"
set -u
cd "$GRAFT_REPO_ROOT"; tag=$1; sel=$2
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
if [ -n "$sel" ]; then
  timeout -k 10 600 python -u -m pytest $sel -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 python -u bench.py --no-cpu-baseline > $out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $out/bench.log; exit $rc; }
tail -1 $out/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
def show(n, r):
    di = r.get('drop_in') or {}
    print(f\"{n}: {r['ms_per_step']} ms host {r.get('host_enqueue_ms_per_step')} | drop-in {di.get('ms_per_step')} ms host {di.get('host_enqueue_ms_per_step')}\")
show('pointnetpp', d); show('dgcnn', d['secondary'])
for k, v in (d.get('other_configs') or {}).items(): show(k, v)"
timeout -k 10 300 python -u scripts/host_profile_dropin.py pointnetpp > $out/host_dropin.txt 2>&1; rc=$?
echo "host profile rc=$rc"; head -3 $out/host_dropin.txt
exit $rc
