# Round 5: EdgeConv tests + a PointNet++ / DGCNN bench line with the live roofline (no CPU baseline).
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r05_roof; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_edgeconv.py -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-drop-in --others none > $out/bench.log 2>&1 || exit $?
tail -1 $out/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k in ('roofline',):
    r=d[k]; print(d['ms_per_step'], r['kernel'], r['frac'], r.get('with_concurrent_side_mfma'))
s=d['secondary']; r=s['roofline']; print(s['ms_per_step'], r['kernel'], r['frac'], r.get('with_concurrent_side_mfma'))"
