# Round-4 check: graph / optimizer / model GPU tests, then two default bench lines (no CPU baseline)
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/check; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_graphs.py tests/test_gpu_optim.py tests/test_gpu_models.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench$i.json 2>$out/bench$i.err || { tail $out/bench$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['secondary']
print(d['ms_per_step'], d['drop_in']['ms_per_step'], s['ms_per_step'], s['drop_in']['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])" $out/bench$i.json
done
