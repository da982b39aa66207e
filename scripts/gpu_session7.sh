# full GPU suite, then two PointNet++ / one DGCNN bench lines (no CPU baseline)
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-s7}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
ms() { tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_enqueue_ms_per_step'])"; }
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --secondary none --no-cpu-baseline --no-roofline > $out/pn_$r.log 2>&1 || exit $?
  echo "pointnetpp: $(ms $out/pn_$r.log)"
done
timeout -k 10 300 python -u bench.py --model dgcnn --secondary none --no-cpu-baseline --no-roofline > $out/dg.log 2>&1 || exit $?
echo "dgcnn: $(ms $out/dg.log)"
