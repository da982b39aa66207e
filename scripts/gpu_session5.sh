# host phase split, wgrad block-count A/B, DGCNN edge-inverse placement A/B, then the full GPU suite
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-s5}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for p in loss backward; do
  timeout -k 10 200 python -u scripts/host_phases.py pointnetpp $p > $out/host_$p.log 2>&1 || exit $?
  grep -v amdgpu.ids $out/host_$p.log
done
bash scripts/gpu_libs_ab.sh ${tag}_ab 2 "- _w512 _w256" || exit $?
bash scripts/gpu_libs_ab.sh ${tag}_abd 1 "- _w512 _w256" --model dgcnn || exit $?
for e in backward side; do
  timeout -k 10 300 python -u bench.py --model dgcnn --secondary none --no-cpu-baseline --no-roofline --edge-inverse $e > $out/edge_$e.log 2>&1 || exit $?
  echo "dgcnn edge-inverse $e: $(tail -1 $out/edge_$e.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_enqueue_ms_per_step'])")"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log; exit $rc
