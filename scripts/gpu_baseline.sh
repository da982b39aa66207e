# Quick measurement pass: a -k test subset, the default bench (no CPU baseline), and a
# kernel trace of the PointNet++ step.  usage: scripts/gpu_baseline.sh <tag> [pytest -k expr]
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-base}; kexpr=${2:-}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
if [ -n "$kexpr" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "$kexpr" > $out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed" $out/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E " $out/pytest_gpu.log | head; exit $rc; }
fi
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $out/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run --output-format csv -- \
   python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --secondary none \
   > "$GRAFT_REPO_ROOT/$out/prof.log" 2>&1; rc=$?
cd "$GRAFT_REPO_ROOT"; echo "prof rc=$rc"; tail -1 $out/prof.log | cut -c1-200
