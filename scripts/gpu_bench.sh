# Default bench line (+ optional extra args) on one MI355X box (via gpurun).
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-bench}; shift || true
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u bench.py "$@" > $out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $out/bench.log | cut -c1-3000
exit $rc
