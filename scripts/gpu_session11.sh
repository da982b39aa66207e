# full GPU suite, then PointNet++ with / without the FP1 skip-column dX trim (2 rounds)
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-s11}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
ms() { tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_enqueue_ms_per_step'])"; }
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --secondary none --no-cpu-baseline --no-roofline > $out/pn_fpdx_$r.log 2>&1 || exit $?
  echo "pointnetpp FP1 dx trim: $(ms $out/pn_fpdx_$r.log)"
  timeout -k 10 300 python -u -c "
import sys; sys.argv = ['bench.py', '--secondary', 'none', '--no-cpu-baseline', '--no-roofline']
sys.path[:0] = ['.', '3d-semantic-segmentation-benchmark_amd']
import pcseg.common as c
orig = c.UnitPointNet.forward_rows
c.UnitPointNet.forward_rows = lambda self, x, kin=None, dropout=None, dx_from=0: orig(self, x, kin, dropout, 0)
import bench; bench.main()" > $out/pn_nofpdx_$r.log 2>&1 || exit $?
  echo "pointnetpp no FP1 trim: $(ms $out/pn_nofpdx_$r.log)"
done
