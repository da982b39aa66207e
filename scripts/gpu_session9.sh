# Morton-seeded coordinate kNN: the kNN tests, then DGCNN with / without the seeds (2 rounds)
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-s9}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "knn or dgcnn or edge" > $out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
ms() { tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_enqueue_ms_per_step'])"; }
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --model dgcnn --secondary none --no-cpu-baseline --no-roofline > $out/dg_seed_$r.log 2>&1 || exit $?
  echo "dgcnn morton seeds: $(ms $out/dg_seed_$r.log)"
  timeout -k 10 300 python -u -c "
import sys; sys.argv = ['bench.py', '--model', 'dgcnn', '--secondary', 'none', '--no-cpu-baseline', '--no-roofline']
sys.path[:0] = ['.', '3d-semantic-segmentation-benchmark_amd']
import pcseg.models as mm
mm._xyz_seeds = lambda xyz, k: None
import bench; bench.main()" > $out/dg_noseed_$r.log 2>&1 || exit $?
  echo "dgcnn no seeds: $(ms $out/dg_noseed_$r.log)"
done
