# thin wgrad sweep: register stages x 32-wide tiles (engine tests at the most aggressive setting first)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
PCS_WGRAD_STAGES=4 PCS_WGRAD_THIN32=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -q -x -k wgrad -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_engine.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_engine.log; [ $rc -eq 0 ] || exit $rc
for cfg in "2 0" "4 0" "2 1" "4 1"; do
  set -- $cfg
  PCS_WGRAD_STAGES=$1 PCS_WGRAD_THIN32=$2 GEMM_SHAPES=sa1,sa2,dg.e2 GEMM_REPS=20 timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/wg_$1_$2.log 2>&1 || exit $?
  echo "== stages $1 thin32 $2"; grep -v amdgpu gpurun_out/wg_$1_$2.log | awk -F'wgrad' '{print substr($1,1,40) "wgrad" $2}'
done
