# One box session: FPS checks, engine tests, a two-build A/B (libpcseg.so vs libpcseg_ref.so),
# then the round-end sequence (full GPU suite, smoke, rocprof stats, default bench line).
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-s}; mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
bash scripts/gpu_fps.sh ${tag}_fps || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$tag/engine.log 2>&1; rc=$?
echo "engine tests rc=$rc"; tail -2 gpurun_out/$tag/engine.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_lib_ab.sh ${tag}_ab 2 || exit $?
bash scripts/gpu_round_end.sh
