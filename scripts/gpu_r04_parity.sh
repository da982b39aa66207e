# Model three-way parity tests with their clause reports (-s), for profiles/<round>_threeway_report.txt
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-parity}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_models.py -m gpu -k "three_way or golden or harness_a" -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $out/threeway.log 2>&1; rc=$?
grep -E "passed|failed" $out/threeway.log | tail -2; exit $rc
