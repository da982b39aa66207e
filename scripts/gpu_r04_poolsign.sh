# single-extreme fused pooling (GEMM epilogue + EdgeConv forward; sign of gamma picks max or min): parity tests, then A/B vs HEAD build
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/poolsign; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py tests/test_gpu_models.py tests/test_gpu_edgeconv.py tests/test_gpu_ops.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
bash scripts/gpu_libs_ab.sh poolsign_ab 2 "- _ref" && \
bash scripts/gpu_libs_ab.sh poolsign_ab_dg 2 "- _ref" --model dgcnn
