# Two-level accumulation A/B: precision diagnostics, per-shape GEMM timing and step time of
# pcseg/libpcseg.so (new) vs pcseg/libpcseg_ref.so (previous build).
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-acc}; out=gpurun_out/$tag; mkdir -p $out
P=$GRAFT_REPO_ROOT/3d-semantic-segmentation-benchmark_amd/pcseg
timeout -k 10 300 python3 -u scripts/diag/stack_grad_error.py > $out/stack_new.log 2>&1 || exit $?
PCS_LIB=$P/libpcseg_ref.so timeout -k 10 300 python3 -u scripts/diag/stack_grad_error.py > $out/stack_ref.log 2>&1 || exit $?
timeout -k 10 300 python3 -u scripts/diag/pointnext_grad_trace.py > $out/trace_new.log 2>&1 || exit $?
for v in new ref; do
  lib=$P/libpcseg.so; [ $v = ref ] && lib=$P/libpcseg_ref.so
  PCS_LIB=$lib timeout -k 10 300 python3 -u scripts/gemm_bench.py > $out/gemm_$v.log 2>&1 || exit $?
done
bash scripts/gpu_lib_ab.sh $tag 3 --model pointnetpp --steps 20 --warmup 5 || exit $?
bash scripts/gpu_lib_ab.sh $tag/dg 2 --model dgcnn --steps 10 --warmup 3 || exit $?
