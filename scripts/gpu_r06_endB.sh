# Round-6 evidence, part B: PMC HBM traffic per kernel (FETCH_SIZE / WRITE_SIZE passes) for the four
# workloads, then the default bench line (CPU baseline, roofline, drop-in, other configs).
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r06_end; mkdir -p $out
export TMPDIR=/tmp
bash scripts/gpu_pmc.sh r06 pointnetpp dgcnn pointnetpp_msg pointnext > $out/pmc.log 2>&1; rc=$?; echo "pmc rc=$rc"; tail -4 $out/pmc.log; [ $rc -eq 0 ] || exit $rc
cd "$GRAFT_REPO_ROOT" && timeout -k 10 700 python -u bench.py --detail-out $out/bench_detail.json > $out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $out/bench.log | cut -c1-400
