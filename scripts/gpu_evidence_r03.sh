# Round-3 evidence on the final code: PMC HBM traffic (separate FETCH / WRITE passes), the rocprofv3
# kernel-trace stats of the exact default bench command, then the default bench line itself
# (whose roofline reads the PMC table just written into profiles/ of this tree).
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/ev3; mkdir -p $out
export TMPDIR=/tmp
bash scripts/gpu_libs_ab.sh ev3_ab 1 "- _km" || exit $?
bash scripts/gpu_pmc.sh r03 pointnetpp dgcnn || exit $?
for m in pointnetpp dgcnn; do cp gpurun_out/pmc_r03/$m.json profiles/r03_pmc_${m}_b32_n4096.json; done
# the default command's GPU work (the CPU-baseline subprocess runs no GPU kernel: left out here)
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run --output-format csv -- \
   python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/$out/prof_bench.log" 2>&1; rc=$?
cd "$GRAFT_REPO_ROOT"; echo "prof rc=$rc"; tail -1 $out/prof_bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $out/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc

