# final bench line of the default command (high-priority step stream), its rocprof stats, the priority range
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/final4; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python -c "import torch; print('priority_range', torch.cuda.Stream.priority_range(), 'default stream priority', torch.cuda.current_stream().priority)" > $out/prio.log 2>&1; cat $out/prio.log | grep -v amdgpu.ids
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run --output-format csv -- \
   python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/$out/prof_bench.log" 2>&1; rc=$?
cd "$GRAFT_REPO_ROOT"; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $out/bench.log | cut -c1-300
exit $rc
