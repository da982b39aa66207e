# graph-mode bench under HIP graph-queue settings (DEBUG_HIP_FORCE_GRAPH_QUEUES)
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-gq}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_edgeconv.py tests/test_gpu_models.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "edgeconv or dgcnn_color_vs" > $out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for q in 1 2 4 8; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --graph --secondary none > $out/bench_q$q.log 2>&1; rc=$?
  echo "q=$q rc=$rc"; [ $rc -eq 0 ] || { tail -3 $out/bench_q$q.log; exit $rc; }
  tail -1 $out/bench_q$q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('q=$q', d['ms_per_step'], d['host_enqueue_ms_per_step'])"
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --graph --secondary none > $out/bench_pc0.log 2>&1; rc=$?
tail -1 $out/bench_pc0.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pc=0', d['ms_per_step'], d['host_enqueue_ms_per_step'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --graph --no-prefetch --secondary none > $out/bench_nopf.log 2>&1; rc=$?
tail -1 $out/bench_nopf.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('nopf', d['ms_per_step'], d['host_enqueue_ms_per_step'])"
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$out/prof" -o run --output-format csv -- \
   python3 "$GRAFT_REPO_ROOT/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --secondary none --graph \
   > "$GRAFT_REPO_ROOT/$out/prof.log" 2>&1; echo "prof rc=$?"
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $out/bench_default.log 2>&1; rc=$?; echo "bench default rc=$rc"
tail -1 $out/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['ms_per_step'], r['kernel'], r['frac'], [ (t['kernel'][:40], t['in_step_ms']) for t in r['top_kernels']]); print(d['secondary']['ms_per_step'], d['secondary']['step_roofline'])"
