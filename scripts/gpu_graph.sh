# HIP-graph replay cost probe + the PointNet++ step in graph mode + host profile of the eager step.
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-graph}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for pc in unset 1 0; do
  if [ $pc = unset ]; then timeout -k 10 120 python -u scripts/graph_probe.py 240 > $out/probe_$pc.log 2>&1 || exit $?
  else DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 120 python -u scripts/graph_probe.py 240 > $out/probe_$pc.log 2>&1 || exit $?; fi
  cat $out/probe_$pc.log | grep kernels
done
for pc in unset 1; do
  if [ $pc = unset ]; then timeout -k 10 300 python -u bench.py --graph --no-cpu-baseline --secondary none --no-roofline > $out/bench_graph_$pc.log 2>&1 || exit $?
  else DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 300 python -u bench.py --graph --no-cpu-baseline --secondary none --no-roofline > $out/bench_graph_$pc.log 2>&1 || exit $?; fi
  tail -1 $out/bench_graph_$pc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('graph pc=$pc', d['ms_per_step'], d['host_enqueue_ms_per_step'])"
done
timeout -k 10 300 python -u scripts/host_profile.py > $out/host_profile.log 2>&1 || exit $?
head -60 $out/host_profile.log
