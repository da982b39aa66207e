# Graph-mode step time under the HIP runtime's graph-execution settings (one bench process each).
# usage: scripts/gpu_graph_env.sh <tag> [model]
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-genv}; m=${2:-pointnetpp}; out=gpurun_out/$tag; mkdir -p $out
run() {   # name, env assignments...
  local nm=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --graph --model $m --secondary none --no-cpu-baseline --no-roofline > $out/${m}_$nm.log 2>&1 || return $?
  echo "$m $nm: $(tail -1 $out/${m}_$nm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_enqueue_ms_per_step'])")"
}
echo "eager: $(timeout -k 10 300 python -u bench.py --model $m --secondary none --no-cpu-baseline --no-roofline 2>/dev/null | tail -1 | cut -c1-160)" && \
run default HIP_NOTHING=1 && \
run pktcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 && \
run pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && \
run queues1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1 && \
run queues4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 && \
run batch64 DEBUG_HIP_GRAPH_BATCH_SIZE=64
