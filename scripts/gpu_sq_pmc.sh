# SQ / TCP counters of one command's kernels, one rocprofv3 --pmc pass per counter group.
# usage: scripts/gpu_sq_pmc.sh <tag> <python script>   -> gpurun_out/sq_<tag>/<group>/
set -u
cd "$GRAFT_REPO_ROOT"
tag=$1; script=$2
out="$GRAFT_REPO_ROOT/gpurun_out/sq_$tag"; mkdir -p "$out"
export TMPDIR=/tmp
g1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
g2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
i=0
for g in "$g1" "$g2"; do
  i=$((i+1))
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $g --kernel-trace -d "$out/g$i" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/$script" > "$out/g$i.log" 2>&1; rc=$?
  echo "group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
