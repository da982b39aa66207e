# row-GEMM tile sweep over the mid/large engine shapes (forced tile for every launch)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for t in default 128,128 64,128 128,64 64,64; do
  if [ $t = default ]; then unset PCS_GEMM_TILE; else export PCS_GEMM_TILE=$t; fi
  GEMM_SHAPES=sa2,sa3,sa4,fp GEMM_REPS=20 timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/tile_$t.log 2>&1 || exit $?
  echo "== tile $t"; grep -v amdgpu gpurun_out/tile_$t.log | awk -F'|' '{print substr($1,1,30) substr($1,40,20) "|" substr($2,1,24) "|" substr($3,1,22)}'
done
