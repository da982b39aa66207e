# Round 5: the thin-layer backward -- fused vs split (--bwd-fuse), and the fused kernel's grid /
# occupancy variants (per-mode grid = the product; fbold = round 4's smallest grid over the modes;
# fbw3 = W fragments from LDS at 3 blocks per CU), PointNet++ B=32.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_bench_ab.sh r05_fuse --bwd-fuse "default off" 2 --no-drop-in --others none || exit $?
bash scripts/gpu_libs_ab.sh r05_ab10 3 "- _fbold _fbw3" || exit $?
