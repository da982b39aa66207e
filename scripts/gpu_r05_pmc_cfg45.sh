# Round 5: PMC HBM traffic per kernel for BASELINE configs 4 / 5's per-GPU halves (MSG B=32, PointNeXt-B B=16 x 24576).
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_pmc.sh r05 pointnetpp_msg pointnext
