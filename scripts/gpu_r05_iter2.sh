# Round 5: wgrad split A/B (shorter lane blocks) + the PointNet++ per-queue breakdown / timeline.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_libs_ab.sh r05_ab9 3 "- _wg2048 _wg4096" || exit $?
bash scripts/gpu_r05_iter.sh r05_it5 "" pointnetpp || exit $?
