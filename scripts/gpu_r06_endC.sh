# Round-6 evidence, parts B + the bounds-checked suite in one call: PMC passes and the default bench
# line (gpu_r06_endB.sh), then the whole GPU suite against libpcseg_debug.so (gpu_debug_suite.sh).
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r06_endB.sh || exit $?
bash scripts/gpu_debug_suite.sh r06_debug
