# dx_col0 path A/B: k-major W with scalar loads (libpcseg.so) vs W^T rows + transpose launch (libpcseg_tr.so)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_libs_ab.sh s8_ab 3 "- _tr" || exit $?
