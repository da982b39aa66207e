# Round-4 experiment runner: targeted GPU tests + microbenchmarks (args: tag, pytest -k expr, then commands)
set -u
cd "$GRAFT_REPO_ROOT"; tag=$1; kexpr=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
if [ -n "$kexpr" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -k "$kexpr" -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
  tail -2 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $out/pytest.log | head -20; exit $rc; }
fi
i=0
for c in "$@"; do
  i=$((i+1)); echo "== $c"
  timeout -k 10 300 bash -c "$c" > $out/cmd$i.log 2>&1; rc=$?; tail -15 $out/cmd$i.log
  [ $rc -eq 0 ] || exit $rc
done
