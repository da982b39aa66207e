# rocprofv3 kernel stats of scripts/stack_bwd_bench.py per shape and policy
set -u
cd "$GRAFT_REPO_ROOT"; tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for sh in "$@"; do for pol in default all; do
  cd /tmp && STACK_SHAPES=$sh timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/${sh}_$pol" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/scripts/stack_bwd_bench.py" $pol > "$GRAFT_REPO_ROOT/$out/${sh}_$pol.log" 2>&1 || exit $?
  cd "$GRAFT_REPO_ROOT"; tail -1 $out/${sh}_$pol.log
  f=$(find $out/${sh}_$pol -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:14]: print(f\"{float(r['AverageNs'])/1e3:9.1f} us x{int(r['Calls']):4d}  {r['Name'][:110]}\")
"
done; done
