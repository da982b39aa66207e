# DGCNN step: the round-5 head buffer (EdgeConv second output) vs the round-4 copies, R rounds.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r05_headbuf; mkdir -p $out; R=${1:-3}
A="--model dgcnn --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none"
for r in $(seq $R); do
  timeout -k 10 300 python -u bench.py $A > $out/new_$r.log 2>&1 || exit $?
  echo "new round $r: $(tail -1 $out/new_$r.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
  timeout -k 10 300 python -u scripts/bench_old_head.py $A > $out/old_$r.log 2>&1 || exit $?
  echo "old round $r: $(tail -1 $out/old_$r.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
