# A/B: bench under alternating env settings in ONE call (box-to-box variance is ~10%).
# usage: AB_A="VAR=val" AB_B="VAR=val" bash scripts/gpu_ab.sh
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then E="${AB_A:-X_NONE=1}"; else E="${AB_B:-X_NONE=1}"; fi
    env $E timeout -k 10 120 python bench.py --no-cpu-baseline --no-roofline --steps 30 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/ab_$v.log 2>&1 || exit $?
    echo "$v ($E): $(tail -1 gpurun_out/ab_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
