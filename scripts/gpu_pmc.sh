# HBM traffic per kernel from PMC counters, one model per pair of passes (FETCH_SIZE, WRITE_SIZE:
# separate runs, kernel-trace only; MI355X_MICROARCH.md "HBM": FETCH_SIZE doubled on gfx950).
# usage: scripts/gpu_pmc.sh <tag> [model ...]   -> gpurun_out/pmc_<tag>/<model>.{txt,json}
set -u
cd "$GRAFT_REPO_ROOT"
tag=${1:-r02}; shift || true
models=${*:-pointnetpp dgcnn}
out="$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag"; mkdir -p "$out"
export TMPDIR=/tmp
for m in $models; do
  ARGS="--model $m --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none"
  for c in FETCH_SIZE WRITE_SIZE; do
    cd /tmp && timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d "$out/${m}_$c" -o run --output-format csv -- \
       python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$out/${m}_$c.log" 2>&1; rc=$?
    echo "$m pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  cd "$GRAFT_REPO_ROOT" && python3 scripts/pmc_traffic.py "$out/${m}_FETCH_SIZE" "$out/${m}_WRITE_SIZE" \
     --json "$out/$m.json" > "$out/$m.txt" 2>&1; echo "$m parse rc=$?"; head -5 "$out/$m.txt"
done
