# SQ counters of the stack-backward bench (one shape, one policy): two rocprofv3 --pmc passes.
# usage: scripts/gpu_r04_sqpmc.sh <tag> <shape> <policy>
set -u
cd "$GRAFT_REPO_ROOT"; tag=$1; sh=$2; pol=$3
out="$GRAFT_REPO_ROOT/gpurun_out/sq_$tag"; mkdir -p "$out"
export TMPDIR=/tmp
g1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
g2="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
i=0
for g in "$g1" "$g2"; do
  i=$((i+1))
  cd /tmp && STACK_SHAPES=$sh timeout -s KILL 120 rocprofv3 --pmc $g --kernel-trace -d "$out/g$i" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/scripts/stack_bwd_bench.py" $pol > "$out/g$i.log" 2>&1; rc=$?
  echo "group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd "$GRAFT_REPO_ROOT"
python3 - "$out" <<'PY'
import csv, glob, re, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob(out + '/g*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        n = re.sub(r'\(.*', '', r['Kernel_Name']).replace('void ', '').replace('pcs::', '')[:60]
        agg[n][r['Counter_Name']] += float(r['Counter_Value'])
for n, d in sorted(agg.items(), key=lambda kv: -kv[1].get('SQ_WAVE_CYCLES', 0))[:12]:
    w = d.get('SQ_WAVE_CYCLES', 0) or 1
    gui = d.get('GRBM_GUI_ACTIVE', 0) or 1
    print(f"{n:60s} waitany {d.get('SQ_WAIT_ANY',0)/w:5.2f} waitinst {d.get('SQ_WAIT_INST_ANY',0)/w:5.2f} "
          f"active {d.get('SQ_ACTIVE_INST_ANY',0)/w:5.2f} mfma_busy/simd {d.get('SQ_VALU_MFMA_BUSY_CYCLES',0)/(gui*1024):5.2f} "
          f"valu {d.get('SQ_INSTS_VALU',0):.3g} lds {d.get('SQ_INSTS_LDS',0):.3g} mfma {d.get('SQ_INSTS_MFMA',0):.3g} "
          f"waitlds {d.get('SQ_WAIT_INST_LDS',0)/w:5.2f} bankconf {d.get('SQ_LDS_BANK_CONFLICT',0):.3g}")
PY
