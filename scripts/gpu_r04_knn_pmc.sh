# SQ counters of the DGCNN kNN (scripts/knn_seed_ab.py: unseeded + seeded graphs), one pass per group
set -u
cd "$GRAFT_REPO_ROOT"; out="$GRAFT_REPO_ROOT/gpurun_out/knn_pmc"; mkdir -p "$out"
export TMPDIR=/tmp
g1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
g2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
g3="SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE"
i=0
for g in "$g1" "$g2" "$g3"; do
  i=$((i+1))
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $g --kernel-trace -d "$out/g$i" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/scripts/knn_seed_ab.py" > "$out/g$i.log" 2>&1; rc=$?
  echo "group $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/g$i.log"; exit $rc; }
done
cd "$GRAFT_REPO_ROOT"
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter(); dur = collections.defaultdict(float)
for g in (1, 2, 3):
    for f in glob.glob(f'{out}/g{g}/**/*counter_collection.csv', recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0].replace('void ', '')
            if 'knn' not in k: continue
            acc[k][r['Counter_Name']] += float(r['Counter_Value'])
            key = (r['Dispatch_Id'], g)
            if key not in seen and g == 1:
                seen.add(key); n[k] += 1; dur[k] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
for k, c in acc.items():
    print(k, 'launches', n[k], 'avg us', round(dur[k] / max(n[k], 1), 1))
    wc = c['SQ_WAVE_CYCLES'] or 1
    print('  per wave-cycle: wait_any %.2f wait_inst %.2f active_inst %.2f | active valu %.2f lds %.2f sca %.2f misc %.2f' % (
        c['SQ_WAIT_ANY'] / wc, c['SQ_WAIT_INST_ANY'] / wc, c['SQ_ACTIVE_INST_ANY'] / wc, c['SQ_ACTIVE_INST_VALU'] / wc,
        c['SQ_ACTIVE_INST_LDS'] / wc, c['SQ_ACTIVE_INST_SCA'] / wc, c['SQ_ACTIVE_INST_MISC'] / wc))
    print('  insts: valu %d mfma %d lds %d salu %d smem %d vmem_rd %d vmem_wr %d' % tuple(c[x] for x in (
        'SQ_INSTS_VALU', 'SQ_INSTS_MFMA', 'SQ_INSTS_LDS', 'SQ_INSTS_SALU', 'SQ_INSTS_SMEM', 'SQ_INSTS_VMEM_RD', 'SQ_INSTS_VMEM_WR')))
    print('  mfma busy / (gui * 1024): %.3f  lds bank conflict / lds active: %.3f  waves %d' % (
        c['SQ_VALU_MFMA_BUSY_CYCLES'] / ((c['GRBM_GUI_ACTIVE'] or 1) * 1024), c['SQ_LDS_BANK_CONFLICT'] / (c['SQ_ACTIVE_INST_LDS'] or 1), c['SQ_WAVES']))
PY
