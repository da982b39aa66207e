"""Per-dispatch SQ counter summary of a rocprofv3 --pmc run (scripts/gpu_gemm_pmc.sh).

usage: sq_summary.py counter_collection.csv [name_filter]
Columns: duration, MFMA busy cycles per SIMD-cycle (GRBM_GUI_ACTIVE x 1024 SIMDs),
and the wave-cycle split WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY (fractions of
SQ_WAVE_CYCLES), LDS bank-conflict cycles.
"""
import collections
import csv
import re
import sys

path = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else 'pcs::'
disp = collections.OrderedDict()
for r in csv.DictReader(open(path)):
    if filt not in r['Kernel_Name']:
        continue
    d = disp.setdefault(r['Dispatch_Id'], {'name': r['Kernel_Name'], 'grid': r['Grid_Size'],
                                            'dur': (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3,
                                            'lds': r['LDS_Block_Size'], 'vgpr': r['VGPR_Count'],
                                            'agpr': r['Accum_VGPR_Count']})
    d[r['Counter_Name']] = float(r['Counter_Value'])
for k, d in disp.items():
    name = re.sub(r'\(.*', '', d['name']).replace('pcs::', '')[:48]
    wave = d.get('SQ_WAVE_CYCLES', 0) or 1
    gui = d.get('GRBM_GUI_ACTIVE', 0) or 1
    mf = d.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (gui * 1024)
    print(f"{name:48s} g{int(d['grid']) // 256:7d} {d['dur']:8.1f}us mfma {mf:5.2f} "
          f"wait {d.get('SQ_WAIT_ANY', 0) / wave:4.2f} inst {d.get('SQ_WAIT_INST_ANY', 0) / wave:4.2f} "
          f"act {d.get('SQ_ACTIVE_INST_ANY', 0) / wave:4.2f} ldsw {d.get('SQ_WAIT_INST_LDS', 0) / wave:4.2f} "
          f"bankc {d.get('SQ_LDS_BANK_CONFLICT', 0) / 1e6:7.2f}M busy {d.get('SQ_BUSY_CYCLES', 0) / gui:5.2f} "
          f"v{d['vgpr']} a{d['agpr']}")
