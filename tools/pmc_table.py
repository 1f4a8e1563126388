"""Summarise gpurun_out/pmc_*/ counter CSVs per kernel (mean per dispatch)."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocprof_summary import short_name  # noqa: E402

root = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out'
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, 'pmc_*', '*counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        k = short_name(r['Kernel_Name'])
        if 'spef' not in r['Kernel_Name'] and 'irb' not in k:
            continue
        vals[k][r['Counter_Name']].append(float(r['Counter_Value']))
mean = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in vals.items()}
cols = ['SQ_WAVES', 'SQ_WAVE_CYCLES', 'SQ_BUSY_CYCLES', 'SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY',
        'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_LDS', 'SQ_ACTIVE_INST_VMEM', 'SQ_INSTS_VALU', 'SQ_INSTS_LDS',
        'SQ_INSTS_MFMA', 'SQ_INSTS_VMEM_RD', 'SQ_INSTS_SALU', 'SQ_LDS_BANK_CONFLICT', 'SQ_LDS_IDX_ACTIVE',
        'SQ_VALU_MFMA_BUSY_CYCLES', 'GRBM_GUI_ACTIVE', 'FETCH_SIZE', 'WRITE_SIZE']
for k, d in sorted(mean.items()):
    wc = d.get('SQ_WAVE_CYCLES', 1)
    print(f'== {k}')
    print('   ' + '  '.join(f'{c.replace("SQ_", "")}={d[c]:.3g}' for c in cols if c in d))
    if 'SQ_WAVE_CYCLES' in d:
        print(f'   wait_any {d.get("SQ_WAIT_ANY", 0) / wc:.2f}  wait_inst {d.get("SQ_WAIT_INST_ANY", 0) / wc:.2f}  '
              f'active {d.get("SQ_ACTIVE_INST_ANY", 0) / wc:.2f} (valu {d.get("SQ_ACTIVE_INST_VALU", 0) / wc:.2f} '
              f'lds {d.get("SQ_ACTIVE_INST_LDS", 0) / wc:.2f} vmem {d.get("SQ_ACTIVE_INST_VMEM", 0) / wc:.2f})')
    if 'SQ_INSTS_MFMA' in d and d.get('SQ_WAVES'):
        w = d['SQ_WAVES']
        print(f'   per wave: valu {d["SQ_INSTS_VALU"] / w:.0f} lds {d["SQ_INSTS_LDS"] / w:.0f} mfma {d["SQ_INSTS_MFMA"] / w:.0f} '
              f'vmem_rd {d.get("SQ_INSTS_VMEM_RD", 0) / w:.0f} salu {d.get("SQ_INSTS_SALU", 0) / w:.0f}; '
              f'bank_conflict/idx_active {d["SQ_LDS_BANK_CONFLICT"] / max(1, d["SQ_LDS_IDX_ACTIVE"]):.2f}')
