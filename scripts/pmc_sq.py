"""Per-kernel issue / stall shares from one rocprofv3 --pmc run of SQ counters (gpu_pmc_sq.sh).
SQ_WAVE_CYCLES, SQ_ACTIVE_INST_*, SQ_WAIT_* count quad-cycles summed over waves:
  valu = ACTIVE_INST_VALU / WAVE_CYCLES   (share of a wave's life issuing vector ALU)
  any  = ACTIVE_INST_ANY / WAVE_CYCLES,  wait = WAIT_ANY / WAVE_CYCLES (parked: s_waitcnt, barrier)
  stall = WAIT_INST_ANY / WAVE_CYCLES (issue stalls),  valu_simd = ACTIVE_INST_VALU * 4 /
  (GRBM_GUI_ACTIVE * 1024 SIMDs): the vector ALUs' busy share over the kernel (GUI_ACTIVE in cycles)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    n = name.split('(')[0].replace('void ', '').replace('ctws::', '')
    return n[:40]


def main(d):
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for path in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if 'ctws' not in r['Kernel_Name']:
                    continue
                k = short(r['Kernel_Name'])
                per[k][r['Counter_Name']] += float(r['Counter_Value'])
                disp[k].add(r['Dispatch_Id'])
    rows = []
    for k, v in per.items():
        wc = max(v.get('SQ_WAVE_CYCLES', 0.0), 1.0)
        gui = max(v.get('GRBM_GUI_ACTIVE', 0.0), 1.0)
        rows.append((gui, k, len(disp[k]), v.get('SQ_ACTIVE_INST_VALU', 0) / wc, v.get('SQ_ACTIVE_INST_ANY', 0) / wc,
                     v.get('SQ_WAIT_ANY', 0) / wc, v.get('SQ_WAIT_INST_ANY', 0) / wc,
                     v.get('SQ_ACTIVE_INST_VALU', 0) * 4 / (gui * 1024), v.get('SQ_INSTS_VALU', 0),
                     v.get('SQ_INSTS_LDS', 0), v.get('SQ_WAVES', 0)))
    rows.sort(reverse=True)
    print(f"{'kernel':40s} {'n':>3s} {'gui_Mcyc':>9s} {'valu':>6s} {'any':>6s} {'wait':>6s} {'stall':>6s} "
          f"{'valu_simd':>9s} {'insts_valu':>11s} {'insts_lds':>10s} {'waves':>9s}")
    for gui, k, n, va, an, wa, st, vs, iv, il, wv in rows:
        print(f"{k:40s} {n:3d} {gui / 1e6:9.3f} {va:6.3f} {an:6.3f} {wa:6.3f} {st:6.3f} {vs:9.3f} {iv:11.3e} "
              f"{il:10.3e} {wv:9.0f}")


if __name__ == '__main__':
    main(sys.argv[1])
