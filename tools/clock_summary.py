#!/usr/bin/env python3
"""Per-kernel effective clock from a rocprofv3 pass with --kernel-trace --pmc GRBM_GUI_ACTIVE
(tools/clock_probe.sh): clock = GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration (MI355X_MICROARCH.md,
DVFS give-back). Usage: python tools/clock_summary.py gpurun_out/clk_ema [gpurun_out/clk_svf ...]"""
import csv
import os
import sys
from collections import defaultdict


def main():
    for d in sys.argv[1:]:
        grbm, wc = {}, {}
        for r in csv.DictReader(open(os.path.join(d, 'run_counter_collection.csv'))):
            key = r['Dispatch_Id']
            if r['Counter_Name'] == 'GRBM_GUI_ACTIVE':
                grbm[key] = grbm.get(key, 0.0) + float(r['Counter_Value'])
            elif r['Counter_Name'] == 'SQ_WAVE_CYCLES':
                wc[key] = wc.get(key, 0.0) + float(r['Counter_Value'])
        per = defaultdict(list)
        for r in csv.DictReader(open(os.path.join(d, 'run_kernel_trace.csv'))):
            key = r['Dispatch_Id']
            if key not in grbm:
                continue
            dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e9
            grid = int(r['Grid_Size_X']) * int(r['Grid_Size_Y']) * int(r['Grid_Size_Z'])
            name = r['Kernel_Name'].split('(')[0].replace('void ', '')
            if dur > 1e-3:
                per[(name, grid)].append((dur * 1e3, grbm[key] / 8 / dur / 1e9, wc.get(key, 0.0)))
        print('==', d)
        for (name, grid), v in sorted(per.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
            ms = sorted(x[0] for x in v)
            ghz = sorted(x[1] for x in v)
            print('  %-34s grid %9d n %2d  median %.3f ms  clock median %.3f GHz (min %.3f max %.3f)  wave_cycles %.3e'
                  % (name[:34], grid, len(v), ms[len(ms) // 2], ghz[len(ghz) // 2], ghz[0], ghz[-1],
                     sorted(x[2] for x in v)[len(v) // 2]))


if __name__ == '__main__':
    main()
