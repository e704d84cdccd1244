#!/usr/bin/env python3
"""Per-(kernel, grid size) duration summary of a rocprofv3 --kernel-trace CSV.

    python tools/trace_summary.py gpurun_out/prof_TAG/kt/run_kernel_trace.csv

bench.py launches its calibration passes on smaller inputs before the timed steps; grouping by
grid size separates those from the timed launches, whose average must agree with the
`avg_launch_ms` bench.py measures with HIP events.
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_meta import resolve_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv')
    ap.add_argument('--json', help='update this file: {"config<N>": {kernel: avg ms of its largest-grid launches}}')
    ap.add_argument('--config', type=int, default=None,
                    help='bench config (only for traces without a bench line next to them; else checked)')
    a = ap.parse_args()
    # prof_TAG/kt/run_kernel_trace.csv: the bench line is prof_TAG/kt.log
    prof_dir = os.path.dirname(os.path.dirname(os.path.abspath(a.csv)))
    if a.json:
        a.config = resolve_config(prof_dir, a.config)
    rows = list(csv.DictReader(open(a.csv)))
    g = defaultdict(list)
    for r in rows:
        grid = int(r['Grid_Size_X']) * int(r['Grid_Size_Y']) * int(r['Grid_Size_Z'])
        name = r['Kernel_Name'].split('(')[0]
        g[(name, grid)].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
    print('%-48s %10s %6s %10s %10s %10s %10s' % ('kernel', 'grid', 'calls', 'avg_ms', 'median_ms', 'min_ms', 'max_ms'))
    med = lambda d: sorted(d)[len(d) // 2]
    for (name, grid), d in sorted(g.items(), key=lambda kv: -sum(kv[1])):
        print('%-48s %10d %6d %10.4f %10.4f %10.4f %10.4f' % (name[:48], grid, len(d), sum(d) / len(d), med(d), min(d),
                                                             max(d)))
    if a.json:
        # bench.py's kernel names: the median over the largest-grid launches (the timed steps)
        names = {'k_front': 'k_front', 'k_channelize': 'k_channelize', 'k_lpf_phase': 'k_lpf_phase',
                 'k_trig_spec': 'k_trig_spec', 'k_pulse_heights': 'k_pulse_heights'}
        best = {}
        for (name, grid), d in g.items():
            for key, short in names.items():
                if key in name and (short not in best or grid > best[short][0]):
                    # median of the full-size launches (calibration passes on smaller inputs can
                    # share the grid size; the cold first launch is an outlier)
                    big = [x for x in d if x >= 0.5 * max(d)]
                    best[short] = (grid, med(big))
        rec = json.load(open(a.json)) if os.path.exists(a.json) else {}
        rec['config%d' % a.config] = {k: round(v[1], 4) for k, v in best.items()}
        rec['config%d' % a.config]['source'] = a.csv
        rec['config%d' % a.config]['bench_config'] = a.config
        json.dump(rec, open(a.json, 'w'), indent=1)


if __name__ == '__main__':
    main()
