#!/usr/bin/env python3
"""Per-(kernel, grid size) duration summary of a rocprofv3 --kernel-trace CSV.

    python tools/trace_summary.py gpurun_out/prof_TAG/kt/run_kernel_trace.csv

bench.py launches its calibration passes on smaller inputs before the timed steps; grouping by
grid size separates those from the timed launches, whose average must agree with the
`avg_launch_ms` bench.py measures with HIP events.
"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    g = defaultdict(list)
    for r in rows:
        grid = int(r['Grid_Size_X']) * int(r['Grid_Size_Y']) * int(r['Grid_Size_Z'])
        name = r['Kernel_Name'].split('(')[0]
        g[(name, grid)].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
    print('%-48s %10s %6s %10s %10s %10s' % ('kernel', 'grid', 'calls', 'avg_ms', 'min_ms', 'max_ms'))
    for (name, grid), d in sorted(g.items(), key=lambda kv: -sum(kv[1])):
        print('%-48s %10d %6d %10.4f %10.4f %10.4f' % (name[:48], grid, len(d), sum(d) / len(d), min(d), max(d)))


if __name__ == '__main__':
    main()
