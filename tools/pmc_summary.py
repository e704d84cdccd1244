#!/usr/bin/env python3
"""Summarise tools/profile.sh output: per-kernel mean counter value per dispatch.

    python tools/pmc_summary.py gpurun_out/prof_TAG [--json profiles/pmc_traffic.json]

FETCH_SIZE / WRITE_SIZE are rocprofv3 KiB; HBM bytes per launch = 2 x FETCH_SIZE (gfx950 counts
half of a wide coalesced read, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both x 1024. The PMC passes
run bench.py on one step of the workload given to tools/profile.sh (2^30 samples at configs 3 and 5);
the config and the samples per launch are read from the run's own bench line (prof_TAG/kt.log,
tools/prof_meta.py) and filed under that config; bench.py scales `traffic` to its own launch size.
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_meta import resolve  # noqa: E402

KEEP = ('k_front', 'k_channelize', 'k_lpf_phase', 'k_trig_spec', 'k_trig_fix', 'k_tile_sums', 'k_tile_scan',
        'k_gather_events')


def short(name):
    for k in KEEP:
        if k in name:
            return k
    return None


def read(d):
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
    grid = {}
    for f in glob.glob(os.path.join(d, '*', 'run_counter_collection.csv')):
        for row in csv.DictReader(open(f)):
            k = short(row['Kernel_Name'])
            if not k:
                continue
            g = int(row['Grid_Size'])
            key = (os.path.basename(os.path.dirname(f)), row['Dispatch_Id'], g)
            c = per[k][row['Counter_Name']]
            c[key] = c.get(key, 0.0) + float(row['Counter_Value'])
            grid[k] = max(grid.get(k, 0), g)
    out = {}
    for k, cs in per.items():  # only the largest launches (the timed step, not calibration)
        out[k] = {}
        for c, v in cs.items():
            vals = [x for key, x in v.items() if key[2] == grid[k]]
            # calibration passes on smaller inputs can share the grid size (runs shrink with
            # the input): keep the full-size launches
            vals = [x for x in vals if x >= 0.5 * max(vals)] or vals
            out[k][c] = sum(vals) / len(vals)
        out[k]['grid'] = grid[k]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--json')
    ap.add_argument('--summary-out', help='also write the per-kernel lines to this file (profiles/...)')
    ap.add_argument('--samples-log2', type=int, default=None,
                    help='ADC samples per launch (only for runs without a bench line; else checked)')
    ap.add_argument('--config', type=int, default=None,
                    help='bench config (only for runs without a bench line; else checked)')
    a = ap.parse_args()
    a.config, samples = resolve(a.dir.rstrip('/'), a.config, None if a.samples_log2 is None else 1 << a.samples_log2)
    a.samples_log2 = samples.bit_length() - 1
    assert 1 << a.samples_log2 == samples
    s = read(a.dir)
    res = {}
    lines = []
    for k, c in sorted(s.items()):
        line = {n: round(v, 1) for n, v in sorted(c.items())}
        if 'FETCH_SIZE' in c and 'WRITE_SIZE' in c:
            hbm = (2 * c['FETCH_SIZE'] + c['WRITE_SIZE']) * 1024
            line['hbm_bytes_per_launch'] = hbm
            line['hbm_bytes_per_sample'] = hbm / (1 << a.samples_log2)
        if 'SQ_WAVE_CYCLES' in c:
            w = c['SQ_WAVE_CYCLES']
            for n in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU',
                      'SQ_WAIT_INST_LDS'):
                if n in c:
                    line[n + '/WAVE_CYCLES'] = round(c[n] / w, 3)
        res[k] = line
        lines.append('%s %s' % (k, json.dumps(line)))
        print(lines[-1])
    if a.summary_out:
        with open(a.summary_out, 'w') as f:
            f.write('\n'.join(lines) + '\n')
    if a.json:
        out = {k: {'hbm_bytes_per_launch': v.get('hbm_bytes_per_launch'),
                   'hbm_bytes_per_sample': v.get('hbm_bytes_per_sample'),
                   'pmc_samples': 1 << a.samples_log2, 'source': a.dir.rstrip('/'),
                   'bench_config': a.config, 'summary': a.summary_out}
               for k, v in res.items() if 'hbm_bytes_per_launch' in v}
        rec = json.load(open(a.json)) if os.path.exists(a.json) else {}
        rec = {k: v for k, v in rec.items() if k.startswith('config')}   # config-keyed layout
        rec['config%d' % a.config] = out
        json.dump(rec, open(a.json, 'w'), indent=1)


if __name__ == '__main__':
    main()
