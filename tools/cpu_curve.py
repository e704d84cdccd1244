#!/usr/bin/env python3
"""CPU-baseline scaling curve on the GPU box (no GPU use): the oracle chain-parallel leg of
tools/cpu_baseline.py at several worker counts on a bench-like config-3 input generated on the host
(signals.make_case: 1024 ch, seeded tones + noise + pulses), to show where the box's CPU share
saturates (the cgroup quota, not sched_getaffinity).

    python tools/cpu_curve.py [--samples-log2 26] [--workers 4,8,16,32,64,256] > profiles/r03/r03_cpu_curve.json
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--samples-log2', type=int, default=26)
    ap.add_argument('--workers', default='4,8,16,32,64,256')
    a = ap.parse_args()
    import signals
    C = 1024
    case = signals.make_case(C, 1 << 20, seed=3, pulses_per_ch=0.0)
    reps = (1 << a.samples_log2) // case.iq.shape[0]
    iq = np.tile(case.iq, (reps, 1))
    with tempfile.TemporaryDirectory(dir='/dev/shm' if os.path.isdir('/dev/shm') else None) as d:
        inp, cfgp = os.path.join(d, 'in.npy'), os.path.join(d, 'cfg.npz')
        np.save(inp, iq)
        np.savez(cfgp, C=C, pfb=case.pfb, bins=case.bins, lut_i=case.lut_i, lut_q=case.lut_q, lpf=case.lpf12,
                 fir=case.fir12, thr=np.full(C, -3000, np.int32), mode=np.int64(1))
        r = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'cpu_baseline.py'), '--input', inp, '--cfg', cfgp,
                            '--one-core-samples', str(1 << 20), '--all-core-samples', str(iq.shape[0]),
                            '--curve', a.workers], capture_output=True, text=True, timeout=1500)
        if r.returncode:
            sys.exit(r.stderr[-2000:])
        print(r.stdout.strip().splitlines()[-1])


if __name__ == '__main__':
    main()
