#!/usr/bin/env python3
"""Co-residency probe: does a trigger launch on a second context's stream overlap a front-end
launch on the first context's stream (distinct HW queues), or do they serialise?

    python tools/overlap_probe.py front.so trigger.so [--log2-samples 28] [--rows 131072]
Times (HIP wall, median of 5): front-end call alone, trigger-only call alone, both issued
back-to-back on their own streams."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('front_lib')
    ap.add_argument('trig_lib')
    ap.add_argument('--log2-samples', type=int, default=28)
    ap.add_argument('--rows', type=int, default=1 << 17)
    args = ap.parse_args()
    import torch
    import bench
    from mkids_sdr_amd import codecs
    from mkids_sdr_amd.channelizer import Channelizer
    C, N, fs = 1024, 2048, 550e6
    S = 1 << args.log2_samples
    dev = torch.device('cuda', 0)
    feed = bench.setup_feedline(C, fs, 1000)
    mf = codecs.fir_quantise(np.loadtxt(os.path.join(ROOT, 'tests/golden/fir/matched_30us.txt')))
    A = Channelizer(C, max_chunk=S, sample_rate=fs, lib_path=os.path.abspath(args.front_lib))
    B = Channelizer(C, max_chunk=args.rows * N, sample_rate=fs, lib_path=os.path.abspath(args.trig_lib))
    for ch in (A, B):
        ch.set_bins(feed['dds']['bins'])
        ch.set_dds(feed['dds']['lut_i'], feed['dds']['lut_q'])
        ch.set_fir(np.tile(mf, (C, 1)))
        ch.set_thresholds(np.full(C, -3000, np.int32))
    x = torch.randint(-3000, 3000, (2 * S,), dtype=torch.int16, device=dev)
    raw = torch.randint(-2000, 2000, (args.rows * C,), dtype=torch.int16, device=dev)
    phase = torch.empty((S // N) * C, dtype=torch.float32, device=dev)
    capA = (S // N) * C // 8 + 1024
    capB = args.rows * C // 8 + 1024
    evA = torch.empty(capA, dtype=torch.int64, device=dev)
    evB = torch.empty(capB, dtype=torch.int64, device=dev)
    cA = torch.zeros(2, dtype=torch.int64, device=dev)
    cB = torch.zeros(2, dtype=torch.int64, device=dev)

    def run(a, b):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if a:
            A.process_device(x, S, phase, evA, capA, cA)
        if b:
            B.trigger_phase_device(raw, args.rows, evB, capB, cB)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) * 1e3

    out = {}
    for name, a, b in (('front_call', 1, 0), ('trigger_call', 0, 1), ('both', 1, 1)):
        run(a, b)
        out[name] = float(np.median([run(a, b) for _ in range(5)]))
    out['serial_sum'] = out['front_call'] + out['trigger_call']
    print(json.dumps(out))


if __name__ == '__main__':
    main()
