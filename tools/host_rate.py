#!/usr/bin/env python3
"""PCIe-inclusive throughput of the host-buffer API (mkid_process): int16 I/Q in host memory,
phase + packets back to host memory, 1024 channels. The bench's `value` uses HBM-resident
inputs (mkid_process_device); this is the rate a caller handing over host buffers sees.

    python tools/host_rate.py [--log2-samples 28] [--max-chunk-log2 26] [--no-phase]
"""
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
    ap.add_argument('--log2-samples', type=int, default=28)
    ap.add_argument('--max-chunk-log2', type=int, default=26)
    ap.add_argument('--no-phase', action='store_true')
    ap.add_argument('--reps', type=int, default=3)
    a = ap.parse_args()
    import torch
    from mkids_sdr_amd.channelizer import Channelizer
    C = 1024
    S = 1 << a.log2_samples
    rng = np.random.default_rng(0)
    iq = rng.integers(-3000, 3000, size=(S, 2), dtype=np.int16)
    ch = Channelizer(C, max_chunk=1 << a.max_chunk_log2, sample_rate=550e6)
    ch.set_thresholds(np.full(C, -(1 << 30), np.int32))
    ch.process(iq[: 1 << 20], want_phase=not a.no_phase)   # warm-up (lazy staging buffers)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        ch.process(iq, want_phase=not a.no_phase)
        ts.append(time.perf_counter() - t0)
    best = min(ts)
    print(json.dumps(dict(samples=S, max_chunk=1 << a.max_chunk_log2, seconds=best,
                          msps=S / best / 1e6, phase_to_host=not a.no_phase)))
    ch.close()


if __name__ == '__main__':
    main()
