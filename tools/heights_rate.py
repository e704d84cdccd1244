#!/usr/bin/env python3
"""Time mkid_pulse_heights (k_heights.hip) at the bench's packet volume: phase [2^19][1024]
(one 2^30-sample step of config 3's geometry) and ~690k packets spread over the channels, for
ncoeff 100 (PulseAnalysis.coeff, pulses.py:59). Prints one JSON line.

    python tools/heights_rate.py [--packets 690000] [--ncoeff 100] [--reps 20]
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
    ap.add_argument('--packets', type=int, default=690000)
    ap.add_argument('--ncoeff', type=int, default=100)
    ap.add_argument('--reps', type=int, default=20)
    args = ap.parse_args()
    import torch
    from mkids_sdr_amd.channelizer import Channelizer
    C, J, pre = 1024, 1 << 19, 40
    ch = Channelizer(C, max_chunk=1 << 20)
    rng = np.random.default_rng(0)
    ch.set_pulse_filter(rng.normal(size=(C, args.ncoeff)).astype(np.float32), pre)
    d_ph = torch.randn(J, C, device='cuda')
    chs = rng.integers(0, C, args.packets)
    ts = np.sort(rng.integers(pre, J - args.ncoeff, args.packets))
    ev = ((chs.astype(np.uint64) << np.uint64(52)) | ts.astype(np.uint64)).view(np.int64)
    d_ev = torch.from_numpy(ev).cuda()
    d_h = torch.empty(args.packets, dtype=torch.float32, device='cuda')
    torch.cuda.synchronize()
    for _ in range(3):
        ch.pulse_heights_device(d_ph, J, 0, d_ev, args.packets, d_h)
    torch.cuda.synchronize()
    # the context runs on its own stream: bracket with device-wide synchronisation
    torch.cuda.synchronize()
    s = time.perf_counter()
    for _ in range(args.reps):
        ch.pulse_heights_device(d_ph, J, 0, d_ev, args.packets, d_h)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - s) / args.reps * 1e3
    print(json.dumps(dict(kernel='k_pulse_heights', packets=args.packets, ncoeff=args.ncoeff,
                          ms_per_call=round(ms, 4), mpackets_per_s=round(args.packets / ms / 1e3, 1),
                          phase_bytes_read_per_packet=4 * args.ncoeff)))
    ch.close()


if __name__ == '__main__':
    main()
