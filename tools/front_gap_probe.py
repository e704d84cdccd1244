#!/usr/bin/env python3
"""Why is k_front3 slower in the SVF bench than in the EMA bench (4.93 vs
4.15 ms, same kernel, same input)? The SVF step spends ~14 ms after each front end in a
trigger that keeps only a few waves busy; this probe runs the EMA step (front end + EMA trigger)
with a controlled gap after each step and times the front end with HIP events:

  none      back to back (the EMA bench)
  spin      a one-wave GPU spin kernel of GAP ms on the stream (a light GPU load, like the SVF
            trigger's long tail)
  idle      the host sleeps GAP ms with the GPU idle
  svf       the real SVF step (front end + SVF trigger), for reference

    python tools/front_gap_probe.py [--gap-ms 14] [--steps 12] [--log2-samples 30]
Prints one JSON line: per mode the median / min front-end ms and the median step ms.
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
    ap.add_argument('--gap-ms', type=float, default=14.0)
    ap.add_argument('--steps', type=int, default=12)
    ap.add_argument('--log2-samples', type=int, default=30)
    args = ap.parse_args()
    import torch
    import bench
    from mkids_sdr_amd import _lib, codecs, lut
    from mkids_sdr_amd.channelizer import Channelizer

    C, fs = 1024, 550e6
    N = 2 * C
    S = 1 << args.log2_samples
    J = S // N
    dev = torch.device('cuda', 0)
    feed = bench.setup_feedline(C, fs, 1000)
    mf = codecs.fir_quantise(np.loadtxt(os.path.join(ROOT, 'tests/golden/fir/matched_30us.txt')))
    tones = np.zeros(C, dtype=[('amp', '<f4'), ('phase0', '<f4'), ('freq_index', '<i4'), ('pad', '<i4')])
    tones['amp'] = feed['tone_amp']
    tones['phase0'] = -np.asarray(feed['phases'])
    tones['freq_index'] = feed['freq_index']
    d_tones = torch.from_numpy(tones.view(np.uint8)).to(dev)
    rng = np.random.default_rng(42)
    ps, pt, pa = bench.make_pulses(C, S, N, 1.0 / 2048, rng)
    pul = np.zeros(len(ps), dtype=[('start', '<i8'), ('tone', '<i4'), ('amp_rad', '<f4')])
    pul['start'], pul['tone'], pul['amp_rad'] = ps, pt, pa
    d_pul = torch.from_numpy(pul.view(np.uint8)).to(dev)
    base = torch.from_numpy(feed['base']).to(dev)
    x = torch.empty(S * 2, dtype=torch.int16, device=dev)
    phase = torch.empty(J * C, dtype=torch.float32, device=dev)
    cap = J * C // 8 + 1024
    d_ev = torch.empty(cap, dtype=torch.int64, device=dev)
    d_cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    ch = Channelizer(C, max_chunk=S, sample_rate=fs)
    ch.set_bins(np.asarray(feed['dds']['bins']))
    ch.set_dds(feed['dds']['lut_i'], feed['dds']['lut_q'])
    ch.set_lpf(codecs.fir_quantise(np.loadtxt(os.path.join(ROOT, 'tests/golden/fir/BlackmanFilter_250kHz.txt'))))
    ch.set_fir(np.tile(mf, (C, 1)))
    ch.set_thresholds(np.full(C, -(1 << 30), np.int32))
    ch.synth_adc(x, S, 0, base, d_tones, d_pul, len(ps), 0.1 * N, 65.0 * N, 390 * N, 0.01 * 32767 / np.sqrt(2.0), 42)
    # rotate the loops as tools/kbench.py does (avgIQ -> DDS phase), so the phase sits near 0 and the
    # trigger sees the bench's packet rate
    ch.set_accumulator(True)
    ch.process_device(x, S, phase, d_ev, cap, d_cnt)
    torch.cuda.synchronize()
    mi, mq = ch.avg_iq()
    ch.set_accumulator(False)
    dds = lut.define_dds_lut(list(feed['f_rf']), feed['f_base'], C, fs, phase=np.arctan2(mq, mi))
    ch.set_dds(dds['lut_i'], dds['lut_q'])
    ch.set_thresholds(np.full(C, -3000, np.int32))
    torch.cuda.synchronize()
    stream = torch.cuda.Stream(dev)          # the context and the spin kernel share it
    ch.set_stream(stream.cuda_stream)
    # torch.cuda._sleep's cycle count is in the GPU's own clock ticks: on the box this gave a
    # ~0.75 ms spin for a nominal 14 ms (profiles/r06/r06c_front_gap_probe.json); the 'idle' mode
    # is the one with the full gap
    spin_cycles = int(args.gap_ms * 1e-3 * 100e6)
    out = {}
    for mode in ('none', 'spin', 'idle', 'svf', 'none'):
        ch.set_baseline(_lib.BASE_SVF if mode == 'svf' else _lib.BASE_EMA, 41, 82, 93623, 8192)
        ch.reset()
        fronts, steps = [], []
        for k in range(args.steps + 3):
            ch.set_timing(True)
            t0 = time.perf_counter()
            ch.process_device(x, S, phase, d_ev, cap, d_cnt)
            if mode == 'spin':
                with torch.cuda.stream(stream):
                    torch.cuda._sleep(spin_cycles)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            t = ch.timing()
            ch.set_timing(False)
            if mode == 'idle':
                time.sleep(args.gap_ms * 1e-3)
            if k >= 3:
                fronts.append(t['k_front'][0])
                steps.append(dt)
        key = mode if mode not in out else mode + '_again'
        out[key] = dict(front_ms_median=float(np.median(fronts)), front_ms_min=float(np.min(fronts)),
                        step_ms_median=float(np.median(steps)))
        print(key, out[key], file=sys.stderr, flush=True)
    ch.close()
    print(json.dumps(dict(gap_ms=args.gap_ms, samples=S, channels=C, modes=out)))


if __name__ == '__main__':
    main()
