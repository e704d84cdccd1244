#!/usr/bin/env python3
"""Interleaved A/B timing of libmkidgpu build variants in ONE process (cdna guide §5.4 rule 24).

    python tools/kbench.py [--log2-samples 28] [--rounds 5] [--baseline svf] variantA.so variantB.so[:split] ...
Each variant gets its own context on the same synthetic 1024-channel input (bench.py's feedline,
calibrated); per round every variant processes the input once; per-kernel HIP-event times are
reported as median / min over rounds.
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
    ap.add_argument('libs', nargs='+')
    ap.add_argument('--log2-samples', type=int, default=28)
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--channels', type=int, default=1024)
    ap.add_argument('--baseline', default='ema', choices=['ema', 'svf'])
    args = ap.parse_args()
    import torch
    import bench
    from mkids_sdr_amd import _lib
    from mkids_sdr_amd import codecs, lut
    from mkids_sdr_amd.channelizer import Channelizer

    C = args.channels
    N = 2 * C
    S = 1 << args.log2_samples
    J = S // N
    fs = 550e6
    dev = torch.device('cuda', 0)
    feed = bench.setup_feedline(C, fs, 1000)
    mf = codecs.fir_quantise(np.loadtxt(os.path.join(ROOT, 'tests/golden/fir/matched_30us.txt')))
    lpf = codecs.fir_quantise(np.loadtxt(os.path.join(ROOT, 'tests/golden/fir/BlackmanFilter_250kHz.txt')))
    base = torch.from_numpy(feed['base']).to(dev)
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
    x = torch.empty(S * 2, dtype=torch.int16, device=dev)
    sigma = 0.01 * 32767 / np.sqrt(2.0)
    phase = torch.empty(J * C, dtype=torch.float32, device=dev)
    cap = J * C // 8 + 1024
    d_ev = torch.empty(cap, dtype=torch.int64, device=dev)
    d_cnt = torch.zeros(2, dtype=torch.int64, device=dev)

    chans = []
    for i, spec in enumerate(args.libs):
        path, _, front = spec.partition(':')  # lib.so[#a][:split]
        path, _, order = path.partition('#')  # '#a' / '#b': relabelled feedline; '#VAR=VAL': env at create
        env_set = None
        if '=' in order:
            env_set = order.split('=', 1)
            os.environ[env_set[0]] = env_set[1]
            order = ''
        ch = Channelizer(C, max_chunk=S, sample_rate=fs, lib_path=os.path.abspath(path),
                         front=front or 'auto')
        # '#a': the same feedline with its channels relabelled in tools/lds_assign.py slot order
        perm = np.arange(C)
        if order == 'a':
            from tools.lds_assign import slot_order
            perm = slot_order(feed['dds']['bins'], C)
        elif order == 'c':
            from tools.lds_assign import slot_order_f5
            perm = slot_order_f5(feed['dds']['bins'])
        elif order == 'b':
            from tools.lds_assign import slot_order_blocks
            perm = slot_order_blocks(feed['dds']['bins'], C=C)
        ch.set_bins(np.asarray(feed['dds']['bins'])[perm])
        ch.set_lpf(lpf)
        ch.set_fir(np.tile(mf, (C, 1)))
        if i == 0:
            ch.synth_adc(x, S, 0, base, d_tones, d_pul, len(ps), 0.1 * N, 65.0 * N, 390 * N, sigma, 42)
            ch.set_dds(feed['dds']['lut_i'], feed['dds']['lut_q'])
            ch.set_thresholds(np.full(C, -(1 << 30), np.int32))
            if hasattr(ch._L, 'mkid_set_accumulator'):   # older variants accumulate on every call
                ch.set_accumulator(True)
            ch.process_device(x, S, phase, d_ev, cap, d_cnt)
            torch.cuda.synchronize()
            mi, mq = ch.avg_iq()
            if hasattr(ch._L, 'mkid_set_accumulator'):
                ch.set_accumulator(False)
            cal = np.arctan2(mq, mi)
        dds = lut.define_dds_lut(list(np.asarray(feed['f_rf'])[perm]), feed['f_base'], C, fs, phase=cal[perm])
        assert np.array_equal(np.asarray(dds['bins']) % N, np.asarray(feed['dds']['bins'])[perm] % N)
        ch.set_dds(dds['lut_i'], dds['lut_q'])
        ch.set_thresholds(np.full(C, -3000, np.int32))
        if args.baseline == 'svf':   # bench.py's SVF settings (the EMA runs keep the context default)
            ch.set_baseline(_lib.BASE_SVF, 41, 82, 93623, 8192)
        if env_set:
            del os.environ[env_set[0]]
        chans.append(ch)
    times = {p: {} for p in args.libs}
    for r in range(args.rounds + 1):
        for path, ch in zip(args.libs, chans):
            ch.reset()
            ch.set_timing(True)
            ch.process_device(x, S, phase, d_ev, cap, d_cnt)
            torch.cuda.synchronize()
            t = ch.timing()
            ch.set_timing(False)
            if r == 0:
                times[path].setdefault('reruns', []).append(float(ch.trigger_reruns()))
                continue  # warm-up round
            for k, (ms, n) in t.items():
                times[path].setdefault(k, []).append(ms)
        for path, ch in zip(args.libs, chans):  # whole pass without per-kernel events
            ch.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ch.process_device(x, S, phase, d_ev, cap, d_cnt)
            torch.cuda.synchronize()
            if r:
                times[path].setdefault('wall', []).append((time.perf_counter() - t0) * 1e3)
    out = {}
    for path in args.libs:
        out[os.path.basename(path).replace('.so', '')] = {k: dict(median=float(np.median(v)), min=float(np.min(v)))
                                       for k, v in times[path].items()}
    print(json.dumps(dict(samples=S, channels=C, rounds=args.rounds, kernels_ms=out), indent=1))


if __name__ == '__main__':
    main()
