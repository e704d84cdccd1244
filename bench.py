#!/usr/bin/env python3
"""Benchmark: ADC MSample/s per GPU through the full MKID chain at 1024 channels (BASELINE.json
configs[2]: "1024-ch full chain incl. matched-filter pulse trigger, 1 MI355X"), one feedline per
GPU, photon-packet lists gathered to rank 0 over RCCL (configs[3] when N > 1).

A step = one pass of the hot path over one batch of 2^30 synthetic int16 I/Q samples resident in
HBM (4 GiB): PFB+FFT+DDC -> IQ low-pass/2 + phase (materialised, fp32) -> matched filter +
baseline + trigger -> packets; then the packet gather. Prints ONE JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
FP32_PEAK_TFLOPS = 157.3        # MI355X_MICROARCH.md chip table (vector FP32)
ALG_BYTES_PER_SAMPLE = 6.0      # 4 B int16 I/Q in + 2 B fp32 phase out
CHAN_FLOPS_PER_SAMPLE = None    # filled from the FFT size below


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=10)
    p.add_argument('--warmup', type=int, default=2)
    p.add_argument('--channels', type=int, default=1024)
    p.add_argument('--fs', type=float, default=550e6)
    p.add_argument('--log2-samples', type=int, default=30)
    p.add_argument('--pulse-rate', type=float, default=1.0 / 2048,
                   help='Poisson pulses per phase sample per channel')
    p.add_argument('--cpu-samples-log2', type=int, default=26)
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--no-phase', action='store_true', help='do not materialise the phase stream')
    return p.parse_args()


def setup_feedline(C, fs, seed):
    """Tones one per channel via the reference setup math (product host code, mkids_sdr_amd.lut):
    DDS LUTs + bins (define_DDS_LUT / select_bins), DAC comb (define_DAC_LUT) -> ADC base."""
    from mkids_sdr_amd import lut
    N = 2 * C
    res = fs / lut.LUT_LEN
    upb = lut.LUT_LEN // N
    rng = np.random.default_rng(seed)
    bins = rng.permutation(np.arange(1, N))[:C]
    m = rng.integers(-(upb // 4), upb // 4 + 1, C)
    f_base = 4.0e9
    f_rf = [f_base + float((int(b) * upb + int(k)) * res) for b, k in zip(bins, m)]
    f_rf = [f - fs if f - f_base >= fs / 2 else f for f in f_rf]     # keep within +-fs/2 of LO
    dds = lut.define_dds_lut(f_rf, f_base, C, fs)
    I_dac, Q_dac, freqs_dac, sf, phases = lut.define_dac_lut(f_rf, f_base, np.zeros(C), fs)
    base = np.stack([I_dac, -Q_dac], axis=1).astype(np.int16)       # loop-back conjugation
    freq_index = np.array([int(round(((fs - f) % fs) / res)) for f in freqs_dac], np.int64)
    tone_amp = lut.FULL_SCALE / sf
    return dict(dds=dds, base=base, freq_index=freq_index, phases=phases, tone_amp=tone_amp,
                f_rf=f_rf, f_base=f_base)


def make_pulses(C, n_samples, N, rate, rng, tau_fall=65.0, window_phase=390):
    J = n_samples // N
    starts, tones, amps = [], [], []
    for ch in range(C):
        k = rng.poisson(rate * J)
        s = rng.integers(0, J, k) * N + rng.integers(0, N, k)
        starts.append(s)
        tones.append(np.full(k, ch))
        amps.append(np.deg2rad(rng.uniform(20.0, 100.0, k)))
    s = np.concatenate(starts)
    o = np.argsort(s, kind='stable')
    return s[o], np.concatenate(tones)[o], np.concatenate(amps)[o]


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        dist.init_process_group('nccl')
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)

    from mkids_sdr_amd import _lib
    from mkids_sdr_amd.channelizer import Channelizer
    from mkids_sdr_amd import codecs

    C = args.channels
    N = 2 * C
    S = 1 << args.log2_samples
    J = S // N
    fs = args.fs
    feed = setup_feedline(C, fs, 1000 + rank)
    mf = codecs.fir_quantise(np.loadtxt(os.path.join(ROOT, 'tests', 'golden', 'fir', 'matched_30us.txt')))
    lpf = codecs.fir_quantise(np.loadtxt(os.path.join(ROOT, 'tests', 'golden', 'fir',
                                                      'BlackmanFilter_250kHz.txt')))

    ch = Channelizer(C, device=local, max_chunk=S, dead_time=32, sample_rate=fs)
    stream = torch.cuda.current_stream(dev)
    ch.set_stream(stream.cuda_stream)
    ch.set_bins(feed['dds']['bins'])
    ch.set_dds(feed['dds']['lut_i'], feed['dds']['lut_q'])
    ch.set_lpf(lpf)
    ch.set_fir(np.tile(mf, (C, 1)))
    ch.set_baseline(_lib.BASE_EMA, 41, 82, 93623, 8192)

    # ---- synthetic input resident in HBM ----
    rng = np.random.default_rng(42 + rank)
    base = torch.from_numpy(feed['base']).to(dev)
    tones = np.zeros(C, dtype=[('amp', '<f4'), ('phase0', '<f4'), ('freq_index', '<i4'), ('pad', '<i4')])
    tones['amp'] = feed['tone_amp']
    tones['phase0'] = -np.asarray(feed['phases'])
    tones['freq_index'] = feed['freq_index']
    d_tones = torch.from_numpy(tones.view(np.uint8)).to(dev)
    ps, pt, pa = make_pulses(C, S, N, args.pulse_rate, rng)
    pul = np.zeros(len(ps), dtype=[('start', '<i8'), ('tone', '<i4'), ('amp_rad', '<f4')])
    pul['start'], pul['tone'], pul['amp_rad'] = ps, pt, pa
    d_pul = torch.from_numpy(pul.view(np.uint8)).to(dev) if len(ps) else torch.zeros(16, dtype=torch.uint8, device=dev)
    x = torch.empty(S * 2, dtype=torch.int16, device=dev)
    sigma = 0.01 * 32767 / np.sqrt(2.0)
    ch.synth_adc(x, S, 0, base, d_tones, d_pul, len(ps), 0.1 * N, 65.0 * N, 390 * N, sigma, 42 + rank)

    # ---- loop calibration + thresholds the reference way, on a pulse-free stream:
    #      rotateLoopsReady (ROACH_Setup.py:645-667: DDS phase = arctan2 of the on-resonance avg
    #      IQ, so every channel's phase sits near 0), then loadThresholds (ROACH_Pulses.py:211-299)
    quiet_n = 1 << 24
    q = torch.empty(quiet_n * 2, dtype=torch.int16, device=dev)
    ch.synth_adc(q, quiet_n, 0, base, d_tones, d_pul, 0, 0.1 * N, 65.0 * N, 390 * N, sigma, 7 + rank)
    qphase = torch.empty((quiet_n // N) * C, dtype=torch.float32, device=dev)
    cap = J * C // 8 + 1024
    d_events = torch.empty(cap, dtype=torch.int64, device=dev)
    d_counts = torch.zeros(2, dtype=torch.int64, device=dev)
    ch.set_thresholds(np.full(C, -(1 << 30), np.int32))
    ch.process_device(q, quiet_n, qphase, d_events, cap, d_counts)
    torch.cuda.synchronize(dev)
    mi, mq = ch.avg_iq()
    from mkids_sdr_amd import lut as _lut
    feed['dds'] = _lut.define_dds_lut(feed['f_rf'], feed['f_base'], C, fs, phase=np.arctan2(mq, mi))
    ch.set_dds(feed['dds']['lut_i'], feed['dds']['lut_q'])
    ch.reset()
    ch.process_device(q, quiet_n, qphase, d_events, cap, d_counts)
    torch.cuda.synchronize(dev)
    raw_q = torch.clamp(torch.round(qphase * 8192), -25736, 25736).view(-1, C).cpu().numpy().astype(np.int64)
    thr = codecs.thresholds_from_phase_block(raw_q)
    ch.set_thresholds(thr)
    ch.reset()
    del q, qphase

    phase = None if args.no_phase else torch.empty(J * C, dtype=torch.float32, device=dev)

    from mkids_sdr_amd.feedlines import gather_packets

    def step():
        ch.process_device(x, S, phase, d_events, cap, d_counts)
        if world > 1:   # photon-list gather to rank 0 (the path's one exchange step)
            gather_packets(d_events, int(d_counts[1].item()), dst=0)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ch.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    timing = ch.timing()
    counts = d_counts.cpu().numpy()
    ev_last = int(counts[0])
    reruns = ch.trigger_reruns()

    if rank == 0:
        total = S * args.steps * world
        value = total / dt / 1e6
        ms_step = dt / args.steps * 1e3
        kt = {k: (v[0] / max(v[1], 1)) for k, v in timing.items()}
        dom = max(kt, key=kt.get)
        n_launch = timing[dom][1] // args.steps if timing[dom][1] else 1
        # algorithmic HBM bytes per ADC sample of each kernel (DESIGN.md "Kernels"): the fused
        # front end reads 4 B of I/Q and writes 1 B of raw phase (+2 B of float phase)
        alg = {'k_front': 5.0 + (0.0 if args.no_phase else 2.0),
               'k_channelize': 4.0, 'k_lpf_phase': 1.0 + (0.0 if args.no_phase else 2.0),
               'k_trigger': 0.0, 'k_compact': 0.0}
        per_launch_samples = S / max(n_launch, 1)
        a_bytes = alg.get(dom, 0.0) * per_launch_samples
        achieved = a_bytes / (kt[dom] * 1e-3) / 1e9 if kt[dom] > 0 else 0.0
        traffic = None
        prof = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
        if os.path.exists(prof):
            try:
                bps = json.load(open(prof)).get(dom, {}).get('hbm_bytes_per_sample')
                traffic = None if bps is None else round(bps * per_launch_samples)
            except Exception:
                traffic = None
        fft_flops = 5.0 * N * np.log2(N) / (N / 2)      # per input sample (hop N/2)
        flops_per_sample = 8 * 4 + fft_flops + 8 + 52 + 20 + 26
        chain_gbps = ALG_BYTES_PER_SAMPLE * total / dt / 1e9
        out = {
            'metric': 'ADC MSample/s/GPU at 1024 ch; achieved HBM GB/s vs roofline',
            'value': round(value, 1),
            'unit': 'MSample/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(ms_step, 3),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'fp32+int16',
            'data': 'synthetic (seeded tone comb + AWGN + Poisson photon pulses, generated in HBM)',
            'config': {'workload': 'config3: %d-ch full chain incl. matched-filter trigger, fs=%.0f MS/s, '
                                   '2^%d int16 I/Q samples per GPU per step' % (C, fs / 1e6, args.log2_samples),
                       'channels': C, 'fft_len': N, 'pfb_taps': 4, 'samples_per_step_per_gpu': S,
                       'phase_materialised': not args.no_phase,
                       'parallelism': 'feedline-per-GPU x%d, RCCL packet gather' % world},
            'per_gpu_msps': round(value / world, 1),
            'packets_per_step_rank0': ev_last,
            'injected_pulses_rank0': int(len(ps)),
            'trigger_segments_rerun': reruns,
            'roofline': {'bound': 'hbm', 'kernel': dom, 'achieved': round(achieved, 1),
                         'peak': HBM_PEAK_GBPS, 'unit': 'GB/s',
                         'frac': round(achieved / HBM_PEAK_GBPS, 4), 'traffic': traffic,
                         'alg_bytes_per_launch': a_bytes, 'avg_launch_ms': round(kt[dom], 4),
                         'chain_alg_GBps': round(chain_gbps, 1),
                         'chain_frac': round(chain_gbps / HBM_PEAK_GBPS, 4),
                         'compute_tflops_est': round(flops_per_sample * total / dt / 1e12, 2),
                         'compute_peak_tflops': FP32_PEAK_TFLOPS},
            'kernel_ms': {k: round(v, 4) for k, v in kt.items()},
        }
        if not args.no_cpu_baseline and world == 1:
            out['cpu_baseline'] = cpu_baseline(x, C, feed, lpf, mf, thr, fs, 1 << args.cpu_samples_log2)
        print(json.dumps(out), flush=True)
    ch.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(x, C, feed, lpf, mf, thr, fs, n):
    """The oracle (numpy float64 chain + C trigger, one core) on the first n samples of the same
    GPU input (cpu_baseline.kind = 'port')."""
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    from oracle import chain, trigger
    iq = x[:2 * n].view(-1, 2).cpu().numpy()
    N = 2 * C
    o = chain.OracleChain(C, chain.pfb_prototype(N), feed['dds']['bins'], feed['dds']['lut_i'],
                          feed['dds']['lut_q'], lpf)
    tr = trigger.Trigger(C, np.tile(mf, (C, 1)), thr)
    blk = 1 << 22
    t0 = time.perf_counter()
    nev = 0
    for a in range(0, n, blk):
        r = o.process(iq[a:a + blk])
        _, k, _ = tr.run(r['raw'])
        nev += k
    dt = time.perf_counter() - t0
    return {'value': round(n / dt / 1e6, 3), 'unit': 'MSample/s', 'cores': 1, 'kind': 'port',
            'sample': 'first 2^%d samples of the GPU input, %.1f s, %d packets' % (int(np.log2(n)), dt, nev)}


if __name__ == '__main__':
    main()
