#!/usr/bin/env python3
"""Benchmark: ADC MSample/s per GPU through the full MKID chain (BASELINE.json metric "ADC
MSample/s/GPU at 1024 ch; achieved HBM GB/s vs roofline"), one feedline per GPU, photon-packet
lists gathered to rank 0 over RCCL when N > 1 (configs[3]).

A step = one pass of the hot path over one batch of synthetic int16 I/Q samples resident in HBM:
PFB+FFT+DDC -> IQ low-pass/2 + phase (materialised, fp32) -> matched filter + baseline + trigger
-> packets (-> per-packet fp32 optimal-filter pulse heights for config 5); then the packet gather.
Prints ONE JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config {2,3,5}] [--baseline {ema,svf}]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Without an external launcher (no WORLD_SIZE in the environment), `--gpus N > 1` starts N fresh
rank processes itself (`launch_ranks`: child processes, never an exec; the parent touches no GPU)
and relays rank 0's line — one feedline per GPU, as the reference runs one ROACH per feedline into
one PacketMaster (PacketMaster.c:216-218, 577-625). Under an external launcher WORLD_SIZE must
equal --gpus.

Configs (BASELINE.json `configs`; the default is configs[2], the one the
metric is quoted on):
  2  256 ch, N = 512, fs = 550 MS/s, 2^28 samples per step
  3  1024 ch, N = 2048, fs = 550 MS/s, 2^30 samples per step (default)
  5  2048 ch, N = 4096, fs = 2 GS/s, 2^30 samples per step, pulse heights in the step

Roofline: algorithmic bytes are 4 B of int16 I/Q read + 2 B of fp32 phase
written per ADC sample for the chain; a kernel's own share of those bytes over its HIP-event
launch time (on the stream it runs on) is `roofline.achieved`. Intermediate traffic (the
Fix16_13 raw phase, the staged baseband of the split front end) is overhead, reported as such.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
FP32_PEAK_TFLOPS = 157.3        # MI355X_MICROARCH.md chip table (vector FP32)
ALG_BYTES_PER_SAMPLE = 6.0      # 4 B int16 I/Q in + 2 B fp32 phase out

CONFIGS = {
    2: dict(channels=256, fs=550e6, log2=28, heights=False,
            name='config2: 256-ch PFB+FFT + DDC + phase (+ trigger), fs=550 MS/s'),
    3: dict(channels=1024, fs=550e6, log2=30, heights=False,
            name='config3: 1024-ch full chain incl. matched-filter trigger, fs=550 MS/s'),
    5: dict(channels=2048, fs=2e9, log2=30, heights=True,
            name='config5: 2048-ch full chain + per-packet fp32 optimal-filter pulse heights, fs=2 GS/s'),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=10)
    # the first launches of a fresh process run slower while the clock ramps (rocprofv3 traces,
    # profiles/r04/r04_v_*: config 3 k_front3 4.99, 4.65, 4.33, 4.30 ms then ~4.25; config 5 6.69 ->
    # 5.45 over six launches): ten untimed steps reach the steady state of a continuous stream
    p.add_argument('--warmup', type=int, default=10)
    p.add_argument('--config', type=int, default=3, choices=sorted(CONFIGS))
    p.add_argument('--baseline', default='ema', choices=['ema', 'svf'])
    p.add_argument('--rearm-q8', type=int, default=None,
                   help='trigger re-arm hysteresis /256 (mkid_set_rearm); default 96 for svf (removes the '
                        'pulse-tail re-fires on the operating-condition stream, DESIGN.md §2), 0 for ema')
    p.add_argument('--log2-samples', type=int, default=None, help='override the config sample count')
    p.add_argument('--pulse-rate', type=float, default=1.0 / 2048,
                   help='Poisson pulses per phase sample per channel')
    p.add_argument('--cpu-samples-log2', type=int, default=26, help='one-core CPU baseline sample')
    p.add_argument('--cpu-all-samples-log2', type=int, default=28, help='all-core CPU baseline sample')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--no-phase', action='store_true', help='do not materialise the phase stream')
    p.add_argument('--copy-mib', type=int, default=2048, help='stream-copy probe size (MiB)')
    p.add_argument('--backend', default='auto', choices=['auto', 'nccl', 'gloo'],
                   help='packet gather: RCCL on device buffers (one GPU per rank) or gloo through '
                        'pinned host memory (ranks may share a GPU); auto = nccl when every rank has '
                        'a GPU of its own, else gloo (decided by each rank, before any GPU call)')
    p.add_argument('--check-gather', action='store_true',
                   help='N > 1: verify that rank 0 received every rank\'s last-step packet list unchanged')
    p.add_argument('--force-gather', action='store_true',
                   help='run the packet gather (process group, double-buffered slots, side-stream '
                        'gather, barrier + max timing) even at N = 1: a world-size-1 group')
    p.add_argument('--launch-probe', action='store_true',
                   help='launcher check: each rank joins a gloo group, rank 0 prints the ranks\' '
                        'environment as one JSON line; no GPU call (CPU test of launch_ranks)')
    p.add_argument('--atten-span', type=float, default=20.0,
                   help='per-resonator attenuations uniform in [0, span] dB (define_DAC_LUT amplitudes)')
    p.add_argument('--loop-ratio-min', type=float, default=0.1,
                   help='IQ-loop radius / |centre| log-uniform in [min, 10]; 0: every loop centred at the origin')
    p.add_argument('--witness-samples-log2', type=int, default=24,
                   help='N > 1: samples of each rank\'s own feedline re-run for its parity witness')
    p.add_argument('--no-witness', action='store_true',
                   help='skip the parity witness: the one-core CPU sample (the first 2^cpu-samples-log2 '
                        'samples of the step input) re-run on the GPU from a reset context and compared '
                        'with the oracle outputs the CPU leg computes anyway')
    return p.parse_args()


def setup_feedline(C, fs, seed, atten_span=20.0, ratio_min=0.1):
    """Tones one per channel via the reference setup math (product host code, mkids_sdr_amd.lut):
    DDS LUTs + bins (define_DDS_LUT / select_bins), DAC comb (define_DAC_LUT) -> ADC base.

    Operating conditions of the reference: per-resonator attenuations uniform
    in [0, atten_span] dB, tone amplitudes 10^((atten_min - a)/20) inside one full-scale comb
    (define_DAC_LUT, ROACH_Setup.py:499-502), and every tone behind a resonator IQ loop (iqsweep.RESDIFF
    geometry, iqsweep.py:824-858) of radius R about a centre at 1 - R of the tone, R = ratio / (1 + ratio)
    with loop radius / |centre| log-uniform in [ratio_min, 10] (a fifth of the loops centred at the
    origin, R = 1). A photon moves the tone along its loop: the pulse amplitude of the synthetic source
    is tone_amp * gain * R. The centres are loaded after the loop rotation (main(): rotateLoopsReady,
    ROACH_Setup.py:645-667, then loadIQcenters, :595-617)."""
    from mkids_sdr_amd import lut
    N = 2 * C
    res = fs / lut.LUT_LEN
    upb = lut.LUT_LEN // N
    rng = np.random.default_rng(seed)
    bins = rng.permutation(np.arange(1, N))[:C]
    m = rng.integers(-(upb // 4), upb // 4 + 1, C) if upb >= 4 else np.zeros(C, int)
    f_base = 4.0e9
    f_rf = [f_base + float((int(b) * upb + int(k)) * res) for b, k in zip(bins, m)]
    f_rf = [f - fs if f - f_base >= fs / 2 else f for f in f_rf]     # keep within +-fs/2 of LO
    attens = rng.uniform(0.0, atten_span, C) if atten_span > 0 else np.zeros(C)
    if ratio_min > 0:
        ratio = np.exp(rng.uniform(np.log(ratio_min), np.log(10.0), C))
        ratio[rng.random(C) < 0.2] = np.inf
    else:
        ratio = np.full(C, np.inf)
    R = np.where(np.isfinite(ratio), ratio / (1.0 + np.where(np.isfinite(ratio), ratio, 0.0)), 1.0)
    dds = lut.define_dds_lut(f_rf, f_base, C, fs)
    I_dac, Q_dac, freqs_dac, sf, phases = lut.define_dac_lut(f_rf, f_base, attens, fs)
    base = np.stack([I_dac, -Q_dac], axis=1).astype(np.int16)       # loop-back conjugation
    freq_index = np.array([int(round(((fs - f) % fs) / res)) for f in freqs_dac], np.int64)
    tone_amp = lut.FULL_SCALE / sf
    gain = 10 ** ((attens.min() - attens) / 20.)
    return dict(dds=dds, base=base, freq_index=freq_index, phases=phases, tone_amp=tone_amp,
                f_rf=f_rf, f_base=f_base, attens=attens, gain=gain, loop_R=R)


def resolve_backend(backend, world, device_count=None):
    """--backend auto: RCCL when every rank has a GPU of its own (device_count() >= world, which does
    not initialise the GPU), gloo otherwise (N ranks rehearsing on fewer GPUs)."""
    if backend != 'auto':
        return backend
    if device_count is None:
        import torch
        device_count = torch.cuda.device_count()
    return 'nccl' if device_count >= world else 'gloo'


def make_pulses(C, n_samples, N, rate, rng):
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


def detector_score(ev, j_last, ps, pt, N, early=2, late=60, isolation=400, atten=None, loop_R=None):
    """Packets of the last step against the injected pulses (start sample ps, channel pt): a packet
    of channel c at row r matches a pulse of c starting at row p when p - early <= r <= p + late.
    Returns the fraction of isolated pulses (no other pulse of the channel within `isolation`
    rows) with exactly one packet, and the packets matching no pulse, histogrammed by their delay
    after the channel's previous pulse (a tail re-fire sits 60-300 rows after it, a noise trigger
    anywhere) and, given the per-channel attenuations and loop fractions R (loop radius over the
    tone's distance from the origin), by the channel's attenuation and R."""
    ev = np.asarray(ev, np.uint64)
    ch = ((ev >> np.uint64(52)) & np.uint64(0xFFF)).astype(np.int64)
    row = ((ev & np.uint64((1 << 28) - 1)).astype(np.int64) - j_last) % (1 << 28)
    prow = np.asarray(ps, np.int64) // N
    pch = np.asarray(pt, np.int64)
    key = pch * (1 << 40) + prow
    o = np.argsort(key)
    key, pch, prow = key[o], pch[o], prow[o]
    k = np.searchsorted(key, ch * (1 << 40) + row + early, side='right') - 1
    ok = (k >= 0) & (pch[np.maximum(k, 0)] == ch) & (row >= prow[np.maximum(k, 0)] - early) & \
        (row <= prow[np.maximum(k, 0)] + late)
    nhit = np.bincount(k[ok], minlength=len(key))
    same_prev = np.r_[False, pch[1:] == pch[:-1]] & (np.r_[0, np.diff(prow)] < isolation)
    same_next = np.r_[pch[1:] == pch[:-1], False] & (np.r_[np.diff(prow), 0] < isolation)
    iso = ~(same_prev | same_next)
    um = ~ok
    prev = (k >= 0) & (pch[np.maximum(k, 0)] == ch)
    delay = np.where(prev, row - prow[np.maximum(k, 0)], -1)[um]
    edges = [61, 100, 200, 300, 1000, 1 << 40]
    hist = {'no_earlier_pulse': int((delay < 0).sum())}
    for lo, hi in zip(edges[:-1], edges[1:]):
        hist['%d-%s' % (lo, hi - 1 if hi < (1 << 40) else 'inf')] = int(((delay >= lo) & (delay < hi)).sum())
    out = dict(isolated=int(iso.sum()), exactly_one_frac=round(float((nhit[iso] == 1).mean()), 4) if iso.any() else None,
               missed=int((nhit[iso] == 0).sum()), multi=int((nhit[iso] > 1).sum()),
               unmatched_packets=int(um.sum()), packets=int(len(ev)), pulses=int(len(key)),
               unmatched_per_pulse=round(float(um.sum()) / max(1, len(key)), 5),
               unmatched_delay_rows=hist)
    if atten is not None and um.any():
        a = np.asarray(atten, np.float64)[ch[um]]
        out['unmatched_by_atten_db'] = [{'atten_db': [lo, lo + 5], 'packets': int(((a >= lo) & (a < lo + 5)).sum())}
                                        for lo in range(0, int(np.ceil(a.max() + 1e-9)) + 1, 5)
                                        if ((a >= lo) & (a < lo + 5)).any()]
    if loop_R is not None and um.any():
        r = np.asarray(loop_R, np.float64)[ch[um]]
        out['unmatched_by_loop_R'] = [{'R': [lo, hi], 'packets': int(((r >= lo) & (r < hi)).sum())}
                                      for lo, hi in ((0.0, 0.25), (0.25, 0.5), (0.5, 0.75), (0.75, 1.01))]
    return out


def pulse_filter(C, npre=20, ncoeff=100, tau_fall=65.0):
    """Config 5 per-channel filter: the matched (template) filter of the injected pulse shape
    -(1 - e^{-t/0.1}) e^{-t/65} (pulses.py:470-472) over ncoeff phase rows starting npre rows
    before the packet's peak stamp, normalised to unit response to a unit-amplitude pulse; one
    row per channel (mkid_set_pulse_filter). Returns (coeff [C][ncoeff], pre)."""
    t = np.arange(ncoeff, dtype=np.float64) - npre
    tpl = np.where(t >= 0, -(1 - np.exp(-np.maximum(t, 0) / 0.1)) * np.exp(-np.maximum(t, 0) / tau_fall), 0.0)
    g = tpl / np.dot(tpl, tpl)
    return np.tile(g.astype(np.float32), (C, 1)), npre


def gather_report(gather, ev_slots, cnt_slots, last, rank, world, ctrl, args):
    """After the timed loop (outside it): per-rank packet counts of the last step and, with
    --check-gather, whether rank 0's gathered lists equal every rank's own list byte for byte
    (sha256 of the int64 words exchanged over the host control group)."""
    import hashlib
    import torch.distributed as dist
    n = int(cnt_slots[last][1].item())
    mine = ev_slots[last][:n].cpu().numpy()
    own = (n, hashlib.sha256(mine.tobytes()).hexdigest())
    allown = [None] * world
    dist.all_gather_object(allown, own, group=ctrl)
    out = {'backend': args.backend, 'ranks': world, 'overlapped': True,
           'packets_gathered_total': int(gather.total) if rank == 0 else None,
           'last_step_counts': [a[0] for a in allown]}
    if args.check_gather and rank == 0:
        got = gather.last
        ok = got is not None and len(got) == world and all(
            (int(g.numel()), hashlib.sha256(g.numpy().tobytes()).hexdigest()) == tuple(allown[r])
            for r, g in enumerate(got))
        out['lists_equal_rank_own'] = bool(ok)
        out['feedlines_distinct'] = len({a[1] for a in allown}) == world
    return out


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` without an external launcher: start N rank processes running this
    script with the same arguments (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set,
    rendezvous on 127.0.0.1), wait for them, relay rank 0's JSON line and return the exit status.
    The parent imports no torch and never touches a GPU, and the ranks are fresh child processes
    (no exec). If a rank fails, the others are stopped (by their own PIDs) and its status is
    returned; rank 0 must print exactly one JSON line."""
    import signal
    import threading
    port = os.environ.get('MASTER_PORT') or str(_free_port())
    procs = []
    lines = []

    def relay(pipe):
        for ln in pipe:
            if ln.startswith('{'):
                lines.append(ln.strip())
            else:
                sys.stderr.write(ln)
        pipe.close()

    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, '-u', os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, text=True))
    reader = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    reader.start()
    status = 0
    live = list(range(n))
    while live:
        time.sleep(0.2)
        for r in list(live):
            rc = procs[r].poll()
            if rc is None:
                continue
            live.remove(r)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                sys.stderr.write('bench.py: rank %d exited with %d; stopping the other ranks\n' % (r, rc))
                for o in live:
                    try:
                        os.kill(procs[o].pid, signal.SIGTERM)
                    except OSError:
                        pass
                deadline = time.time() + 20
                for o in live:
                    try:
                        procs[o].wait(max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        procs[o].kill()
                        procs[o].wait()
                live = []
    reader.join(timeout=30)
    if status == 0:
        if len(lines) != 1:
            sys.stderr.write('bench.py: rank 0 printed %d JSON lines, expected 1\n' % len(lines))
            return 1
        print(lines[0], flush=True)
    return status


def launch_probe(world, rank):
    """--launch-probe: join a gloo group (no GPU call) and report every rank's view of the launch."""
    import torch.distributed as dist
    if os.environ.get('MKID_PROBE_FAIL_RANK') == str(rank):
        sys.exit(3)            # test hook: a rank that dies before the rendezvous
    dist.init_process_group('gloo')
    mine = {'rank': dist.get_rank(), 'world': dist.get_world_size(), 'env_rank': rank,
            'local_rank': int(os.environ.get('LOCAL_RANK', '0')), 'pid': os.getpid(),
            'ppid': os.getppid(), 'master_addr': os.environ.get('MASTER_ADDR')}
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    if rank == 0:
        print(json.dumps({'launch_probe': True, 'n_gpus': world, 'ranks': allr}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if 'WORLD_SIZE' in os.environ and world != args.gpus:
        raise SystemExit('WORLD_SIZE=%d but --gpus %d: launch one rank per GPU' % (world, args.gpus))
    if args.launch_probe:
        return launch_probe(world, rank)
    import torch
    import torch.distributed as dist

    # the rank's GPU first, then the process group bound to it (RCCL communicators are created
    # for this device, not guessed from the rank)
    # device_count() does not initialise the GPU; ranks share a device only when there are more
    # ranks than GPUs (a one-GPU box rehearsing N > 1, gloo backend only: RCCL needs distinct GPUs)
    ndev = torch.cuda.device_count()
    args.backend = resolve_backend(args.backend, world, ndev)
    gpu = local % max(ndev, 1)
    if world > 1 and args.backend == 'nccl' and world > ndev:
        raise SystemExit('%d ranks on %d GPUs: RCCL needs one GPU per rank (use --backend gloo)' % (world, ndev))
    torch.cuda.set_device(gpu)
    dev = torch.device('cuda', gpu)
    ctrl = None
    grouped = world > 1 or args.force_gather
    if grouped:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        if world == 1:                          # --force-gather: a world-size-1 group
            os.environ.setdefault('MASTER_PORT', str(_free_port()))
            os.environ.setdefault('RANK', '0')
            os.environ.setdefault('WORLD_SIZE', '1')
        if args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
            ctrl = dist.new_group(backend='gloo')     # host control channel (packet counts)
        else:
            dist.init_process_group('gloo')

    from mkids_sdr_amd import _lib
    from mkids_sdr_amd.channelizer import Channelizer
    from mkids_sdr_amd import codecs

    cf = CONFIGS[args.config]
    C = cf['channels']
    N = 2 * C
    log2 = cf['log2'] if args.log2_samples is None else args.log2_samples
    S = 1 << log2
    J = S // N
    fs = cf['fs']
    feed = setup_feedline(C, fs, 1000 + rank, args.atten_span, args.loop_ratio_min)
    mf = codecs.fir_quantise(np.loadtxt(os.path.join(ROOT, 'tests', 'golden', 'fir', 'matched_30us.txt')))
    lpf = codecs.fir_quantise(np.loadtxt(os.path.join(ROOT, 'tests', 'golden', 'fir',
                                                      'BlackmanFilter_250kHz.txt')))
    base_mode = _lib.BASE_SVF if args.baseline == 'svf' else _lib.BASE_EMA

    ch = Channelizer(C, device=gpu, max_chunk=S, dead_time=32, sample_rate=fs)
    # one stream for the context's kernels and torch's work on this rank: a torch.cuda.Stream,
    # not torch's default stream, whose handle is 0 (mkid_set_stream(NULL) selects the
    # context's own non-blocking stream, which events on torch's default stream do not order)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ch.set_stream(stream.cuda_stream)
    ch.set_bins(feed['dds']['bins'])
    ch.set_dds(feed['dds']['lut_i'], feed['dds']['lut_q'])
    ch.set_lpf(lpf)
    ch.set_fir(np.tile(mf, (C, 1)))
    ch.set_baseline(base_mode, 41, 82, 93623, 8192)
    if args.rearm_q8 is None:
        args.rearm_q8 = 96 if args.baseline == 'svf' else 0
    ch.set_rearm(args.rearm_q8)

    # ---- synthetic input resident in HBM ----
    rng = np.random.default_rng(42 + rank)
    base = torch.from_numpy(feed['base']).to(dev)
    tones = np.zeros(C, dtype=[('amp', '<f4'), ('phase0', '<f4'), ('freq_index', '<i4'), ('pad', '<i4')])
    tones['amp'] = feed['tone_amp'] * feed['gain'] * feed['loop_R']   # a photon moves the tone along its loop
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
    #      on snapshots of the RUNNING stream: the quiet block is processed twice and the second
    #      pass (filters settled, no start-up transient) is the snapshot
    quiet_n = min(1 << 24, S)
    q = torch.empty(quiet_n * 2, dtype=torch.int16, device=dev)
    ch.synth_adc(q, quiet_n, 0, base, d_tones, d_pul, 0, 0.1 * N, 65.0 * N, 390 * N, sigma, 7 + rank)
    qphase = torch.empty((quiet_n // N) * C, dtype=torch.float32, device=dev)
    cap = J * C // 8 + 1024
    d_events = torch.empty(cap, dtype=torch.int64, device=dev)
    d_counts = torch.zeros(2, dtype=torch.int64, device=dev)
    ch.set_thresholds(np.full(C, -(1 << 30), np.int32))
    ch.set_accumulator(True)             # startAccumulator (ROACH_Setup.py:654-659)
    ch.process_device(q, quiet_n, qphase, d_events, cap, d_counts)
    torch.cuda.synchronize(dev)
    mi, mq = ch.avg_iq()
    ch.set_accumulator(False)
    from mkids_sdr_amd import lut as _lut
    feed['dds'] = _lut.define_dds_lut(feed['f_rf'], feed['f_base'], C, fs, phase=np.arctan2(mq, mi))
    ch.set_dds(feed['dds']['lut_i'], feed['dds']['lut_q'])
    # loadIQcenters (ROACH_Setup.py:595-617): the loop centre of each tone at 1 - R of its rotated
    # rest IQ (the average IQ of the settled quiet stream)
    ch.reset()
    ch.process_device(q, quiet_n, qphase, d_events, cap, d_counts)
    ch.set_accumulator(True)             # the settled second pass only
    ch.process_device(q, quiet_n, qphase, d_events, cap, d_counts)
    torch.cuda.synchronize(dev)
    mi, mq = ch.avg_iq()
    ch.set_accumulator(False)            # off in the timed steps (the reference accumulates on demand)
    feed['ic'] = ((1.0 - feed['loop_R']) * mi).astype(np.float32)
    feed['qc'] = ((1.0 - feed['loop_R']) * mq).astype(np.float32)
    ch.set_centers(feed['ic'], feed['qc'])
    ch.reset()
    ch.process_device(q, quiet_n, qphase, d_events, cap, d_counts)
    ch.process_device(q, quiet_n, qphase, d_events, cap, d_counts)
    torch.cuda.synchronize(dev)
    raw_q = torch.clamp(torch.round(qphase * 8192), -25736, 25736).view(-1, C).cpu().numpy().astype(np.int64)
    thr = codecs.thresholds_from_phase_block(raw_q)
    ch.set_thresholds(thr)
    ch.reset()
    del q, qphase

    phase = None if args.no_phase else torch.empty(J * C, dtype=torch.float32, device=dev)
    heights = None
    if cf['heights']:
        if phase is None:
            raise SystemExit('config 5 needs the phase stream (pulse heights read it)')
        coeff, pre = pulse_filter(C)
        ch.set_pulse_filter(coeff, pre)
        heights = torch.empty(cap, dtype=torch.float32, device=dev)

    # packet buffers: one slot per step in flight; with N > 1 two, so that the gather of step k
    # (rank 0's PacketMaster role) overlaps step k+1's kernels (feedlines.PacketGather)
    slots = 2 if grouped else 1
    ev_slots = [d_events] + [torch.empty(cap, dtype=torch.int64, device=dev) for _ in range(slots - 1)]
    cnt_slots = [d_counts] + [torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(slots - 1)]
    gather = None
    if grouped:
        from mkids_sdr_amd.feedlines import PacketGather
        gather = PacketGather(ev_slots, cnt_slots, args.backend, dev, dst=0, ctrl_group=ctrl,
                              keep_last=args.check_gather)
    j0 = [0]
    kstep = [0]

    def step():
        k = kstep[0]
        s_ev, s_cnt = ev_slots[k % slots], cnt_slots[k % slots]
        if gather is not None:
            gather.before_step(k)
        ch.process_device(x, S, phase, s_ev, cap, s_cnt)
        if heights is not None:
            # every packet of the step; the written count d_counts[1] is read on the device (no
            # host round trip inside the step); NaN where the window leaves the step's rows
            ch.pulse_heights_counted(phase, J, j0[0], s_ev, s_cnt[1:], cap, heights)
        j0[0] += J
        if gather is not None:   # photon-list gather to rank 0 (the path's one exchange step)
            gather.after_step(k)
        kstep[0] += 1

    # per-kernel breakdown (kernel_ms) from the last warm-up steps, every kernel timed; the timed
    # steps below time only the front end (the roofline kernel): each timed launch records two
    # HIP events, and an event record costs ~5 us of stream time (profiles/r04/r04_v traces), ~2 % of
    # a config-2 step if every kernel were timed
    nbreak = min(3, args.warmup)
    for i in range(args.warmup):
        if i == args.warmup - nbreak:
            ch.set_timing(True)
        step()
    if gather is not None:
        gather.flush()
    torch.cuda.synchronize(dev)
    breakdown = ch.timing() if nbreak else {}
    ch.set_timing(True, kernels=['k_front', 'k_channelize'])
    if grouped:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if gather is not None:
        gather.flush()           # the last step's lists are on rank 0 inside the timed region
    torch.cuda.synchronize(dev)
    if grouped:
        dist.barrier()
    dt = time.perf_counter() - t0
    gather_info = None
    if grouped:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=ctrl)
        dt = float(tt.item())
        gather_info = gather_report(gather, ev_slots, cnt_slots, (kstep[0] - 1) % slots, rank, world,
                                    ctrl, args)
    timing = ch.timing()
    last = (kstep[0] - 1) % slots
    d_events, d_counts = ev_slots[last], cnt_slots[last]
    counts = d_counts.cpu().numpy()
    ev_last = int(counts[0])
    det = None
    if rank == 0:
        det = detector_score(d_events[:int(counts[1])].cpu().numpy().view(np.uint64),
                             (args.warmup + args.steps - 1) * J, ps, pt, N,
                             atten=feed['attens'], loop_R=feed['loop_R'])
    reruns = ch.trigger_reruns()
    ch.set_timing(False)
    # N > 1: every rank's own feedline gets a parity witness: the first
    # 2^witness-samples-log2 samples of its step input re-run from a reset context, compared with
    # the oracle in a CPU child pinned to a CPU of its own; rank 0 reports all ranks. Outside the
    # timed region; the CPU throughput legs stay at N = 1.
    parity_ranks = None
    if world > 1 and not args.no_witness:
        n_w = min(1 << args.witness_samples_log2, S)
        wit_r = witness_device(ch, x, n_w, C, N, dev, heights is not None)
        par_r = cpu_baseline(x, C, feed, lpf, mf, thr, n_w, n_w, base_mode, wit_r, witness_only=True,
                             cpu=rank, rearm_q8=args.rearm_q8)
        par_r = dict(par_r, rank=rank)
        parity_ranks = [None] * world
        dist.all_gather_object(parity_ranks, par_r, group=ctrl)

    if rank == 0:
        # measured HBM roof in the same run: stream copy of copy_mib MiB (the library's float4
        # copy, HIP-event timed on the context stream) and torch's copy_ (torch events); the
        # faster of the two is the measured roof
        nb = args.copy_mib << 20
        src = torch.empty(nb // 4, dtype=torch.int32, device=dev).fill_(1)
        dst = torch.empty_like(src)
        torch.cuda.synchronize(dev)
        ch.set_timing(True)
        for _ in range(6):
            ch.stream_copy(dst, src, nb)
        ct = ch.timing()['k_stream_copy']
        ch.set_timing(False)
        lib_copy = 2.0 * nb / (ct[0] / ct[1] * 1e-3) / 1e9
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        dst.copy_(src)
        e0.record()
        for _ in range(6):
            dst.copy_(src)
        e1.record()
        torch.cuda.synchronize(dev)
        torch_copy = 2.0 * nb * 6 / (e0.elapsed_time(e1) * 1e-3) / 1e9
        copy_gbps = max(lib_copy, torch_copy)
        del src, dst

        total = S * args.steps * world
        value = total / dt / 1e6
        ms_step = dt / args.steps * 1e3
        kt = {k: (v[0] / max(v[1], 1)) for k, v in timing.items() if v[1] > 0}
        # the other kernels' averages from the warm-up breakdown (the timed steps time the front)
        kb = {k: (v[0] / max(v[1], 1)) for k, v in breakdown.items() if v[1] > 0}
        kall = dict(kb, **kt)
        # the roofline is the front end's (the kernel that owns the algorithmic bytes); with the
        # slow SVF baseline the trigger can take longer, reported as dominant_kernel
        per_step = {k: (kt[k] * timing[k][1] / args.steps if k in kt else kb[k] * breakdown[k][1] / nbreak)
                    for k in kall}
        slowest = max(per_step, key=per_step.get)
        fronts = [k for k in ('k_front', 'k_channelize') if k in kt]
        dom = fronts[0] if fronts else slowest
        if dom not in kt:   # no front-end launch timed (not a bench path): fall back to the breakdown
            kt[dom] = kall[dom]
            timing[dom] = (kall[dom] * breakdown[dom][1], breakdown[dom][1])
        n_launch = timing[dom][1] // args.steps if timing[dom][1] else 1
        per_launch_samples = S / max(n_launch, 1)
        ph_b = 0.0 if args.no_phase else 2.0
        # algorithmic bytes per ADC sample of each kernel's share of the chain;
        # intermediates (raw Fix16_13 phase 1 B/sample, staged z 16 B/sample) are overhead
        alg = {'k_front': 4.0 + ph_b, 'k_channelize': 4.0, 'k_lpf_phase': ph_b,
               'k_trigger': 0.0, 'k_compact': 0.0, 'k_pulse_heights': 0.0}
        overhead = {'k_front': 1.0, 'k_channelize': 8.0, 'k_lpf_phase': 8.0 + 1.0, 'k_trigger': 1.25}
        a_bytes = alg.get(dom, 0.0) * per_launch_samples
        achieved = a_bytes / (kt[dom] * 1e-3) / 1e9 if kt[dom] > 0 else 0.0
        traffic = None
        prof = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
        if os.path.exists(prof):
            try:
                rec = json.load(open(prof)).get('config%d' % args.config, {}).get(dom, {})
                bps = rec.get('hbm_bytes_per_sample')
                traffic = None if bps is None else round(bps * per_launch_samples)
            except (OSError, ValueError):
                traffic = None
        prof_ms = None
        kp = os.path.join(ROOT, 'profiles', 'kernel_avg_ms.json')
        if os.path.exists(kp):
            try:
                prof_ms = json.load(open(kp)).get('config%d' % args.config, {}).get(dom)
            except (OSError, ValueError):
                prof_ms = None
        fft_flops = 5.0 * N * np.log2(N) / (N / 2)      # per input sample (hop N/2)
        flops_per_sample = 8 * 4 + fft_flops + 8 + 52 + 20 + 26
        chain_gbps = (4.0 + ph_b) * total / dt / 1e9
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
            'dtype': 'int16 in, fp32 DSP, int16 Fix16_13 trigger',
            'data': 'synthetic (seeded tone comb + AWGN + Poisson photon pulses, generated in HBM)',
            'config': {'workload': '%s, 2^%d int16 I/Q samples per GPU per step' % (cf['name'], log2),
                       'config': args.config, 'channels': C, 'fft_len': N, 'pfb_taps': 4,
                       'fs': fs, 'samples_per_step_per_gpu': S, 'baseline': args.baseline,
                       'rearm_q8': args.rearm_q8, 'atten_span_db': args.atten_span,
                       'loop_ratio_min': args.loop_ratio_min,
                       'phase_materialised': not args.no_phase,
                       'pulse_heights_in_step': bool(cf['heights']),
                       'parallelism': 'feedline-per-GPU x%d%s' % (
                           world, '' if not grouped else ', packet gather to rank 0 over %s' % (
                               'RCCL' if args.backend == 'nccl' else 'gloo (pinned host buffers)'))},
            'per_gpu_msps': round(value / world, 1),
            'packets_per_step_rank0': ev_last,
            'injected_pulses_rank0': int(len(ps)),
            'packets_per_injected_pulse': round(ev_last / max(1, len(ps)), 4),
            'detector': det,
            'trigger_segments_rerun': reruns,
            'roofline': {'bound': 'hbm', 'kernel': dom, 'dominant_kernel': slowest, 'achieved': round(achieved, 1),
                         'peak': HBM_PEAK_GBPS, 'unit': 'GB/s',
                         'frac': round(achieved / HBM_PEAK_GBPS, 4), 'traffic': traffic,
                         'alg_bytes_per_sample': alg.get(dom, 0.0),
                         'overhead_bytes_per_sample': overhead.get(dom, 0.0),
                         'alg_bytes_per_launch': a_bytes, 'avg_launch_ms': round(kt[dom], 4),
                         'avg_launch_ms_rocprof': prof_ms,
                         'stream_copy_GBps': round(copy_gbps, 1),
                         'stream_copy_detail': {'mkid_stream_copy': round(lib_copy, 1),
                                                'torch_copy_': round(torch_copy, 1), 'MiB': args.copy_mib},
                         'frac_vs_measured': round(achieved / copy_gbps, 4) if copy_gbps > 0 else None,
                         'chain_alg_GBps': round(chain_gbps, 1),
                         'chain_frac': round(chain_gbps / HBM_PEAK_GBPS, 4),
                         'chain_frac_vs_measured': round(chain_gbps / copy_gbps, 4) if copy_gbps > 0 else None,
                         'compute_tflops_est': round(flops_per_sample * total / dt / 1e12, 2),
                         'compute_peak_tflops': FP32_PEAK_TFLOPS},
            'kernel_ms': {k: round(v, 4) for k, v in kall.items()},
            'kernel_ms_source': 'front end: HIP events over the timed steps; others: the last %d warm-up steps' % nbreak,
        }
        if gather_info is not None:
            out['gather'] = gather_info
        if parity_ranks is not None:
            out['parity_ranks'] = parity_ranks
            out['parity_ranks_green'] = all(p.get('green') for p in parity_ranks)
        if not args.no_cpu_baseline and world == 1:
            n1 = min(1 << args.cpu_samples_log2, S)
            wit = None
            if not args.no_witness:
                wit = witness_device(ch, x, n1, C, N, dev, heights is not None)
            out['cpu_baseline'] = cpu_baseline(x, C, feed, lpf, mf, thr, n1, 1 << args.cpu_all_samples_log2,
                                               base_mode, wit, rearm_q8=args.rearm_q8)
            par = out['cpu_baseline'].pop('parity', None)
            if par is not None:
                out['parity'] = par
        print(json.dumps(out), flush=True)
    ch.close()
    if grouped:
        dist.destroy_process_group()


def witness_device(ch, x, n, C, N, dev, with_heights):
    """Full-size parity witness, GPU side (after the timed loop): the first n samples of the step
    input re-run through the product path from a reset context — the same geometry and
    configuration as every timed step, the same samples the CPU leg's oracle processes. Returns
    host copies: phase float32 [n/N][C], Fix16_13 raw int16 [n/N][C], packets uint64 and (config
    5) the per-packet heights of those packets."""
    import torch
    J = n // N
    cap = J * C // 4 + 1024
    ph = torch.empty(J * C, dtype=torch.float32, device=dev)
    ev = torch.empty(cap, dtype=torch.int64, device=dev)
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    ch.reset()
    ch.process_device(x, n, ph, ev, cap, cnt)
    torch.cuda.synchronize(dev)
    c = cnt.cpu().numpy()
    if c[0] > c[1]:
        raise RuntimeError('witness: %d packets produced, %d fit' % (c[0], c[1]))
    out = dict(phase=ph.view(J, C).cpu().numpy(), raw=ch.raw_phase(),
               packets=ev[:int(c[1])].cpu().numpy().view(np.uint64).copy())
    if with_heights:
        h = torch.empty(max(int(c[1]), 1), dtype=torch.float32, device=dev)
        ch.pulse_heights_device(ph, J, 0, ev, int(c[1]), h)
        torch.cuda.synchronize(dev)
        out['heights'] = h[:int(c[1])].cpu().numpy()
        coeff, pre = pulse_filter(C)
        out['coeff'], out['pre'] = coeff, np.int64(pre)
    return out


def cpu_baseline(x, C, feed, lpf, mf, thr, n1, nall, mode, witness=None, witness_only=False, cpu=0,
                 rearm_q8=0):
    """The oracle (numpy float64 chain + C trigger, in the step's baseline mode) on a bounded
    sample of the same GPU input, timed by tools/cpu_baseline.py in a child process: (i) one
    pinned core, (ii) all usable cores chunk-parallel (cpu_baseline.kind = 'port'). `value` is the
    one-core rate. With `witness` (witness_device's arrays for the first n1 samples) the child
    also compares the oracle outputs of its one-core leg with them; the result comes back as
    'parity'. witness_only (N > 1, every rank): no timing legs, only the witness comparison of the
    first n1 samples in a child pinned to CPU `cpu`; returns the 'parity' block."""
    from mkids_sdr_amd.pfb import pfb_prototype
    n = n1 if witness_only else max(n1, nall)
    n = min(n, x.numel() // 2)
    tmp = '/dev/shm' if os.path.isdir('/dev/shm') else '/tmp'
    inp = os.path.join(tmp, 'mkid_cpu_in_%d.npy' % os.getpid())
    cfgp = os.path.join(tmp, 'mkid_cpu_cfg_%d.npz' % os.getpid())
    witp = os.path.join(tmp, 'mkid_cpu_wit_%d.npz' % os.getpid())
    try:
        np.save(inp, x[:2 * n].view(-1, 2).cpu().numpy())
        np.savez(cfgp, C=C, pfb=pfb_prototype(2 * C), bins=feed['dds']['bins'], lut_i=feed['dds']['lut_i'],
                 lut_q=feed['dds']['lut_q'], lpf=lpf, fir=np.tile(mf, (C, 1)), thr=np.asarray(thr),
                 mode=np.int64(mode), rearm_q8=np.int64(rearm_q8), ic=feed['ic'], qc=feed['qc'], attens=feed['attens'],
                 loop_R=feed['loop_R'])
        cmd = [sys.executable, os.path.join(ROOT, 'tools', 'cpu_baseline.py'), '--input', inp,
               '--cfg', cfgp, '--one-core-samples', str(min(n1, n)), '--all-core-samples', str(min(nall, n))]
        if witness is not None:
            np.savez(witp, **witness)
            cmd += ['--witness', witp]
        if witness_only:
            cmd += ['--witness-only', '--cpu', str(cpu)]
        del witness
        env = dict(os.environ)
        for k in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS'):
            env[k] = '1'
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            if witness_only:
                return {'green': False, 'error': 'witness child failed: %s' % r.stderr[-400:]}
            return {'value': None, 'unit': 'MSample/s', 'cores': 1, 'kind': 'port',
                    'sample': 'cpu baseline failed: %s' % r.stderr[-400:]}
        res = json.loads(r.stdout.strip().splitlines()[-1])
        if witness_only:
            return res['parity']
    finally:
        for p in (inp, cfgp, witp):
            try:
                os.remove(p)
            except OSError:
                pass
    one, allc = res['one_core'], res['all_cores']
    out = {'value': one['value'], 'unit': 'MSample/s', 'cores': 1, 'kind': 'port',
           'sample': one['sample'] + ' (1 pinned core, OMP/BLAS threads 1)',
           'all_cores': allc, 'c1_cpu_only': res['c1'], 'cpu_model': res['cpu_model'],
           'os_cpu_count': res['os_cpu_count'], 'sched_affinity': res['sched_affinity'],
           'cpu_quota_cores': res.get('cpu_quota_cores')}
    if 'parity' in res:
        out['parity'] = res['parity']
    return out


if __name__ == '__main__':
    main()
