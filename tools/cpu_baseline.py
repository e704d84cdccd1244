#!/usr/bin/env python3
"""CPU baseline of bench.py: the oracle — numpy float64 chain
K1-K6 (oracle/chain.py) + C trigger K7-K8 (oracle/trigger.c) — timed on the host cores on a
bounded sample of the GPU workload, in two forms:

  (i)  one core: one process pinned to one CPU, OMP/BLAS threads 1;
  (ii) all cores: the sample cut into W chunks processed by W pinned single-thread processes,
       each chunk preceded by a warm-up prefix (the PFB/low-pass history, (2T-1+24) hops, and
       the trigger's speculative warm-up, 520 rows — the same overlap the device uses) whose
       outputs are discarded; the rate counts chunk samples only.

It also times config 1 (64 ch, 2^16 samples, CPU only) on one core. Runs as its own process
(bench.py starts it with subprocess, so no process that touched the GPU forks or execs); reads the
input sample and the channel configuration from files bench.py wrote. Prints one JSON line.

TEST / MEASUREMENT INFRASTRUCTURE: this is the only bench leg that imports oracle/.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _single_thread_env():
    for k in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS', 'NUMEXPR_NUM_THREADS'):
        os.environ[k] = '1'


def _pin(cpu):
    try:
        os.sched_setaffinity(0, {cpu})
    except (AttributeError, OSError):
        pass


def cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def _load_cfg(path):
    import numpy as np
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}


def run_chunk(args):
    """Worker: process samples [a, b) of the shared input with a warm-up prefix; returns
    (samples counted, seconds, packets)."""
    cpu, inp, cfgp, a, b, prefix = args
    _single_thread_env()
    _pin(cpu)
    sys.path.insert(0, ROOT)
    import numpy as np
    from oracle import chain, trigger
    cfg = _load_cfg(cfgp)
    C = int(cfg['C'])
    N = 2 * C
    iq = np.load(inp, mmap_mode='r')
    o = chain.OracleChain(C, cfg['pfb'], cfg['bins'], cfg['lut_i'], cfg['lut_q'], cfg['lpf'])
    tr = trigger.Trigger(C, cfg['fir'], cfg['thr'])
    p0 = max(0, a - prefix)
    t0 = time.perf_counter()
    # warm-up prefix: history of the chain and of the trigger (outputs discarded)
    nev = 0
    blk = 1 << 22
    if a > p0:
        r = o.process(np.asarray(iq[p0:a]))
        tr.run(r['raw'])
    for s in range(a, b, blk):
        e = min(b, s + blk)
        r = o.process(np.asarray(iq[s:e]))
        _, k, _ = tr.run(r['raw'])
        nev += k
    dt = time.perf_counter() - t0
    assert (b - a) % N == 0
    return b - a, dt, nev


def c1_timing(cpu):
    """Config 1: 64 ch, N = 128, 2^16 samples at 512 MS/s through the numpy replay (one core)."""
    _single_thread_env()
    _pin(cpu)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import numpy as np
    import signals
    from oracle import trigger
    case = signals.make_case(64, 1 << 16, seed=1000, noise=30.0, pulses_per_ch=1.0)
    o = signals.oracle_chain(case)
    reps, t0 = 0, time.perf_counter()
    nev = 0
    while time.perf_counter() - t0 < 2.0 or reps < 3:
        o.reset()
        r = o.process(case.iq)
        _, nev, _ = trigger.Trigger(64, case.fir12, np.full(64, -300)).run(r['raw'])
        reps += 1
    dt = (time.perf_counter() - t0) / reps
    return dict(value=round((1 << 16) / dt / 1e6, 3), unit='MSample/s', cores=1,
                sample='config 1: 64 ch, 2^16 samples, %d packets, %d reps' % (nev, reps))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--input', required=True, help='.npy int16 [S][2] sample of the GPU input')
    ap.add_argument('--cfg', required=True, help='.npz channel configuration')
    ap.add_argument('--one-core-samples', type=int, required=True)
    ap.add_argument('--workers', type=int, default=0, help='0: min(16, usable CPUs)')
    ap.add_argument('--all-core-samples', type=int, required=True)
    a = ap.parse_args()
    import numpy as np
    cfg = _load_cfg(a.cfg)
    C = int(cfg['C'])
    N = 2 * C
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else list(range(os.cpu_count()))
    out = dict(cpu_model=cpu_model(), os_cpu_count=os.cpu_count(), sched_affinity=len(aff))
    prefix = (16 + 520) * N   # >= (2T-1+24) hops of ADC history + 520 trigger warm-up rows

    # (i) one core, one process
    n1 = a.one_core_samples - a.one_core_samples % N
    s, dt, nev = run_chunk((aff[0], a.input, a.cfg, 0, n1, 0))
    out['one_core'] = dict(value=round(s / dt / 1e6, 3), unit='MSample/s', cores=1,
                           sample='first %d samples of the GPU input, %.1f s, %d packets' % (s, dt, nev))

    # (ii) all cores: W pinned single-thread processes, chunk-parallel with a warm-up prefix
    W = a.workers or min(16, len(aff))
    W = max(1, min(W, len(aff)))
    n = a.all_core_samples - a.all_core_samples % (N * W)
    per = n // W
    jobs = [(aff[i], a.input, a.cfg, i * per, (i + 1) * per, prefix) for i in range(W)]
    import multiprocessing as mp
    ctx = mp.get_context('fork')   # this process never touched the GPU
    t0 = time.perf_counter()
    with ctx.Pool(W) as pool:
        res = pool.map(run_chunk, jobs)
    wall = time.perf_counter() - t0
    tot = sum(r[0] for r in res)
    out['all_cores'] = dict(value=round(tot / wall / 1e6, 3), unit='MSample/s', cores=W,
                            sample='%d samples of the GPU input in %d chunks (+%d-sample warm-up prefix '
                                   'each), %.1f s wall, %d packets' % (tot, W, prefix, wall,
                                                                       sum(r[2] for r in res)))
    out['c1'] = c1_timing(aff[0])
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
