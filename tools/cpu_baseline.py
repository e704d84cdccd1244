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
# witness bars (tests/test_gpu_parity.py IQ_TOL_REL / PHASE_TOL): the absolute IQ bar below the floor
# and the IQ floor |y - c| >= IQ_FLOOR |y|max above which the 1e-5 rad phase bar holds
IQ_TOL = 1e-7
IQ_FLOOR = 0.01          # = IQ_TOL / 1e-5


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


def _trigger(trigger, cfg):
    """The oracle trigger in the bench step's baseline mode (EMA 1 / SVF 2, register constants
    of set_alpha.py / set_svf.py / set_base_thresh.py)."""
    mode = int(cfg['mode']) if 'mode' in cfg else 1
    q8 = int(cfg['rearm_q8']) if 'rearm_q8' in cfg else 0
    return trigger.Trigger(int(cfg['C']), cfg['fir'], cfg['thr'], mode=mode, rearm_q8=q8)


def run_chunk(args, collect=None):
    """Worker: process samples [a, b) of the shared input with a warm-up prefix; returns
    (samples counted, seconds, packets). `collect` (a dict) receives the per-block oracle
    outputs (phase float64, raw int16, packets) — list appends of arrays the chain produces
    anyway, so the timing is unchanged."""
    cpu, inp, cfgp, a, b, prefix, blk = args
    _single_thread_env()
    _pin(cpu)
    sys.path.insert(0, ROOT)
    import numpy as np
    from oracle import chain, trigger
    cfg = _load_cfg(cfgp)
    C = int(cfg['C'])
    N = 2 * C
    iq = np.load(inp, mmap_mode='r')
    o = chain.OracleChain(C, cfg['pfb'], cfg['bins'], cfg['lut_i'], cfg['lut_q'], cfg['lpf'],
                          cfg.get('ic'), cfg.get('qc'))
    tr = _trigger(trigger, cfg)
    p0 = max(0, a - prefix)
    t0 = time.perf_counter()
    # warm-up prefix: history of the chain and of the trigger (outputs discarded)
    nev = 0
    if a > p0:
        r = o.process(np.asarray(iq[p0:a]))
        tr.run(r['raw'])
    for s in range(a, b, blk):
        e = min(b, s + blk)
        r = o.process(np.asarray(iq[s:e]))
        ev, k, _ = tr.run(r['raw'])
        nev += k
        if collect is not None:
            cen = o.ic[None, :] + 1j * o.qc[None, :]
            collect.setdefault('ymc', []).append(np.abs(r['y'] - cen).astype(np.float32))
            collect.setdefault('ymed', []).append(np.median(np.abs(r['y']), axis=0))
            collect.setdefault('phase', []).append(r['phase'])
            collect.setdefault('raw', []).append(r['raw'])
            collect.setdefault('packets', []).append(ev)
    dt = time.perf_counter() - t0
    assert (b - a) % N == 0
    return b - a, dt, nev


def cpu_quota_cores():
    """CPUs this process may use per the cgroup CPU quota (cgroup v2 cpu.max / v1 cfs), or None
    when unlimited: sched_getaffinity can list every CPU of the machine while the container's
    share is much smaller."""
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, per = f.read().split()[:2]
        if q != 'max':
            return float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        with open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us') as f:
            q = int(f.read())
        with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as f:
            per = int(f.read())
        if q > 0:
            return q / per
    except (OSError, ValueError):
        pass
    return None


def witness_compare(col, witp, cfg):
    """Full-size parity witness (bench.py `parity`): the oracle outputs of the one-core leg
    against the device's outputs for the same samples. Bars (tests/test_gpu_parity.py,
    north_star): phase within 1e-5 rad; Fix16_13 phase within 1 LSB (rounding-boundary flips);
    packets bit-exact when the oracle trigger runs on the device's own Fix16_13 phase; full-chain
    packets equal on every channel without a flip; (config 5) heights within 1e-5 relative of the
    float64 oracle on the device's own phase and packets."""
    import numpy as np
    from oracle import trigger
    w = np.load(witp, allow_pickle=False)
    dph, draw, dpk = w['phase'], w['raw'], w['packets']
    oph = np.concatenate(col['phase'])
    oraw = np.concatenate(col['raw'])
    opk = np.concatenate(col['packets']) if col['packets'] else np.zeros(0, np.uint64)
    C = int(cfg['C'])
    assert dph.shape == oph.shape == draw.shape, (dph.shape, oph.shape, draw.shape)
    err = np.abs((dph.astype(np.float64) - oph + np.pi) % (2 * np.pi) - np.pi)
    # the bars of tests/test_gpu_parity.py: 1e-5 rad at every sample above the IQ floor
    # |y - c| >= IQ_FLOOR |y|max; below it the absolute IQ bar |dphi| |y - c| <= IQ_TOL |y|max
    ymc = np.concatenate(col['ymc']).astype(np.float64)
    settle = 16
    ymax = float(np.max(np.median(np.stack(col['ymed']), axis=0)))   # |y|max: the strongest tone
    held = ymc >= IQ_FLOOR * ymax
    low = ~held & (err >= 1e-5)
    iq_rel = float((err * ymc)[low].max() / ymax) if low.any() and ymax > 0 else 0.0
    # tone channels only (the others carry no tone: their |y - c| is noise)
    tones = np.asarray(cfg['tone_mask'], bool) if 'tone_mask' in cfg else np.ones(C, bool)
    held_t, err_t = held[:, tones], err[:, tones]
    below_t = ~held_t[settle:]
    dr = draw.astype(np.int32) - oraw.astype(np.int32)
    flips = dr != 0
    own = _trigger(trigger, cfg).run(draw)[0]
    own_equal = np.array_equal(np.sort(own), np.sort(dpk))
    ch_of = lambda p: ((p >> np.uint64(52)) & np.uint64(0xFFF)).astype(np.int64)
    dset = [set() for _ in range(C)]
    oset = [set() for _ in range(C)]
    for p, c in zip(dpk.tolist(), ch_of(dpk).tolist()):
        dset[c].add(p)
    for p, c in zip(opk.tolist(), ch_of(opk).tolist()):
        oset[c].add(p)
    diverged = [c for c in range(C) if dset[c] != oset[c]]
    flip_ch = set(np.nonzero(flips.any(axis=0))[0].tolist())
    unexplained = [c for c in diverged if c not in flip_ch]
    out = dict(samples=int(dph.shape[0] * 2 * C), rows=int(dph.shape[0]), channels=C,
               phase_max_err_rad=float(err[held].max()),
               phase_max_err_all_rows_rad=float(err.max()),
               phase_max_err_settled_rad=float(err[settle:].max()) if err.shape[0] > settle else None,
               phase_p999999_err_rad=float(np.quantile(err, 0.999999)),
               phase_tol_rad=1e-5, iq_err_below_floor_max_rel=iq_rel, iq_tol_rel=IQ_TOL,
               iq_floor_rel=IQ_FLOOR, samples_below_floor=int((~held).sum()), settle_rows=settle,
               settled_max_err_above_floor=float(err_t[settle:][held_t[settle:]].max())
               if held_t[settle:].any() else None,
               settled_tone_samples_below_floor_frac=float(below_t.mean()) if below_t.size else 0.0,
               channels_below_floor=int(below_t.any(axis=0).sum()),
               channels_mostly_below_floor=int((below_t.mean(axis=0) > 0.5).sum()) if below_t.size else 0,
               raw_flip_rate=float(flips.mean()), raw_max_abs_diff=int(np.abs(dr).max()),
               channels_with_flip=len(flip_ch),
               packets_device=int(dpk.size), packets_oracle_chain=int(opk.size),
               packets_equal_on_device_raw=bool(own_equal),
               channels_diverged_full_chain=len(diverged),
               channels_diverged_without_flip=len(unexplained))
    if 'attens' in cfg:
        # per-channel tone amplitude / loop columns: max phase error of the channels in each
        # attenuation band and each loop radius / |centre| band
        errc = err.max(axis=0)
        att = np.asarray(cfg['attens'], np.float64)
        R = np.asarray(cfg['loop_R'], np.float64)
        ratio = np.where(R < 1.0, R / np.maximum(1.0 - R, 1e-12), np.inf)
        out['by_atten_db'] = [dict(atten_db=[lo, hi], channels=int(m.sum()),
                                   max_err_rad=float(errc[m].max()) if m.any() else None)
                              for lo, hi in ((0, 5), (5, 10), (10, 15), (15, 20.001))
                              for m in [(att >= lo) & (att < hi)]]
        out['by_loop_ratio'] = [dict(ratio=[lo, hi], channels=int(m.sum()),
                                     max_err_rad=float(errc[m].max()) if m.any() else None)
                                for lo, hi in ((0.0, 0.3), (0.3, 1.0), (1.0, 10.0), (10.0, np.inf))
                                for m in [(ratio >= lo) & (ratio < hi) if np.isfinite(hi) else ratio >= lo]]
        out['by_loop_ratio'][-1]['ratio'] = [10.0, 'inf (centre at the origin)']
    green = (out['phase_max_err_rad'] <= 1e-5 and iq_rel <= IQ_TOL and out['raw_max_abs_diff'] <= 1
             and own_equal and not unexplained)
    if 'heights' in w.files:
        sys.path.insert(0, ROOT)
        from oracle import heights as oh
        ref = oh.pulse_heights(dph, dpk, w['coeff'], int(w['pre']), 0)
        got = w['heights'].astype(np.float64)
        nan_eq = bool(np.array_equal(np.isnan(ref), np.isnan(got)))
        ok = ~np.isnan(ref)
        rel = np.abs(got[ok] - ref[ok]) / np.maximum(np.abs(ref[ok]), 1e-3) if ok.any() else np.zeros(1)
        end2end = oh.pulse_heights(oph, dpk, w['coeff'], int(w['pre']), 0)
        e2e = np.abs(got[ok] - end2end[ok]) / np.maximum(np.abs(end2end[ok]), 1e-3) if ok.any() else np.zeros(1)
        out['heights'] = dict(n=int(got.size), nan_positions_equal=nan_eq, max_rel_err=float(rel.max()),
                              tol_rel=1e-5, max_rel_err_vs_oracle_phase=float(e2e.max()))
        green = green and nan_eq and out['heights']['max_rel_err'] <= 1e-5
    out['green'] = bool(green)
    return out


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
    ap.add_argument('--workers', type=int, default=0,
                    help='0: every usable CPU (sched_getaffinity), capped at the cgroup CPU quota')
    ap.add_argument('--all-core-samples', type=int, required=True)
    ap.add_argument('--witness', default=None, help='.npz device outputs for the one-core sample')
    ap.add_argument('--witness-only', action='store_true',
                    help='N > 1 per-rank witness: only the oracle run + comparison of the one-core sample')
    ap.add_argument('--cpu', type=int, default=0, help='--witness-only: index of the usable CPU to pin')
    ap.add_argument('--curve', default=None,
                    help='comma-separated worker counts: time only the chunk-parallel leg at each (the '
                         'cgroup cap is not applied), e.g. 4,8,16,32,64,256, and print one JSON line')
    a = ap.parse_args()
    import numpy as np
    cfg = _load_cfg(a.cfg)
    C = int(cfg['C'])
    N = 2 * C
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else list(range(os.cpu_count()))
    quota = cpu_quota_cores()
    out = dict(cpu_model=cpu_model(), os_cpu_count=os.cpu_count(), sched_affinity=len(aff),
               cpu_quota_cores=quota)
    if a.curve:
        import multiprocessing as mp
        prefix = (16 + 520) * N
        pts = []
        for W in [int(x) for x in a.curve.split(',')]:
            W = max(1, min(W, len(aff)))
            n = a.all_core_samples - a.all_core_samples % (N * W)
            per = n // W
            blk = max(N, min(1 << 22, per) // N * N)
            jobs = [(aff[i], a.input, a.cfg, i * per, (i + 1) * per, prefix, blk) for i in range(W)]
            t0 = time.perf_counter()
            with mp.get_context('fork').Pool(W) as pool:
                res = pool.map(run_chunk, jobs)
            wall = time.perf_counter() - t0
            pts.append(dict(workers=W, value=round(sum(r[0] for r in res) / wall / 1e6, 3), wall_s=round(wall, 2),
                            samples=int(sum(r[0] for r in res))))
        out['curve'] = pts
        print(json.dumps(out), flush=True)
        return
    # >= (2T-1+24) hops of ADC history + 520 trigger warm-up rows (the EMA baseline's merge
    # horizon). The SVF baseline needs ~10^5 rows to merge exactly; its chunks use
    # the same prefix, so their first rows' packets are approximate (a timing baseline only).
    prefix = (16 + 520) * N

    if a.witness_only:
        n1 = a.one_core_samples - a.one_core_samples % N
        col = {}
        run_chunk((aff[a.cpu % len(aff)], a.input, a.cfg, 0, n1, 0, 1 << 22), collect=col)
        out['parity'] = witness_compare(col, a.witness, cfg)
        print(json.dumps(out), flush=True)
        return
    # (i) one core, one process
    n1 = a.one_core_samples - a.one_core_samples % N
    col = {} if a.witness else None
    s, dt, nev = run_chunk((aff[0], a.input, a.cfg, 0, n1, 0, 1 << 22), collect=col)
    out['one_core'] = dict(value=round(s / dt / 1e6, 3), unit='MSample/s', cores=1,
                           sample='first %d samples of the GPU input, %.1f s, %d packets' % (s, dt, nev))
    if col is not None:
        out['parity'] = witness_compare(col, a.witness, cfg)
        del col

    # (ii) all cores: W pinned single-thread processes (one per usable CPU, at most the cgroup
    #      quota: processes beyond it only time-share), chunk-parallel with a warm-up prefix
    W = a.workers or len(aff)
    if quota is not None:
        W = min(W, max(1, int(quota)))
    W = max(1, min(W, len(aff)))
    n = a.all_core_samples - a.all_core_samples % (N * W)
    per = n // W
    blk = max(N, min(1 << 22, per) // N * N)
    jobs = [(aff[i], a.input, a.cfg, i * per, (i + 1) * per, prefix, blk) for i in range(W)]
    import multiprocessing as mp
    ctx = mp.get_context('fork')   # this process never touched the GPU
    t0 = time.perf_counter()
    with ctx.Pool(W) as pool:
        res = pool.map(run_chunk, jobs)
    wall = time.perf_counter() - t0
    tot = sum(r[0] for r in res)
    out['all_cores'] = dict(value=round(tot / wall / 1e6, 3), unit='MSample/s', cores=W,
                            cores_note='one pinned single-thread process per usable CPU '
                                       '(sched_getaffinity %d, cgroup quota %s)' % (len(aff), quota),
                            sample='%d samples of the GPU input in %d chunks (+%d-sample warm-up prefix '
                                   'each, not counted), %.1f s wall, %d packets' % (tot, W, prefix, wall,
                                                                                   sum(r[2] for r in res)))
    out['c1'] = c1_timing(aff[0])
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
