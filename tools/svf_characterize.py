#!/usr/bin/env python3
"""Why the SVF baseline emits packets that match no injected pulse, on the
oracle (CPU, bit-exact with the device trigger): one synthetic Fix16_13 phase stream — white noise
(sigma 300 raw, the bench stream's level) plus Poisson photon pulses -A (1 - e^{-t/0.1}) e^{-t/65}
(pulses.py:470-472), A ~ U(20, 100) deg, 1 per 2048 rows per channel — through the same trigger in
EMA (set_alpha.py) and SVF (set_svf.py) mode with thresholds by the reference's loadThresholds rule
on a quiet block. Every packet is matched to the last pulse of its channel that started at or
before it (bench.py's window: -2 .. +60 rows); the unmatched ones are histogrammed by their delay
after that pulse and by the pulse's amplitude, and the baseline e = f - B at the packet is kept.

    python tools/svf_characterize.py [--rows 400000] [--channels 64] > profiles/r03/r03_svf_unmatched.json
    python tools/svf_characterize.py --rearm 0,64,128,192,256   # re-arm hysteresis (mkid_set_rearm)

Round 5 adds the re-arm level (hysteresis, mkid_set_rearm): each (mode, rearm_q8) pair reports the
unmatched packets per pulse and the pulses that got no packet at all (missed), so the price of the
later re-arm (a pulse on the previous pulse's tail) is measured beside its benefit.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def synth(C, J, seed, rate):
    rng = np.random.default_rng(seed)
    ph = rng.normal(0.0, 300.0, (J, C))
    t = np.arange(600, dtype=np.float64)
    shape = (1 - np.exp(-t / 0.1)) * np.exp(-t / 65.0)
    pulses = []
    for c in range(C):
        k = rng.poisson(rate * J)
        for s0, a in zip(np.sort(rng.integers(2000, J - 600, k)), rng.uniform(20, 100, k)):
            ph[s0:s0 + 600, c] -= np.deg2rad(a) * 8192 * shape
            pulses.append((int(s0), c, float(a)))
    return np.clip(np.rint(ph), -25736, 25736).astype(np.int16), pulses


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rows', type=int, default=400000)
    ap.add_argument('--channels', type=int, default=64)
    ap.add_argument('--rate', type=float, default=1.0 / 2048)
    ap.add_argument('--rearm', default='0', help='comma-separated re-arm fractions (/256) to evaluate')
    a = ap.parse_args()
    from oracle import trigger
    from mkids_sdr_amd import codecs
    C, J = a.channels, a.rows
    raw, pulses = synth(C, J, 7, a.rate)
    quiet, _ = synth(C, 20480, 8, 0.0)
    thr = np.array([codecs.threshold_from_phase(quiet[:, c])[0] for c in range(C)], np.int32)
    mf = codecs.fir_quantise(np.loadtxt(os.path.join(ROOT, 'tests', 'golden', 'fir', 'matched_30us.txt')))
    taps = np.tile(mf, (C, 1))
    byc = {}
    for s0, c, amp in pulses:
        byc.setdefault(c, []).append((s0, amp))
    out = dict(rows=J, channels=C, pulses=len(pulses), sigma_raw=300, thresholds_median=int(np.median(thr)))
    runs = [(('ema' if mode == 1 else 'svf') + ('' if q == 0 else '_rearm%d' % q), mode, q)
            for q in [int(v) for v in a.rearm.split(',')] for mode in (1, 2)]
    for name, mode, q8 in runs:
        ev = trigger.Trigger(C, taps, thr, mode=mode, rearm_q8=q8).run(raw)[0]
        u = codecs.unpack_wide(ev)
        ch = np.asarray(u['ch'] if isinstance(u, dict) else u[0])
        ts = np.asarray(u['ts'] if isinstance(u, dict) else u[3]).astype(np.int64)
        base = np.asarray(u['base'] if isinstance(u, dict) else u[2])
        delays, amps, unmatched, matched = [], [], 0, 0
        nop = 0
        hit = set()
        for c_, t_ in zip(ch.tolist(), ts.tolist()):
            ps = byc.get(c_, [])
            starts = np.array([p[0] for p in ps]) if ps else np.zeros(0, np.int64)
            k = np.searchsorted(starts, t_ + 2, side='right') - 1
            if k < 0:
                nop += 1
                unmatched += 1
                continue
            d = t_ - int(starts[k])
            if -2 <= d <= 60:
                matched += 1
                hit.add((c_, int(starts[k])))
            else:
                unmatched += 1
                delays.append(d)
                amps.append(ps[k][1])
        delays = np.asarray(delays)
        amps = np.asarray(amps)
        rec = dict(rearm_q8=q8, packets=int(len(ev)), matched=matched, unmatched=unmatched,
                   unmatched_before_any_pulse=nop,
                   unmatched_per_pulse=round(unmatched / max(1, len(pulses)), 4),
                   pulses_missed=int(len(pulses) - len(hit)),
                   missed_per_pulse=round((len(pulses) - len(hit)) / max(1, len(pulses)), 4))
        if len(delays):
            edges = [61, 100, 150, 200, 300, 400, 600, 1000, 2000, 10 ** 9]
            h = np.histogram(delays, bins=edges)[0]
            rec['unmatched_delay_rows_hist'] = {'%d-%d' % (edges[i], edges[i + 1] - 1): int(h[i])
                                               for i in range(len(h))}
            rec['unmatched_delay_median'] = float(np.median(delays))
            rec['unmatched_pulse_amp_deg_median'] = float(np.median(amps))
            # where the pulse tail A e^{-t/65} (filtered) crosses the threshold: ~65 ln(A / |thr|)
            tcross = 65.0 * np.log(np.deg2rad(amps) * 8192 / abs(float(np.median(thr))))
            rec['unmatched_minus_tail_crossing_rows_median'] = float(np.median(delays - tcross))
        out[name] = rec
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
