"""The trigger as a photon detector, scored against injected truth (signals.match_pulses).

Thresholds are set the reference's way — loadThresholds (ROACH_Pulses.py:211-299) on a snapshot
of the running, loop-rotated stream (rotateLoopsReady, ROACH_Setup.py:645-667) — and pulses
follow the reference's synthetic shape (pulses.py:470-472) at the amplitudes of
FakeObservation (pulses.py:172). Bars: >= 95 % of isolated pulses give exactly one packet; packets
that match no pulse (noise, start-up) stay below 5 % of the pulses; no packet inside the
start-of-stream hold-off (trig_common.h kHoldOff, oracle/trigger.c HOLDOFF).
"""
import numpy as np
import pytest

import signals
from oracle import trigger as otrig

HOLDOFF = 64


def _rotated_oracle_raw(case_fn, C, S, seed, noise, ppc):
    """Oracle chain with the loops rotated to phase 0 (DDS phase = arctan2 of the average IQ)."""
    quiet = case_fn(C, S // 2, seed=seed, noise=noise, pulses_per_ch=0)
    y = signals.oracle_chain(quiet).process(quiet.iq)['y']
    phi = np.angle(y[HOLDOFF:].mean(axis=0))
    quiet = case_fn(C, S // 2, seed=seed, noise=noise, pulses_per_ch=0, dds_phase=phi)
    o = signals.oracle_chain(quiet)
    o.process(quiet.iq)                      # first pass: filters settle
    rq = o.process(quiet.iq)['raw']          # snapshot of the running stream
    thr = signals.thresholds_from_quiet(quiet, rq)
    case = case_fn(C, S, seed=seed, noise=noise, pulses_per_ch=ppc, dds_phase=phi)
    return case, thr, signals.oracle_chain(case).process(case.iq)['raw']


def test_oracle_detector_against_truth():
    C, S = 64, 1 << 20
    case, thr, raw = _rotated_oracle_raw(signals.make_case, C, S, seed=11, noise=232.0, ppc=6.0)
    assert np.all(thr < 0) and np.all(thr > -2000), thr
    ev, n, _ = otrig.Trigger(C, case.fir12, thr).run(raw)
    m = signals.match_pulses(ev, case.pulses, case.N)
    ts = (np.asarray(ev, np.uint64) & np.uint64((1 << 28) - 1)).astype(np.int64)
    assert ts.min() >= HOLDOFF - 1                       # nothing fires during the hold-off
    assert m['isolated'] > 50
    assert m['exactly_one'] >= 0.95 * m['isolated'], m
    assert m['extra'] <= 0.05 * m['pulses'] + 2, m


@pytest.mark.gpu
def test_gpu_detector_against_truth(gpu):
    """The device chain end to end (k_front + k_trigger), thresholds from the device's own
    phase snapshot of the running rotated stream."""
    from mkids_sdr_amd.channelizer import Channelizer
    from mkids_sdr_amd import codecs
    C, S, seed, noise = 256, 1 << 23, 21, 232.0
    quiet = signals.make_case(C, S // 4, seed=seed, noise=noise, pulses_per_ch=0)
    ch = Channelizer(C, max_chunk=S)
    try:
        ch.set_bins(quiet.bins)
        ch.set_dds(quiet.lut_i, quiet.lut_q)
        ch.set_lpf(quiet.lpf12)
        ch.set_fir(quiet.fir12)
        ch.set_accumulator(True)
        ch.process(quiet.iq, want_phase=False)
        mi, mq = ch.avg_iq()
        ch.set_accumulator(False)
        phi = np.arctan2(mq, mi)
        quiet = signals.make_case(C, S // 4, seed=seed, noise=noise, pulses_per_ch=0, dds_phase=phi)
        ch.set_dds(quiet.lut_i, quiet.lut_q)
        ch.reset()
        ch.process(quiet.iq, want_phase=False)
        ch.process(quiet.iq, want_phase=False)
        thr = codecs.thresholds_from_phase_block(ch.raw_phase())
        assert np.all(thr < 0) and np.all(thr > -2000), thr
        case = signals.make_case(C, S, seed=seed, noise=noise, pulses_per_ch=12.0, dds_phase=phi)
        ch.set_thresholds(thr)
        ch.reset()
        _, ev = ch.process(case.iq, want_phase=False)
    finally:
        ch.close()
    m = signals.match_pulses(ev, case.pulses, case.N)
    ts = (np.asarray(ev, np.uint64) & np.uint64((1 << 28) - 1)).astype(np.int64)
    assert ts.min() >= HOLDOFF - 1
    assert m['isolated'] > 1000, m
    assert m['exactly_one'] >= 0.95 * m['isolated'], m
    assert m['extra'] <= 0.05 * m['pulses'], m
    assert 0.95 <= m['packets'] / m['pulses'] <= 1.05, m
