"""GPU parity under the reference's operating conditions: unequal per-resonator attenuation and
off-origin IQ loop centres.

The reference drives each resonator at its own attenuation — tone amplitudes 10^((atten_min - a)/20)
(define_DAC_LUT, ROACH_Setup.py:499-502) inside one full-scale comb — and measures phase about the
loop centre it loaded (loadIQcenters, ROACH_Setup.py:595-617; the host replay's
atan2(Q - Qc, I - Ic), pulse_triggering_IQ.py:152) after rotating each loop (rotateLoopsReady,
:645-667). signals.make_case reproduces that flow (per-tone attenuation, RESDIFF-style loops of
radius R about a centre at 1 - R, DDS rotation, centres from the average IQ). Each case spreads its
channels over an attenuation span (uniform in [0, span] dB) and over loop radius / |centre| ratios
log-uniform in [0.1, 10] (a fifth of the channels centred at the origin).

Bars: the same as tests/test_gpu_parity.py `compare`: phase within 1e-5 rad at every tone-channel
sample whose |y - c| is at least the IQ floor F = IQ_TOL_REL / 1e-5 * |y|max = 0.01 |y|max (|y|max:
the strongest tone); below F, where the phase of y - c is ill-conditioned in any precision (the
stream's start-up rows, where y passes through the loop centre, and noise on the smallest loops),
the absolute IQ bar |dphi| |y - c| <= IQ_TOL_REL |y|max = 1e-7 |y|max instead. Fix16_13 within 1
LSB, packets bit-exact on the device's own phase, full-chain packets equal except downstream of a
rounding flip. Each case also asserts that at most 1 % of the settled tone samples fall below F
(the share of the operating range the phase bar does not hold).
"""
import json
import os

import numpy as np
import pytest

import signals
import test_gpu_parity as tp

pytestmark = pytest.mark.gpu


def operating_case(C, S, span, seed, pulses_per_ch):
    rng = np.random.default_rng(1000 + seed)
    att = rng.uniform(0.0, span, C)
    ratio = np.exp(rng.uniform(np.log(0.1), np.log(10.0), C))
    ratio[rng.random(C) < 0.2] = np.inf
    kw = dict(seed=seed, atten_db=att, loop_ratio=ratio)
    # 100-row pulse windows (the tail is at e^-1.5 there): the per-sample synthesis of 390-row
    # windows dominates the suite's time at 2048 channels
    case = signals.make_case(C, S, pulses_per_ch=pulses_per_ch, window_phase=100, **kw)
    quiet = signals.make_case(C, min(S, 2 * C * 2048), pulses_per_ch=0, **kw)
    thr = signals.thresholds_from_quiet(quiet, signals.oracle_chain(quiet).process(quiet.iq)['raw'])
    case.ratio = ratio
    return case, thr


def _write_report(name, case, rep):
    d = os.environ.get('MKID_PARITY_REPORT')
    if not d:
        return
    os.makedirs(d, exist_ok=True)
    e, ymc, ymax = rep['err_rows'], rep['ymc'], rep['ymax']
    st = tp.SETTLE_ROWS
    with open(os.path.join(d, name + '.json'), 'w') as f:
        json.dump({'C': case.C, 'rows': int(rep['rows']), 'ymax': ymax, 'amp': case.amps.tolist(),
                   'loop_R': case.loop_R.tolist(), 'radius_rel': (case.loop_radius / ymax).tolist(),
                   'err': np.asarray(rep['err']).tolist(), 'flips': np.asarray(rep['flips']).tolist(),
                   'err_settled': e[st:].max(axis=0).tolist(), 'argmax_row': e.argmax(axis=0).tolist(),
                   'ymc_min': ymc.min(axis=0).tolist(), 'ymc_min_settled': ymc[st:].min(axis=0).tolist(),
                   'abs_iq_err': (e * ymc).max(axis=0).tolist(),
                   'abs_iq_err_settled': (e[st:] * ymc[st:]).max(axis=0).tolist()}, f)


@pytest.mark.parametrize('C,S,span,seed,splits,acc', [
    (256, 2 ** 18, 10.0, 61, [0, 2 ** 17 + 512, 2 ** 18], True),
    (256, 2 ** 18, 20.0, 62, None, True),
    (1024, 2 ** 20, 10.0, 63, [0, 2 ** 19, 2 ** 20], True),
    (1024, 2 ** 20, 20.0, 64, None, False),
    (1024, 2 ** 22, 20.0, 66, [0, 2 ** 21, 2 ** 22], False),      # 2048 rows per channel
    (2048, 2 ** 20, 20.0, 65, [0, 3 * 2 ** 17 + 4096, 2 ** 20], True),
    (2048, 2 ** 22, 20.0, 67, [0, 2 ** 21, 2 ** 22], False),      # k_front5<false>, 1024 rows
])
def test_operating_conditions(gpu, C, S, span, seed, splits, acc):
    case, thr = operating_case(C, S, span, seed, max(0.5, S / (2 * C) / 400))
    rep = {}
    try:
        tp.compare(case, thr, splits or [0, S], report=rep, acc=acc)
    finally:
        if rep:
            _write_report('operating_C%d_span%d_S%d' % (C, int(span), S), case, rep)
    st = tp.SETTLE_ROWS
    below = rep['ymc'][st:] < tp.IQ_TOL_REL / tp.PHASE_TOL * rep['ymax']
    assert below.mean() <= 0.01, '%.3g of the settled tone samples below the IQ floor' % below.mean()


@pytest.mark.parametrize('C,S,seed', [(1024, 2 ** 20, 68), (2048, 2 ** 20, 69)])
def test_accumulator_leaves_outputs_bit_identical(gpu, C, S, seed):
    """The accumulating front-end variants (k_front5<true>, k_front3 with y-sum stores) and the
    streaming ones produce bit-identical phase and packets."""
    case, thr = operating_case(C, S, 20.0, seed, 1.0)
    splits = [0, S // 2, S]
    ph_a, ev_a, means = tp.run_gpu(case, thr, splits, acc=True)
    ph_s, ev_s, _ = tp.run_gpu(case, thr, splits, acc=False)
    assert means is not None
    assert np.array_equal(ph_a.view(np.uint32), ph_s.view(np.uint32))
    assert np.array_equal(tp.sort_events(ev_a), tp.sort_events(ev_s))


def test_small_dc_gain_low_pass(gpu):
    """Low-pass taps with a DC gain |G| < 0.25 (here the default taps >> 3, G ~ 1/8) switch the
    centred low-pass off (c' = 0, r = -c: c / G would scale the accumulation's rounding by 1 / G,
    ADVICE r05); the chain still meets the phase bars against the oracle run with the same taps and
    the centres scaled with the gain."""
    C, S = 256, 2 ** 18
    case, thr = operating_case(C, S, 20.0, 70, 2.0)
    g0 = case.lpf12.sum()
    case.lpf12 = np.trunc(case.lpf12 / 8).astype(np.int64)
    rho = case.lpf12.sum() / g0
    assert abs(case.lpf12.sum() / 2048) < 0.25
    case.ic = (case.ic * rho).astype(np.float32)
    case.qc = (case.qc * rho).astype(np.float32)
    quiet = signals.oracle_chain(case).process(case.iq[:2 * C * 2048])['raw']
    thr = signals.thresholds_from_quiet(case, quiet)
    tp.compare(case, thr, [0, S // 2, S], expect_events=False)
