"""Seeded synthetic MKID feedline cases for the parity tests (test infrastructure).

A case is the reference's own setup path driven end to end: tones one per channel at a coarse bin
plus a residual that is a multiple of fs/2^16 (ROACH_Setup.py:83-84, 534-550); DDS LUTs from
freqCombLUT('no', ...) per channel (ROACH_Setup.py:523-530); the DAC comb from freqCombLUT('yes',
...) with seed-1000 random phases (ROACH_Setup.py:426-429), mirrored as define_DAC_LUT does
(:485-495) and conjugated back by the loop-back. Photon pulses are injected as phase
modulation of one tone, -A (1-e^{-t/tr}) e^{-t/tf} (ReadoutControls/lib/pulses.py:470-472), plus
AWGN; the ADC stream is truncated to int16 like int() in freqCombLUT.
"""
import numpy as np

from oracle import chain, setup_ref

FS = 512e6
LUT_LEN = 2 ** 16


class Case:
    pass


def make_case(C, n_samples, fs=FS, n_tones=None, seed=0, noise=30.0, pulses_per_ch=0.0,
              amp_deg=(20.0, 100.0), tau_rise=0.1, tau_fall=65.0, window_phase=390,
              pulse_margin=64, dds_phase=None, atten_db=None, loop_ratio=None):
    """Return a Case with .iq int16 [S][2] and every configuration array both sides need.
    dds_phase [C] (rad): per-channel DDS LUT phase, e.g. rotateLoopsReady's arctan2 of the
    average IQ (ROACH_Setup.py:645-667); the tones and noise do not depend on it.

    atten_db [n_tones]: per-resonator attenuation (dB); tone amplitudes 10^((min - a)/20), the
    rule of define_DAC_LUT (ROACH_Setup.py:499-502), then the comb is scaled to full scale as
    freqCombLUT does (:451-461), so the strongest tone keeps the comb's level.

    loop_ratio [n_tones] (or scalar): IQ-loop radius / |loop centre|. Each tone then passes a
    resonator loop (geometry of iqsweep.RESDIFF, iqsweep.py:824-858: a circle of radius R about an
    offset centre): at rest the tone sits at 1 (its DAC amplitude), the centre at 1 - R and a
    photon moves it along the circle, tone (1 - R + R e^{i delta}), R = ratio / (1 + ratio). The
    centres are then found and loaded the reference's way: the average IQ of a quiet,
    noise-free run (the avgIQ accumulator) rotates the DDS (rotateLoopsReady, ROACH_Setup.py:
    645-667) and ic + i qc = (1 - R) * the rotated rest IQ (findIQcenters / loadIQcenters,
    :595-625). None = centre at the origin (R = 1), the round-1 cases."""
    N = 2 * C
    res = fs / LUT_LEN
    upb = LUT_LEN // N                       # fs/2^16 units per coarse bin
    rng = np.random.default_rng(seed)
    n_tones = C if n_tones is None else n_tones
    if atten_db is None:
        gain = np.ones(n_tones)
    else:
        atten_db = np.asarray(atten_db, np.float64)
        gain = np.array([10 ** (+(atten_db.min() - a) / 20.) for a in atten_db])
    if loop_ratio is None:
        R = np.ones(n_tones)
    else:
        lr = np.broadcast_to(np.asarray(loop_ratio, np.float64), (n_tones,))
        R = np.ones(n_tones)
        fin = np.isfinite(lr)
        R[fin] = lr[fin] / (1.0 + lr[fin])
    bins = rng.permutation(np.arange(1, N))[:n_tones]
    m = rng.integers(-(upb // 4), upb // 4 + 1, n_tones) if upb >= 4 else np.zeros(n_tones, int)
    f_dds = [float((int(b) * upb + int(k)) * res) for b, k in zip(bins, m)]

    # DDS side, reference algorithm (channel m <- tone m; the rest get f=0, bin 0)
    freqs_dds = f_dds + [0.0] * (C - n_tones)
    sel_bins, resid = setup_ref.select_bins(freqs_dds, N, fs, LUT_LEN)
    lut_i = np.zeros((C, LUT_LEN // C), np.int64)
    lut_q = np.zeros((C, LUT_LEN // C), np.int64)
    for ch in range(C):
        ph0 = 0. if dds_phase is None else float(dds_phase[ch])
        I, Q, _, _ = setup_ref.freq_comb_lut('no', [resid[ch]], fs / N * 2, res, [1.], [ph0], 'no')
        lut_i[ch], lut_q[ch] = I, Q

    # DAC side: tone at -f_dds (mod fs), freqCombLUT('yes') with the reference's random phases
    freqs_dac = [(fs - f) % fs for f in f_dds]
    I_dac, Q_dac, sf, phases = setup_ref.freq_comb_lut('yes', freqs_dac, fs, res, list(gain))
    base = np.stack([I_dac, -Q_dac], axis=1).astype(np.float64)   # loop-back conjugation
    tone_amp = setup_ref.FULL_SCALE / sf
    reps = -(-n_samples // LUT_LEN)
    x = np.tile(base, (reps, 1))[:n_samples].copy()
    t = np.arange(n_samples, dtype=np.int64)
    if noise > 0:
        x += rng.normal(0.0, noise, x.shape)

    # pulses: Poisson count per tone channel, uniform start times (ADC samples)
    pulse_list = []
    if pulses_per_ch > 0:
        win = window_phase * N
        for ch in range(n_tones):
            k = rng.poisson(pulses_per_ch)
            lo, hi = pulse_margin * N, max(pulse_margin * N + 1, n_samples - win // 4)
            starts = np.sort(rng.integers(lo, hi, k))
            amps = np.deg2rad(rng.uniform(amp_deg[0], amp_deg[1], k))
            for s0, A in zip(starts, amps):
                pulse_list.append((int(s0), ch, float(A)))
                e = min(n_samples, s0 + win)
                tau = (t[s0:e] - s0).astype(np.float64)
                d = -A * (1 - np.exp(-tau / (tau_rise * N))) * np.exp(-tau / (tau_fall * N))
                th = 2 * np.pi * ((int(round(f_dds[ch] / res)) * t[s0:e]) % LUT_LEN) / LUT_LEN \
                    - phases[ch]
                z = tone_amp * gain[ch] * R[ch] * np.exp(1j * th) * (np.exp(1j * d) - 1)
                x[s0:e, 0] += z.real
                x[s0:e, 1] += z.imag
    iq = np.clip(np.trunc(x), -32768, 32767).astype(np.int16)

    c = Case()
    c.C, c.N, c.fs, c.n_tones = C, N, fs, n_tones
    c.iq = iq
    c.amps = np.zeros(C)
    c.amps[:n_tones] = gain
    c.loop_R = np.ones(C)
    c.loop_R[:n_tones] = R
    c.bins = np.array(sel_bins, np.int64) % N
    c.lut_i, c.lut_q = lut_i, lut_q
    c.pfb = chain.pfb_prototype(N)
    c.lpf12 = setup_ref.fir_quantise(np.loadtxt(_golden('fir/BlackmanFilter_250kHz.txt')))
    mf = setup_ref.fir_quantise(np.loadtxt(_golden('fir/matched_30us.txt')))
    c.fir12 = np.zeros((C, 26), np.int64)
    c.fir12[:n_tones] = mf
    c.ic = np.zeros(C, np.float32)
    c.qc = np.zeros(C, np.float32)
    c.thr = np.full(C, -(1 << 30), np.int64)
    c.tone_amp = tone_amp
    c.phases = phases
    c.f_dds = f_dds
    c.pulses = pulse_list
    c.resid = resid
    if loop_ratio is not None:
        _calibrate_loops(c, base, fs, res, dds_phase)
    return c


def _calibrate_loops(c, base, fs, res, dds_phase):
    """rotateLoopsReady + loadIQcenters on the noise-free, pulse-free comb (see make_case)."""
    C, N = c.C, c.N
    skip = 64                                 # rows of filter start-up
    reps = max(2, -(-(skip + 64) * N // LUT_LEN))
    quiet = np.clip(np.trunc(np.tile(base, (reps, 1))), -32768, 32767).astype(np.int16)
    y = oracle_chain(c).process(quiet)['y'][skip:].mean(axis=0)
    rot = np.angle(y) + (0. if dds_phase is None else np.asarray(dds_phase, np.float64))
    for ch in range(C):
        I, Q, _, _ = setup_ref.freq_comb_lut('no', [c.resid[ch]], fs / N * 2, res, [1.],
                                             [float(rot[ch])], 'no')
        c.lut_i[ch], c.lut_q[ch] = I, Q
    c.dds_phase = rot
    y_rot = oracle_chain(c).process(quiet)['y'][skip:].mean(axis=0)
    cen = (1.0 - c.loop_R) * y_rot
    c.ic = cen.real.astype(np.float32)
    c.qc = cen.imag.astype(np.float32)
    c.loop_radius = np.abs(y_rot) * c.loop_R  # |y - centre| at rest (y units)


def _golden(rel):
    import os
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', rel)


def oracle_chain(case):
    return chain.OracleChain(case.C, case.pfb, case.bins, case.lut_i, case.lut_q, case.lpf12,
                             case.ic, case.qc)


def thresholds_from_quiet(case, raw_quiet, nsigma=2.5):
    """loadThresholds (ROACH_Pulses.py:211-299) per channel on a pulse-free raw phase block."""
    thr = np.full(case.C, -(1 << 30), np.int64)
    for ch in range(case.n_tones):
        thr[ch], _ = setup_ref.threshold_from_phase(raw_quiet[:, ch], nsigma)
    return thr


def wrap(d):
    return (d + np.pi) % (2 * np.pi) - np.pi


def match_pulses(events, pulses, N, early=2, late=60, isolation=400):
    """Score wide packets against injected truth (start ADC sample, channel, amplitude).
    A packet of channel c stamped ts matches a pulse of c starting at phase row p when
    p - early <= ts <= p + late. Returns dict: isolated (pulses with no other pulse of their
    channel within `isolation` rows), exactly_one (isolated pulses with exactly one packet),
    missed, multi, extra (packets matching no pulse)."""
    ev = np.asarray(events, np.uint64)
    ch = ((ev >> np.uint64(52)) & np.uint64(0xFFF)).astype(np.int64)
    ts = (ev & np.uint64((1 << 28) - 1)).astype(np.int64)
    by_ch = {}
    for s0, c, _ in pulses:
        by_ch.setdefault(int(c), []).append(int(s0) // N)
    for c in by_ch:
        by_ch[c] = np.sort(np.array(by_ch[c]))
    hits = {}
    extra = 0
    for c, t in zip(ch, ts):
        p = by_ch.get(int(c))
        if p is None:
            extra += 1
            continue
        k = np.searchsorted(p, t + early, side='right') - 1
        if k >= 0 and p[k] - early <= t <= p[k] + late:
            hits[(int(c), int(p[k]))] = hits.get((int(c), int(p[k])), 0) + 1
        else:
            extra += 1
    iso = exactly = missed = multi = 0
    for c, p in by_ch.items():
        for i, r in enumerate(p):
            if (i > 0 and r - p[i - 1] < isolation) or (i + 1 < len(p) and p[i + 1] - r < isolation):
                continue
            iso += 1
            n = hits.get((c, int(r)), 0)
            exactly += n == 1
            missed += n == 0
            multi += n > 1
    return dict(isolated=iso, exactly_one=exactly, missed=missed, multi=multi, extra=extra,
                packets=int(len(ev)), pulses=len(pulses))
