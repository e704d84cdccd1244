"""Tone-comb / DAC / DDS LUT synthesis and coarse-bin selection — the host setup math of
ROACH_Setup.py:416-550, vectorised (numpy) and generalised from 256 channels / N=512 to C
channels / N=2C. Arithmetic follows the reference operation-for-operation so the results are
bit-identical (pinned by tests/golden/dac_lut.npz = the reference's saved dac.npy.npz).
"""
import math

import numpy as np

FULL_SCALE = 2 ** 15 - 1      # ROACH_Setup.py:420
SCALE_FUDGE = 1.1             # ROACH_Setup.py:453
LUT_LEN = 2 ** 16             # ROACH_Setup.py:83 N_lut_entries
DDS_LAG = 154                 # setEnvironment.sh:24, ROACH_Setup.py:508 ch_shift


def py2round(x):
    """The reference is Python 2: round() is half-away-from-zero (ROACH_Setup.py:498,540,542)."""
    x = float(x)
    return math.copysign(math.floor(abs(x) + 0.5), x)


def freq_comb_lut(echo, freq, sample_rate, resolution, amplitude=None, phase=None,
                  random_phase='yes', return_phases=False):
    """ROACH_Setup.py:416-475 freqCombLUT. Returns (I, Q, scale_factor[, phases])."""
    n_freqs = len(freq)
    amplitude = np.ones(max(256, n_freqs)) if amplitude is None else np.asarray(amplitude, float)
    phase = np.zeros(max(256, n_freqs)) if phase is None else np.array(phase, float)
    size = int(sample_rate / resolution)
    I = np.zeros(size)
    Q = np.zeros(size)
    np.random.seed(1000)                                   # :426
    if random_phase == 'yes' and n_freqs:
        phase[:n_freqs] = np.random.uniform(0, 2 * np.pi, n_freqs)   # :429, same stream
    t = np.arange(size, dtype=np.float64)
    for n in range(n_freqs):                               # accumulation order of :445-446
        arg = 2 * np.pi * freq[n] * t / sample_rate + phase[n]
        I = I + amplitude[n] * np.cos(arg)
        Q = Q + amplitude[n] * np.sin(arg)
    scale_factor = max(np.abs(I).max(), np.abs(Q).max())
    if echo == 'yes':
        scale_factor = SCALE_FUDGE * scale_factor
    I = np.trunc(I * FULL_SCALE / scale_factor).astype(np.int64)   # :461 int()
    Q = np.trunc(Q * FULL_SCALE / scale_factor).astype(np.int64)
    if return_phases:
        return I, Q, scale_factor, phase[:n_freqs].copy()
    return I, Q, scale_factor


def dac_frequencies(dac_freqs, f_base, sample_rate):
    """ROACH_Setup.py:484-498: spectrum mirror about the LO, wrap, quantise to fs/2^16."""
    res = sample_rate / LUT_LEN
    out = []
    for f in dac_freqs:
        m = f_base + (f_base - float(f))
        if m < f_base:
            m += sample_rate
        out.append(py2round((m - f_base) / res) * res)
    return out


def define_dac_lut(dac_freqs, f_base, attens, sample_rate=512e6):
    """ROACH_Setup.py:477-504 define_DAC_LUT. Returns (I_dac, Q_dac, freqs_dac, scale, phases)."""
    freqs_dac = dac_frequencies(dac_freqs, f_base, sample_rate)
    attens = np.asarray(attens, float)
    amplitudes = 10 ** ((attens.min() - attens) / 20.)
    I, Q, sf, ph = freq_comb_lut('yes', freqs_dac, sample_rate, sample_rate / LUT_LEN,
                                 amplitudes, return_phases=True)
    return I, Q, freqs_dac, sf, ph


def select_bins(readout_freqs, fft_len, sample_rate):
    """ROACH_Setup.py:534-550 select_bins: (bins, residuals)."""
    res = sample_rate / LUT_LEN
    bins, resid = [], []
    for f in readout_freqs:
        b = int(py2round(f * fft_len / sample_rate))
        resid.append(py2round((f - b * sample_rate / fft_len) / res) * res)
        bins.append(b)
    return np.array(bins, np.int64), np.array(resid)


def dds_frequencies(dac_freqs, f_base, n_channels, sample_rate):
    """ROACH_Setup.py:509-517: per-channel DDC frequency, unused channels 0."""
    res = sample_rate / LUT_LEN
    out = [0.0] * n_channels
    for n, f in enumerate(dac_freqs):
        f = float(f)
        if f < f_base:
            f += sample_rate
        out[n] = py2round((f - f_base) / res) * res
    return out


def define_dds_lut(dac_freqs, f_base, n_channels=256, sample_rate=512e6, phase=None,
                   ch_shift=DDS_LAG):
    """ROACH_Setup.py:506-532 define_DDS_LUT for C channels (N = 2C). Returns a dict with
    bins, residuals, per-channel LUTs lut_i/lut_q [C][P] (P = 2^16/C) and the DRAM-interleaved
    I_dds/Q_dds [2^16] (index j*2C + 2*((m+ch_shift)%C) + {0,1})."""
    C = n_channels
    N = 2 * C
    res = sample_rate / LUT_LEN
    phase = np.zeros(C) if phase is None else np.asarray(phase, float)
    bins, resid = select_bins(dds_frequencies(dac_freqs, f_base, C, sample_rate), N, sample_rate)
    P = LUT_LEN // C
    rate = sample_rate / N * 2
    t = np.arange(P, dtype=np.float64)
    lut_i = np.empty((C, P), np.int64)
    lut_q = np.empty((C, P), np.int64)
    for m in range(C):
        arg = 2 * np.pi * resid[m] * t / rate + phase[m]
        ci, sq = np.cos(arg), np.sin(arg)
        sf = max(np.abs(ci).max(), np.abs(sq).max())
        lut_i[m] = np.trunc(ci * FULL_SCALE / sf).astype(np.int64)
        lut_q[m] = np.trunc(sq * FULL_SCALE / sf).astype(np.int64)
    I_dds, Q_dds = interleave_dds(lut_i, lut_q, ch_shift)
    return dict(bins=bins, residuals=resid, lut_i=lut_i, lut_q=lut_q, I_dds=I_dds, Q_dds=Q_dds)


def interleave_dds(lut_i, lut_q, ch_shift=DDS_LAG):
    """[C][P] -> DRAM order of ROACH_Setup.py:526-530."""
    C, P = lut_i.shape
    I = np.zeros(C * P, np.int64)
    Q = np.zeros(C * P, np.int64)
    slot = 2 * ((np.arange(C) + ch_shift) % C)
    j = np.arange(P // 2)
    for k in (0, 1):
        idx = j[None, :] * 2 * C + slot[:, None] + k
        I[idx] = lut_i[:, 2 * j + k]
        Q[idx] = lut_q[:, 2 * j + k]
    return I, Q


def deinterleave_dds(I_dds, Q_dds, n_channels, ch_shift=DDS_LAG):
    """Inverse of interleave_dds: DRAM order -> [C][P] (what mkid_set_dds takes)."""
    C = n_channels
    P = len(I_dds) // C
    slot = 2 * ((np.arange(C) + ch_shift) % C)
    j = np.arange(P // 2)
    lut_i = np.empty((C, P), np.int64)
    lut_q = np.empty((C, P), np.int64)
    for k in (0, 1):
        idx = j[None, :] * 2 * C + slot[:, None] + k
        lut_i[:, 2 * j + k] = np.asarray(I_dds)[idx]
        lut_q[:, 2 * j + k] = np.asarray(Q_dds)[idx]
    return lut_i, lut_q
