"""Restatement of the reference's host-side setup math — TEST INFRASTRUCTURE (see oracle/__init__).

Written loop-for-loop after the reference (Python 2 semantics restated explicitly: ``round`` rounds
half away from zero, ``/`` on ints floors) so that it can be pinned by the reference's fixtures:
``dac.npy.npz`` (bit-exact), the castBin register constants and peakfit (tests/golden).
"""
import math
import struct

import numpy as np

FULL_SCALE = 2 ** 15 - 1          # ROACH_Setup.py:420 amp_full_scale
SCALE_FUDGE = 1.1                 # ROACH_Setup.py:453
FIX16_13_PI = 25736               # ROACH_Pulses.py:274 "-25736 = -180 degrees"


def py2round(x):
    """Python-2 ``round``: half away from zero, returns float (ROACH_Setup.py:498, 540, 542)."""
    x = float(x)
    return math.copysign(math.floor(abs(x) + 0.5), x)


def freq_comb_lut(echo, freq, sample_rate, resolution, amplitude=None, phase=None,
                  random_phase='yes'):
    """ROACH_Setup.py:416-475 ``freqCombLUT``. Returns (I, Q, scale_factor, phases)."""
    offset = 0                                   # :417
    N_freqs = len(freq)
    amplitude = [1.] * 256 if amplitude is None else list(amplitude)
    phase = [0.] * max(256, N_freqs) if phase is None else list(phase)
    size = int(sample_rate / resolution)         # :422
    I = np.array([0.] * size)
    Q = np.array([0.] * size)
    np.random.seed(1000)                         # :426
    t_f = np.arange(size, dtype=np.float64)
    for n in range(N_freqs):
        if random_phase == 'yes':
            phase[n] = np.random.uniform(0, 2 * np.pi)   # :429
        # :439-440 evaluated elementwise in the reference's operation order
        # ((((2*pi)*f)*(t+offset))/fs)+phase: identical IEEE operations, vectorised over t.
        x = 2 * np.pi * freq[n] * (t_f + offset) / sample_rate + phase[n]
        y = 2 * np.pi * freq[n] * t_f / sample_rate + phase[n]
        I = I + amplitude[n] * np.cos(x)         # :442-446
        Q = Q + amplitude[n] * np.sin(y)
    a = np.array([abs(I).max(), abs(Q).max()])
    scale_factor = a.max()
    if echo == 'yes':
        scale_factor = SCALE_FUDGE * scale_factor
    I = np.trunc(I * FULL_SCALE / scale_factor).astype(np.int64)   # :461 int() truncation
    Q = np.trunc(Q * FULL_SCALE / scale_factor).astype(np.int64)
    return I, Q, scale_factor, phase[:N_freqs]


def define_dac_lut(dac_freqs, f_base, attens, sample_rate=512e6, lut_len=2 ** 16):
    """ROACH_Setup.py:477-504 ``define_DAC_LUT`` (multi-tone as ROACH_Setup_DAC.py:458).
    Returns (I_dac, Q_dac, freqs_dac, scale_factor)."""
    freq_res = sample_rate / lut_len
    freqs = [float(f) for f in dac_freqs]
    for n, f in enumerate(freqs):                # :485-487 spectrum mirror
        freqs[n] = f_base + (f_base - f)
    for n in range(len(freqs)):                  # :493-495
        if freqs[n] < f_base:
            freqs[n] = freqs[n] + sample_rate
    freqs_dac = [py2round((f - f_base) / freq_res) * freq_res for f in freqs]   # :498
    atten_min = np.min(attens)
    amplitudes = [10 ** (+(atten_min - a) / 20.) for a in attens]           # :501
    I, Q, sf, _ = freq_comb_lut('yes', freqs_dac, sample_rate, freq_res, amplitudes)
    return I, Q, freqs_dac, sf


def select_bins(readout_freqs, fft_len=2 ** 9, sample_rate=512e6, lut_len=2 ** 16):
    """ROACH_Setup.py:534-550 ``select_bins``: returns (bins, residuals)."""
    freq_res = sample_rate / lut_len
    bins, residuals = [], []
    for f in readout_freqs:
        fft_bin = int(py2round(f * fft_len / sample_rate))
        fft_freq = fft_bin * sample_rate / fft_len
        residuals.append(py2round((f - fft_freq) / freq_res) * freq_res)
        bins.append(fft_bin)
    return bins, residuals


def define_dds_lut(dac_freqs, f_base, n_channels=256, fft_len=2 ** 9, sample_rate=512e6,
                   ch_shift=154, phase=None, lut_len=2 ** 16):
    """ROACH_Setup.py:506-532 ``define_DDS_LUT`` generalised to C channels / N-point FFT.
    Returns (I_dds, Q_dds, bins, residuals, per_ch_I [C][P], per_ch_Q [C][P])."""
    freq_res = sample_rate / lut_len
    phase = [0.] * n_channels if phase is None else list(phase)
    freqs = [float(f) for f in dac_freqs]
    for n in range(len(freqs)):
        if freqs[n] < f_base:
            freqs[n] = freqs[n] + sample_rate
    freqs_dds = [0 for _ in range(n_channels)]
    for n in range(len(freqs)):
        freqs_dds[n] = py2round((freqs[n] - f_base) / freq_res) * freq_res   # :517
    bins, resid = select_bins(freqs_dds, fft_len, sample_rate, lut_len)
    L = int(sample_rate / freq_res)
    I_dds, Q_dds = [0.] * L, [0.] * L
    per_i, per_q = [], []
    for m in range(n_channels):
        I, Q, _, _ = freq_comb_lut('no', [resid[m]], sample_rate / fft_len * 2, freq_res, [1.],
                                   [phase[m]], 'no')
        per_i.append(I)
        per_q.append(Q)
        slot = 2 * ((m + ch_shift) % n_channels)
        for j in range(len(I) // 2):            # :526-530
            I_dds[j * 2 * n_channels + slot] = I[2 * j]
            I_dds[j * 2 * n_channels + slot + 1] = I[2 * j + 1]
            Q_dds[j * 2 * n_channels + slot] = Q[2 * j]
            Q_dds[j * 2 * n_channels + slot + 1] = Q[2 * j + 1]
    return (np.array(I_dds, dtype=np.int64), np.array(Q_dds, dtype=np.int64), bins, resid,
            np.array(per_i), np.array(per_q))


def pack_luts(I_dac, Q_dac, I_dds, Q_dds):
    """ROACH_Setup.py:559-569 ``write_LUTs`` byte packing of the dram_memory blob."""
    out = []
    for n in range(len(I_dac) // 2):
        out.append(struct.pack('>h', int(Q_dds[2 * n + 1])) + struct.pack('>h', int(Q_dds[2 * n])) +
                   struct.pack('>h', int(Q_dac[2 * n + 1])) + struct.pack('>h', int(Q_dac[2 * n])) +
                   struct.pack('>h', int(I_dds[2 * n + 1])) + struct.pack('>h', int(I_dds[2 * n])) +
                   struct.pack('>h', int(I_dac[2 * n + 1])) + struct.pack('>h', int(I_dac[2 * n])))
    return b''.join(out)


def find_iq_center(I, Q):
    """ROACH_Setup.py:621-625 ``findIQcenters``."""
    return complex((np.max(I) + np.min(I)) / 2., (np.max(Q) + np.min(Q)) / 2.)


def iq_center_register(ic, qc):
    """ROACH_Setup.py:599-602: (int(I/2**3)<<16) + int(Q/2**3), no masking of a negative Q."""
    return (int(ic / 2 ** 3) << 16) + (int(qc / 2 ** 3) << 0)


def fir_coeff_words(lpf, taps=26):
    """ROACH_Pulses.py:87-95: lpf already multiplied by (2**11-1); returns the 13 register
    payloads (bytes) for FIR_b{2n}b{2n+1}."""
    words = []
    for n in range(taps // 2):
        coeff0 = np.binary_repr(int(lpf[2 * n]), 12)
        coeff1 = np.binary_repr(int(lpf[2 * n + 1]), 12)
        coeffs = int(coeff1 + coeff0, 2)
        words.append(struct.pack('>l', coeffs))
    return words


def fir_quantise(taps_float):
    """ROACH_Pulses.py:69 lpf = array(fir)*(2**11-1), then int() per tap (:88-89)."""
    lpf = np.array(taps_float) * (2 ** 11 - 1)
    return np.array([int(v) for v in lpf], dtype=np.int64)


def find_nearest(array, value):
    """ROACH_Pulses.py:113-115."""
    return (np.abs(array - value)).argmin()


def threshold_from_phase(phase_raw, nsigma=2.5):
    """ROACH_Pulses.py:259-278 (loadThresholds body). phase_raw: Fix16_13 ints.
    Returns (threshold_raw_int, median_raw)."""
    n, bins = np.histogram(phase_raw, bins=100)
    n = np.array(n, dtype='float32') / np.sum(n)
    tot = np.zeros(len(bins))
    for i in range(len(bins)):
        tot[i] = np.sum(n[:i])
    med = bins[find_nearest(tot, 0.5)]
    thresh = bins[find_nearest(tot, 0.05)]
    threshold = int(-nsigma * abs(med - thresh))
    if threshold < -FIX16_13_PI:
        threshold = -FIX16_13_PI
    return threshold, med


def snap_phase_decode(buf):
    """ROACH_Pulses.py:250-253: 'snapPhase_bram' words, two >h samples per word, halves swapped."""
    out = []
    for m in range(len(buf) // 4):
        out.append(struct.unpack('>h', buf[m * 4 + 2:m * 4 + 4])[0])
        out.append(struct.unpack('>h', buf[m * 4 + 0:m * 4 + 2])[0])
    return np.array(out)


def conv_phase_snap_decode(buf):
    """pulse_triggering_v2.py:93-94: one >h sample in bytes [2:4] of every word."""
    return np.array([struct.unpack('>h', buf[4 * m + 2:4 * m + 4])[0] for m in range(len(buf) // 4)])


def twos_comp(val, bits):
    """pulse_triggering_v2.py:22-26."""
    if (val & (1 << (bits - 1))) != 0:
        val = val - (1 << bits)
    return val


def iq_snap_decode(buf):
    """pulse_triggering_IQ.py:121-147: 16 bytes per 2 IQ pairs, nibble-straddled I."""
    h = ["0x{:02x}".format(b) for b in bytearray(buf)]
    I, Q = [], []
    for k in range(len(h) // 16):
        I.append(twos_comp(int(h[6 + 16 * k][3] + h[7 + 16 * k][2:4] + h[8 + 16 * k][2], 16), 16))
        I.append(twos_comp(int(h[11 + 16 * k][3] + h[12 + 16 * k][2:4] + h[13 + 16 * k][2], 16), 16))
        Q.append(twos_comp(int(h[9 + 16 * k][2:4] + h[10 + 16 * k][2:4], 16), 16))
        Q.append(twos_comp(int(h[14 + 16 * k][2:4] + h[15 + 16 * k][2:4], 16), 16))
    return np.array(I), np.array(Q)


def fix16_13_to_deg(raw):
    """ROACH_Pulses.py:378: raw*360/2**16*4/pi."""
    return np.array(raw) * 360. / 2 ** 16 * 4 / np.pi


def bin12_9_to_deg(x):
    """Utils/bin.py:5-7."""
    return (x / 2.0 ** 9 - 4.0) * 180.0 / np.pi


def peakfit(y1, y2, y3):
    """Utils/bin.py:12-16."""
    if y3 + y1 - 2 * y2 == 0:
        return y2
    return y2 - 0.125 * ((y3 - y1) ** 2) / (y3 + y1 - 2 * y2)


def extract_bin(value, nBits=12, binaryPoint=9, nBitsAfterEnd=0, format='rad'):
    """Utils/bin.py:18-29 with the Python-2 integer division of line 22 restated (``//``)."""
    value = value >> nBitsAfterEnd
    bitMask = int('1' * nBits, 2)
    value = value & bitMask
    signBit = int(value) // 2 ** (nBits - 1)
    if signBit != 0:
        value = ((~value) & bitMask) + 1
        value = -value
    value = float(value) / 2.0 ** binaryPoint
    if format == 'deg':
        value = value * 180.0 / np.pi
    return value


def cast_bin(value, nBits=12, binaryPoint=9, quantization='Truncate', format='uint'):
    """Utils/bin.py:31-48 (round() is Python-2 half-away-from-zero)."""
    if format == 'deg':
        value = value * np.pi / 180.0
    value = value * 2 ** binaryPoint
    if quantization == 'Truncate':
        value = int(value)
    else:
        value = int(py2round(value))
    bitMask = int('1' * nBits, 2)
    if value < 0:
        value = -value
        value = ((~value) & bitMask) + 1
    value = value & bitMask
    if format != 'uint':
        value = extract_bin(value, nBits=nBits, binaryPoint=binaryPoint)
        if format == 'deg':
            value = value * 180.0 / np.pi
    return value


def decode_pulses(bram0, bram1, addr0, addr1, n_words=2 ** 14):
    """ROACH_Pulses.py:796-832 ``readPulses`` decode of pulses_bram0/1 between two pulses_addr
    reads. Returns dict ch -> list of (timestamp, baseline12, peak12, p1_deg or None). The
    reference appends p1 only in the wrap branch (:820, :829); kept as None elsewhere."""
    scale_to_degrees = 360. / 2 ** 12 * 4 / np.pi
    out = {}

    def one(n, with_p1):
        raw1 = struct.unpack('>L', bram1[n * 4:n * 4 + 4])[0]
        raw0 = struct.unpack('>L', bram0[n * 4:n * 4 + 4])[0]
        ch = raw1 // 2 ** 24
        p1 = (raw1 % 2 ** 12 - 2 ** 11) * scale_to_degrees if with_p1 else None
        out.setdefault(ch, []).append((raw0 % 2 ** 20, (raw0 >> 20) % 2 ** 12,
                                       (raw1 >> 12) % 2 ** 12, p1))

    if addr1 >= addr0:
        for n in range(addr0, addr1):
            one(n, False)
    else:
        for n in range(addr0, n_words):
            one(n, True)
        for n in range(0, addr1):
            one(n, True)
    return out


def resdiff(x, Q, f0, aleak, ph1, da, ang1, Igain, Qgain, Ioff, Qoff):
    """lib/iqsweep.py:824-858 RESDIFF, element by element (np.vectorize(complex) as written)."""
    x = np.asarray(x, dtype=float)
    l = len(x)
    dx = (x - f0) / f0
    s21a = (np.vectorize(complex)(0, 2.0 * Q * dx)) / (complex(1, 0) + np.vectorize(complex)(0, 2.0 * Q * dx))
    s21a = s21a - complex(.5, 0)
    s21b = np.vectorize(complex)(da * dx, 0) + s21a + aleak * np.vectorize(complex)(1.0 - np.cos(dx * ph1),
                                                                                   -np.sin(dx * ph1))
    Ix1 = s21b.real * Igain
    Qx1 = s21b.imag * Qgain
    nI1 = Ix1 * np.cos(ang1) + Qx1 * np.sin(ang1)
    nQ1 = -Ix1 * np.sin(ang1) + Qx1 * np.cos(ang1)
    nI1 = nI1 + Ioff
    nQ1 = nQ1 + Qoff
    s21 = np.zeros(l * 2)
    s21[:l] = nI1
    s21[l:] = nQ1
    return s21
