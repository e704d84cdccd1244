"""Register / BRAM / packet codecs of the reference's host surface (host code of the product).

Each function restates one reference encoding so that a ChannelizerControls caller and the
FpgaClient shim (mkids_sdr_amd.roach) see the same bytes as on the ROACH:
  fixed point        Utils/bin.py castBin / extractBin / bin12_9ToDeg / peakfit
  FIR registers      ROACH_Pulses.py:59-111 (FIR_b{2n}b{2n+1}: coeff1<<12 | coeff0, 12-bit 2's c.)
  IQ centre register ROACH_Setup.py:595-605 ((int(I/8)<<16) + int(Q/8))
  DRAM LUT blob      ROACH_Setup.py:552-570 (8 x >h per sample pair)
  thresholds         ROACH_Pulses.py:211-299 (histogram/CDF of a Fix16_13 snapshot)
  snapshots          ROACH_Pulses.py:248-253 (snapPhase_bram), pulse_triggering_v2.py:93-95,
                     pulse_triggering_IQ.py:121-147 (conv_phase_snapIQ_bram)
  photon packets     ROACH_Pulses.py:796-859, PacketMaster.c:291-292, 331-337
"""
import math
import struct

import numpy as np

FIX16_13_PI = 25736                      # ROACH_Pulses.py:274
SCALE_TO_ANGLE = 360. / 2 ** 16 * 4 / np.pi   # ROACH_Pulses.py:226 (Fix16_13 LSB in degrees)
PKT_CH_SHIFT, PKT_PEAK_SHIFT, PKT_BASE_SHIFT = 52, 40, 28
PKT_TS_MASK = (1 << 28) - 1


def py2round(x):
    x = float(x)
    return math.copysign(math.floor(abs(x) + 0.5), x)


# ---- fixed point (Utils/bin.py) ------------------------------------------------------------
def extract_bin(value, nBits=12, binaryPoint=9, nBitsAfterEnd=0, format='rad'):
    value = int(value) >> nBitsAfterEnd
    mask = (1 << nBits) - 1
    value &= mask
    if value >> (nBits - 1):          # Python-2 integer division of Utils/bin.py:22
        value = -(((~value) & mask) + 1)
    out = float(value) / 2.0 ** binaryPoint
    return out * 180.0 / np.pi if format == 'deg' else out


def cast_bin(value, nBits=12, binaryPoint=9, quantization='Truncate', format='uint'):
    if format == 'deg':
        value = value * np.pi / 180.0
    value = value * 2 ** binaryPoint
    value = int(value) if quantization == 'Truncate' else int(py2round(value))
    mask = (1 << nBits) - 1
    if value < 0:
        value = ((~(-value)) & mask) + 1
    value &= mask
    if format != 'uint':
        value = extract_bin(value, nBits, binaryPoint)
        if format == 'deg':
            value = value * 180.0 / np.pi
    return value


def peakfit(y1, y2, y3):
    den = y3 + y1 - 2 * y2
    return y2 if den == 0 else y2 - 0.125 * ((y3 - y1) ** 2) / den


def bin12_9_to_rad(x):
    return np.asarray(x) / 2.0 ** 9 - 4.0


def bin12_9_to_deg(x):
    return bin12_9_to_rad(x) * 180.0 / np.pi


def fix16_13_to_deg(raw):
    return np.asarray(raw) * 360. / 2 ** 16 * 4 / np.pi


# ---- baseline registers (lib/set_alpha.py, set_svf.py, set_base_thresh.py) -------------------
def baseline_registers(alpha=0.08, critical_freq=200.0, sample_rate=1e6, q=0.7, base_thresh=1.0):
    kf = 2 * np.sin(np.pi * critical_freq / sample_rate)
    return dict(alpha=cast_bin(alpha, quantization='Round'),
                kf=cast_bin(kf, quantization='Round', nBits=18, binaryPoint=16),
                kq=cast_bin(1. / q, quantization='Round', nBits=18, binaryPoint=16),
                base_thr=cast_bin(base_thresh, quantization='Round', nBits=16, binaryPoint=13))


# ---- FIR taps (ROACH_Pulses.py:59-111) --------------------------------------------------------
def fir_quantise(taps):
    """lpf = array(fir)*(2**11-1); int() per tap (truncation toward zero)."""
    return np.trunc(np.asarray(taps, np.float64) * (2 ** 11 - 1)).astype(np.int64)


def fir_registers(taps12):
    """26 int12 taps -> 13 big-endian words for FIR_b{2n}b{2n+1}."""
    out = []
    for n in range(len(taps12) // 2):
        c0 = int(taps12[2 * n]) & 0xFFF
        c1 = int(taps12[2 * n + 1]) & 0xFFF
        out.append(struct.pack('>l', (c1 << 12) | c0))
    return out


def decode_fir_register(payload):
    """4-byte FIR_b* payload -> (coeff 2n, coeff 2n+1) as signed 12-bit ints. Accepts the
    active-channel form (>l, coeff1<<12|coeff0) and the zeroing form (two >h, :104)."""
    w = struct.unpack('>L', payload)[0]
    def s12(v):
        v &= 0xFFF
        return v - 0x1000 if v & 0x800 else v
    return s12(w), s12(w >> 12)


# ---- IQ centres (ROACH_Setup.py:595-605) ------------------------------------------------------
def center_register(ic, qc):
    return (int(ic / 2 ** 3) << 16) + int(qc / 2 ** 3)


def decode_center_register(w):
    """Inverse of center_register for |I/8|,|Q/8| < 2^15 (handles the unmasked negative Q)."""
    w = int(w) & 0xFFFFFFFF
    if w & 0x80000000:
        w -= 1 << 32               # the register is a signed 32-bit write_int value
    q16 = w & 0xFFFF
    if q16 & 0x8000:
        q16 -= 0x10000
    i16 = (w - q16) >> 16          # arithmetic: already signed
    return 8.0 * i16, 8.0 * q16


# ---- DRAM LUT blob (ROACH_Setup.py:552-570) ---------------------------------------------------
def pack_luts(I_dac, Q_dac, I_dds, Q_dds):
    n = len(I_dac) // 2
    a = np.empty((n, 8), '>i2')
    a[:, 0] = np.asarray(Q_dds)[1::2]
    a[:, 1] = np.asarray(Q_dds)[0::2]
    a[:, 2] = np.asarray(Q_dac)[1::2]
    a[:, 3] = np.asarray(Q_dac)[0::2]
    a[:, 4] = np.asarray(I_dds)[1::2]
    a[:, 5] = np.asarray(I_dds)[0::2]
    a[:, 6] = np.asarray(I_dac)[1::2]
    a[:, 7] = np.asarray(I_dac)[0::2]
    return a.tobytes()


def unpack_luts(blob):
    a = np.frombuffer(blob, '>i2').reshape(-1, 8).astype(np.int64)
    n = a.shape[0]
    I_dac = np.empty(2 * n, np.int64); Q_dac = np.empty(2 * n, np.int64)
    I_dds = np.empty(2 * n, np.int64); Q_dds = np.empty(2 * n, np.int64)
    Q_dds[1::2], Q_dds[0::2], Q_dac[1::2], Q_dac[0::2] = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
    I_dds[1::2], I_dds[0::2], I_dac[1::2], I_dac[0::2] = a[:, 4], a[:, 5], a[:, 6], a[:, 7]
    return I_dac, Q_dac, I_dds, Q_dds


# ---- thresholds (ROACH_Pulses.py:211-299) -----------------------------------------------------
def threshold_from_phase(phase_raw, nsigma=2.5):
    """Per-channel Fix16_13 threshold relative to the baseline, and the median bin edge."""
    n, bins = np.histogram(phase_raw, bins=100)
    n = np.array(n, dtype='float32') / np.sum(n)
    tot = np.zeros(len(bins))
    for i in range(len(bins)):
        tot[i] = np.sum(n[:i])
    med = bins[np.abs(tot - 0.5).argmin()]
    p05 = bins[np.abs(tot - 0.05).argmin()]
    thr = int(-nsigma * abs(med - p05))
    return max(thr, -FIX16_13_PI), med


def thresholds_from_phase_block(raw, nsigma=2.5):
    """raw [J][C] Fix16_13 -> int32 thresholds [C] (loadThresholds for every channel)."""
    raw = np.asarray(raw)
    return np.array([threshold_from_phase(raw[:, c], nsigma)[0] for c in range(raw.shape[1])],
                    np.int32)


# ---- snapshots ----------------------------------------------------------------------------------
def encode_snap_phase(raw):
    """Fix16_13 samples -> snapPhase_bram bytes (2 per word, halves swapped: decode reads [2:4]
    then [0:2], ROACH_Pulses.py:251-253)."""
    r = np.asarray(raw, np.int64)
    if len(r) % 2:
        r = np.append(r, 0)
    a = np.empty((len(r) // 2, 2), '>i2')
    a[:, 1] = r[0::2]
    a[:, 0] = r[1::2]
    return a.tobytes()


def decode_snap_phase(buf):
    a = np.frombuffer(buf, '>i2').reshape(-1, 2).astype(np.int64)
    return np.stack([a[:, 1], a[:, 0]], axis=1).reshape(-1)


def decode_qdr(buf):
    """qdr0_memory longsnapshot words -> Fix16_13 raw, 2 samples per 32-bit word in time order,
    '>h' each (ROACH_Pulses.py:476: struct.unpack('>%dh' % nLongsnapSamples, ...))."""
    return np.frombuffer(bytes(buf), '>i2').astype(np.int64)


def noise_spectrum(phase_deg, n_averages=100, norm1=50.0):
    """The longsnapshot phase-noise spectrum (ROACH_Pulses.py:521-543): the stream cut into
    n_averages pieces of len // n_averages samples, mean over pieces of
    20 log10(|fft(piece)| / norm1 / 1e-6); returns (fftfreq(piece length), spectrum)."""
    x = np.asarray(phase_deg, np.float64)
    n = len(x) // n_averages
    pieces = x[:n * n_averages].reshape(n_averages, n)
    spec = (20 * np.log10(np.abs(np.fft.fft(pieces, axis=1)) / norm1 / 1e-6)).sum(axis=0) / n_averages
    return np.fft.fftfreq(n), spec


def encode_conv_phase_snap(raw):
    """conv_phase_snapPhase_bram: one sample per word in bytes [2:4] (pulse_triggering_v2.py:94)."""
    r = np.asarray(raw, np.int64)
    a = np.zeros((len(r), 2), '>i2')
    a[:, 1] = r
    return a.tobytes()


def decode_conv_phase_snap(buf):
    """conv_phase_snap{I,Q,Phase}_bram: the '>h' sample in bytes [2:4] of every 32-bit word
    (readouttesterIQ.py:71-74, ROACH_Pulses_IQ.py:404-406, pulse_triggering_v2.py:93-94)."""
    return np.frombuffer(buf, '>i2').reshape(-1, 2)[:, 1].astype(np.int64)


def encode_iq_snap(I, Q):
    """conv_phase_snapIQ_bram: 16 bytes per 2 I/Q pairs, I nibble-straddled over bytes 6-8 / 11-13,
    Q in bytes 9-10 / 14-15 (pulse_triggering_IQ.py:133-147)."""
    I = np.asarray(I, np.int64) & 0xFFFF
    Q = np.asarray(Q, np.int64) & 0xFFFF
    k = len(I) // 2
    b = np.zeros((k, 16), np.uint8)
    for h, (i0, i1, q0, q1) in enumerate(zip(I[0::2], I[1::2], Q[0::2], Q[1::2])):
        b[h, 6] = (i0 >> 12) & 0xF
        b[h, 7] = (i0 >> 4) & 0xFF
        b[h, 8] = (i0 & 0xF) << 4
        b[h, 9], b[h, 10] = q0 >> 8, q0 & 0xFF
        b[h, 11] = (i1 >> 12) & 0xF
        b[h, 12] = (i1 >> 4) & 0xFF
        b[h, 13] = (i1 & 0xF) << 4
        b[h, 14], b[h, 15] = q1 >> 8, q1 & 0xFF
    return b.tobytes()


def decode_iq_snap(buf):
    b = np.frombuffer(buf, np.uint8).reshape(-1, 16).astype(np.int64)
    def s16(v):
        return np.where(v & 0x8000, v - 0x10000, v)
    i0 = s16(((b[:, 6] & 0xF) << 12) | (b[:, 7] << 4) | (b[:, 8] >> 4))
    i1 = s16(((b[:, 11] & 0xF) << 12) | (b[:, 12] << 4) | (b[:, 13] >> 4))
    q0 = s16((b[:, 9] << 8) | b[:, 10])
    q1 = s16((b[:, 14] << 8) | b[:, 15])
    return np.stack([i0, i1], 1).reshape(-1), np.stack([q0, q1], 1).reshape(-1)


# ---- photon packets -----------------------------------------------------------------------------
def unpack_wide(words):
    w = np.asarray(words, np.uint64)
    return dict(ch=((w >> np.uint64(52)) & np.uint64(0xFFF)).astype(np.int64),
                peak=((w >> np.uint64(40)) & np.uint64(0xFFF)).astype(np.int64),
                base=((w >> np.uint64(28)) & np.uint64(0xFFF)).astype(np.int64),
                ts=(w & np.uint64(PKT_TS_MASK)).astype(np.int64))


def wide_to_reference(words):
    """Wide device packet -> reference 64-bit packet (same as mkid_pack_reference)."""
    u = unpack_wide(words)
    if np.any(u['ch'] >= 255):
        raise ValueError('reference packet has an 8-bit channel field (255 = end of second)')
    p1 = np.clip(u['peak'] - u['base'] + 2048, 0, 4095)
    out = ((u['ch'].astype(np.uint64) << np.uint64(56)) | (u['peak'].astype(np.uint64) << np.uint64(44)) |
           (p1.astype(np.uint64) << np.uint64(32)) | (u['base'].astype(np.uint64) << np.uint64(20)) |
           (u['ts'].astype(np.uint64) & np.uint64(0xFFFFF)))
    return out


def reference_bram_words(ref_packets):
    """64-bit packets -> (pulses_bram0 word = low 32 bits, pulses_bram1 word = high 32 bits)."""
    p = np.asarray(ref_packets, np.uint64)
    return (p & np.uint64(0xFFFFFFFF)).astype(np.uint32), (p >> np.uint64(32)).astype(np.uint32)


END_OF_SECOND = np.uint64(0xFFFFFFFFFFFFFFFF)   # PacketMaster.c:331-337 (adr 255, all ones)


def py2_str(x):
    """str(x) of a float as Python 2 printed it (and the reference's text files hold, e.g.
    ch_noifreqs_0.txt, ch_snap_0.txt: ROACH_Pulses.py:476-536 write str(q) per line): repr at 12
    significant digits, '.0' kept on integral values."""
    v = float(x)
    if v != v:
        return 'nan'
    if v in (float('inf'), float('-inf')):
        return 'inf' if v > 0 else '-inf'
    t = '%.12g' % v
    if '.' not in t and 'e' not in t:
        t += '.0'
    return t
