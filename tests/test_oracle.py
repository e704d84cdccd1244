"""Pin the CPU oracle against the reference's own fixtures and against itself (C vs Python)."""
import json
import os

import numpy as np
import pytest

import signals
from oracle import chain, setup_ref, trigger, trigger_ref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def golden(name):
    return os.path.join(GOLD, name)


def test_dac_lut_bit_exact():
    """dac.npy.npz (written by ROACH_Setup.py:558) reproduced by the freqCombLUT restatement:
    one DAC tone 100 MHz above a 4 GHz LO (mirrored to bin 52736), seed-1000 phase."""
    d = np.load(golden('dac_lut.npz'))
    I, Q, freqs, sf = setup_ref.define_dac_lut([4.1e9], 4.0e9, [1.0] * 256)
    assert freqs == [412e6]
    assert np.array_equal(I, d['I_dac']) and np.array_equal(Q, d['Q_dac'])
    I_dds, Q_dds, bins, resid, _, _ = setup_ref.define_dds_lut([4.1e9], 4.0e9, 256, 512)
    assert np.array_equal(I_dds, d['I_dds']) and np.array_equal(Q_dds, d['Q_dds'])
    assert bins[0] == 100 and resid[0] == 0.0


def test_castbin_registers_and_vectors():
    g = json.load(open(golden('bin_vectors.json')))
    assert g['registers'] == dict(kf=82, kq=93623, alpha=41, base_thresh=8192)
    for c in g['castBin']:
        assert setup_ref.cast_bin(c['value'], c['nBits'], c['binaryPoint'], c['quantization']) == c['out']
    for p in g['peakfit']:
        assert setup_ref.peakfit(*p['y']) == pytest.approx(p['out'], rel=0, abs=0)
    for d in g['bin12_9ToDeg']:
        assert setup_ref.bin12_9_to_deg(d['x']) == d['out']


def test_py2_semantics():
    assert setup_ref.py2round(2.5) == 3.0 and setup_ref.py2round(-2.5) == -3.0
    # extractBin line 22 is Python-2 integer division: 5 -> +0.009765625, not py3's -7.99
    assert setup_ref.extract_bin(5) == pytest.approx(5 / 512.0)
    assert setup_ref.extract_bin(0xFFF) == pytest.approx(-1 / 512.0)


def test_snapshot_threshold_fixture():
    """ch_snap_0.txt (ROACH_Pulses.py:482-484): Fix16_13 multiples; loadThresholds restatement.
    The threshold value is builder-computed (the reference never recorded one)."""
    deg = np.loadtxt(golden('ch_snap_0.txt'))
    raw = deg / setup_ref.fix16_13_to_deg(1)
    assert np.abs(raw - np.rint(raw)).max() < 1e-6
    raw = np.rint(raw).astype(np.int64)
    assert raw.min() == 14896 and raw.max() == 22288
    thr, med = setup_ref.threshold_from_phase(raw)
    assert thr == -5913
    assert med == pytest.approx(18961.6)


def test_noise_freq_fixture():
    f = np.loadtxt(golden('ch_noifreqs_0.txt'))
    assert np.abs(f - np.fft.fftfreq(len(f))).max() < 1e-12


def test_fir_files_quantisation():
    lpf = setup_ref.fir_quantise(np.loadtxt(golden('fir/BlackmanFilter_250kHz.txt')))
    assert lpf.tolist() == [0, 0, 3, 8, 17, 32, 53, 80, 111, 142, 172, 194, 206, 206, 194, 172, 142,
                            111, 80, 53, 32, 17, 8, 3, 0, 0]
    mf = setup_ref.fir_quantise(np.loadtxt(golden('fir/matched_30us.txt')))
    assert len(mf) == 26 and mf[0] == 160 and mf[-1] == 69
    words = setup_ref.fir_coeff_words(mf)
    assert len(words) == 13 and words[0] == bytes.fromhex('0009b0a0')


def test_packet_decode_roundtrip():
    import struct
    ch, peak, p1, base, ts = 7, 1500, 2100, 1900, 123456
    w1 = (ch << 24) | (peak << 12) | p1
    w0 = (base << 20) | ts
    b0 = bytearray(4 * 2 ** 14)
    b1 = bytearray(4 * 2 ** 14)
    struct.pack_into('>L', b0, 4 * 5, w0)
    struct.pack_into('>L', b1, 4 * 5, w1)
    out = setup_ref.decode_pulses(bytes(b0), bytes(b1), 5, 6)
    assert out == {7: [(ts, base, peak, None)]}
    out = setup_ref.decode_pulses(bytes(b0), bytes(b1), 2 ** 14 - 1, 6)
    assert out[7][0][3] == pytest.approx((p1 - 2048) * 360. / 2 ** 12 * 4 / np.pi)


@pytest.mark.parametrize('mode,rearm_q8', [(0, 0), (1, 0), (2, 0), (1, 128), (2, 200), (2, 256)])
def test_trigger_c_equals_python(oracle_lib, mode, rearm_q8):
    """The C trigger and its pure-Python twin, written independently, agree packet for packet;
    rearm_q8 > 0 exercises the re-arm hysteresis (mkid_set_rearm levels)."""
    rng = np.random.default_rng(mode)
    C, J = 4, 2500
    raw = (rng.normal(0, 120, (J, C)) + 2000).astype(np.int64)
    for c in range(C):
        for s in rng.integers(40, J - 400, 5):
            t = np.arange(300)
            raw[s:s + 300, c] -= (9000 * (1 - np.exp(-t / 0.1)) * np.exp(-t / 65)).astype(np.int64)
    raw = np.clip(raw, -25736, 25736).astype(np.int16)
    taps = np.tile(setup_ref.fir_quantise(np.loadtxt(golden('fir/matched_30us.txt'))), (C, 1))
    thr = np.array([-1400, -2000, -900, -1500]) if mode else np.array([1000, 800, 1200, 900])
    t = trigger.Trigger(C, taps, thr, mode=mode, dead=20, rearm_q8=rearm_q8)
    e1, _, _ = t.run(raw[:1111])
    e2, _, _ = t.run(raw[1111:])
    lv = [int(v) - ((int(v) * rearm_q8) >> 8) for v in thr]     # floor division, restated
    ev, _, _ = trigger_ref.trigger(raw, taps, thr, mode, 41, 82, 93623, 8192, 20, rearm=lv)
    key = lambda w: ((int(w) >> 52), int(w) & ((1 << 28) - 1))
    assert sorted(map(int, e1.tolist() + e2.tolist()), key=key) == sorted(map(int, ev), key=key)
    assert len(ev) >= 10


def test_oracle_chain_tone_is_constant_phase():
    """A bin-centred + residual tone, DDC'd by its own LUT, gives a constant channel phase."""
    c = signals.make_case(64, 2 ** 15, seed=3, noise=0.0)
    r = signals.oracle_chain(c).process(c.iq)
    ph = r['phase'][64:]
    assert np.abs(signals.wrap(ph - ph[0])).max() < 2e-3
    amp = np.abs(r['y'][64:]).mean(0)
    assert np.all(amp > 0.8 * c.tone_amp) and np.all(amp < 1.05 * c.tone_amp)


def test_oracle_chain_streaming_invariance():
    c = signals.make_case(128, 2 ** 16, seed=4, pulses_per_ch=1.0)
    a = signals.oracle_chain(c).process(c.iq)
    o = signals.oracle_chain(c)
    parts = [o.process(c.iq[x:y]) for x, y in ((0, 256), (256, 2 ** 14), (2 ** 14, 2 ** 16))]
    assert np.array_equal(np.concatenate([p['raw'] for p in parts]), a['raw'])
    np.testing.assert_allclose(np.concatenate([p['phase'] for p in parts]), a['phase'], atol=1e-12)


def test_pfb_prototype_matches_product():
    from mkids_sdr_amd.pfb import pfb_prototype
    for N in (128, 512, 2048):
        assert np.array_equal(pfb_prototype(N), chain.pfb_prototype(N))
