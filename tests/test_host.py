"""Host-side product code against the oracle restatement and the reference fixtures (CPU only):
LUT synthesis, register codecs, the FpgaClient register shim and the ChannelizerControls
mirror driving it (no GPU: the shim's data path is not touched)."""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import struct

import numpy as np
import pytest

from mkids_sdr_amd import codecs, lut
from mkids_sdr_amd.roach import FpgaClient, RoachPulses, RoachSetup
from oracle import replay, setup_ref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def test_lut_matches_reference_fixture():
    d = np.load(os.path.join(GOLD, 'dac_lut.npz'))
    I, Q, freqs, sf, _ = lut.define_dac_lut([4.1e9], 4.0e9, [1.0] * 256)
    assert np.array_equal(I, d['I_dac']) and np.array_equal(Q, d['Q_dac'])
    r = lut.define_dds_lut([4.1e9], 4.0e9, 256)
    assert np.array_equal(r['I_dds'], d['I_dds']) and np.array_equal(r['Q_dds'], d['Q_dds'])


@pytest.mark.parametrize('C,fs', [(64, 512e6), (256, 550e6), (1024, 550e6)])
def test_lut_matches_oracle_multitone(C, fs):
    rng = np.random.default_rng(C)
    f = list(4e9 + rng.uniform(-fs / 2, fs / 2, min(C, 40)))
    ph = rng.uniform(0, 2 * np.pi, C)
    a = setup_ref.define_dds_lut(f, 4e9, C, 2 * C, fs, 154, phase=ph)
    b = lut.define_dds_lut(f, 4e9, C, fs, phase=ph)
    assert np.array_equal(a[0], b['I_dds']) and np.array_equal(a[1], b['Q_dds'])
    assert list(a[2]) == list(b['bins'])
    at = rng.uniform(0, 6, len(f))
    A = setup_ref.define_dac_lut(f, 4e9, at, fs)
    B = lut.define_dac_lut(f, 4e9, at, fs)
    assert np.array_equal(A[0], B[0]) and np.array_equal(A[1], B[1]) and A[2] == B[2]


def test_dds_interleave_roundtrip():
    r = lut.define_dds_lut([4.1e9, 4.2e9], 4.0e9, 256, phase=np.linspace(0, 3, 256))
    li, lq = lut.deinterleave_dds(r['I_dds'], r['Q_dds'], 256)
    assert np.array_equal(li, r['lut_i']) and np.array_equal(lq, r['lut_q'])


def test_pack_luts_matches_reference_packing():
    d = np.load(os.path.join(GOLD, 'dac_lut.npz'))
    n = 512  # the struct.pack loop is slow; a prefix pins the byte order
    a = setup_ref.pack_luts(d['I_dac'][:n], d['Q_dac'][:n], d['I_dds'][:n], d['Q_dds'][:n])
    b = codecs.pack_luts(d['I_dac'][:n], d['Q_dac'][:n], d['I_dds'][:n], d['Q_dds'][:n])
    assert a == b
    full = codecs.pack_luts(d['I_dac'], d['Q_dac'], d['I_dds'], d['Q_dds'])
    assert len(full) == 512 * 1024
    back = codecs.unpack_luts(full)
    for x, k in zip(back, ('I_dac', 'Q_dac', 'I_dds', 'Q_dds')):
        assert np.array_equal(x, d[k])


def test_cast_bin_and_registers():
    import json
    g = json.load(open(os.path.join(GOLD, 'bin_vectors.json')))
    for c in g['castBin']:
        assert codecs.cast_bin(c['value'], c['nBits'], c['binaryPoint'], c['quantization']) == c['out']
    r = codecs.baseline_registers()
    assert r == dict(alpha=41, kf=82, kq=93623, base_thr=8192)
    for p in g['peakfit']:
        assert codecs.peakfit(*p['y']) == p['out']


def test_fir_register_codec():
    taps = codecs.fir_quantise(np.loadtxt(os.path.join(GOLD, 'fir', 'matched_30us.txt')))
    words = codecs.fir_registers(taps)
    assert words == setup_ref.fir_coeff_words(taps)
    neg = np.array([-5, 7, -2048, 2047] + [0] * 22)
    for n, w in enumerate(codecs.fir_registers(neg)):
        assert codecs.decode_fir_register(w) == (neg[2 * n], neg[2 * n + 1])
    zero_form = struct.pack('>h', 0) + struct.pack('>h', 0)       # ROACH_Pulses.py:104
    assert codecs.decode_fir_register(zero_form) == (0, 0)


@pytest.mark.parametrize('ic,qc', [(800.0, -24.0), (-8000.0, 16000.0), (-3.0, -9.0), (0.0, 0.0)])
def test_center_register_codec(ic, qc):
    w = codecs.center_register(ic, qc)
    assert w == setup_ref.iq_center_register(ic, qc)
    i2, q2 = codecs.decode_center_register(w)
    assert i2 == 8 * int(ic / 8) and q2 == 8 * int(qc / 8)


def test_threshold_codec_matches_oracle():
    deg = np.loadtxt(os.path.join(GOLD, 'ch_snap_0.txt'))
    raw = np.rint(deg / codecs.fix16_13_to_deg(1)).astype(np.int64)
    assert codecs.threshold_from_phase(raw) == setup_ref.threshold_from_phase(raw)
    block = np.stack([raw, raw[::-1], raw // 2], axis=1)
    thr = codecs.thresholds_from_phase_block(block)
    assert list(thr) == [setup_ref.threshold_from_phase(block[:, c])[0] for c in range(3)]


def test_snapshot_codecs_match_reference_decoders():
    rng = np.random.default_rng(1)
    raw = rng.integers(-25736, 25737, 2048)
    assert np.array_equal(setup_ref.snap_phase_decode(codecs.encode_snap_phase(raw)), raw)
    assert np.array_equal(codecs.decode_snap_phase(codecs.encode_snap_phase(raw)), raw)
    assert np.array_equal(setup_ref.conv_phase_snap_decode(codecs.encode_conv_phase_snap(raw)), raw)
    assert np.array_equal(codecs.decode_conv_phase_snap(codecs.encode_conv_phase_snap(raw)), raw)
    full = rng.integers(-32768, 32768, 2048)          # conv_phase_snapI/Q_bram: full int16 range
    assert np.array_equal(setup_ref.conv_phase_snap_decode(codecs.encode_conv_phase_snap(full)), full)
    assert np.array_equal(codecs.decode_conv_phase_snap(codecs.encode_conv_phase_snap(full)), full)
    I = rng.integers(-32768, 32768, 512)
    Q = rng.integers(-32768, 32768, 512)
    buf = codecs.encode_iq_snap(I, Q)
    a, b = setup_ref.iq_snap_decode(buf)
    assert np.array_equal(a, I) and np.array_equal(b, Q)
    a, b = codecs.decode_iq_snap(buf)
    assert np.array_equal(a, I) and np.array_equal(b, Q)


def test_conv_phase_snapshot_arming():
    """FpgaClient's conv_phase snapshot BRAMs (no GPU: the capture is stubbed with a counter).
    The BRAMs armed by one startSnap strobe share one capture, taken at the first read after the
    strobe; a second read without a new strobe returns the held capture; a never-armed BRAM
    free-runs (a fresh capture per read)."""
    from mkids_sdr_amd.roach import FpgaClient
    roach = FpgaClient(n_channels=64, gpu=False)
    calls = []

    def fake_capture(rows):
        k = len(calls)
        calls.append(rows)
        base = np.arange(rows, dtype=np.int64) + 1000 * k
        return dict(I=base, Q=-base, phase=base // 2)
    roach._capture = fake_capture

    def arm(*names):
        for n in names:
            roach.write_int('conv_phase_startSnap' + n, 0)
        for n in names:
            roach.write_int('conv_phase_snap%s_ctrl' % n, 1)
            roach.write_int('conv_phase_snap%s_ctrl' % n, 0)
        for n in names:
            roach.write_int('conv_phase_startSnap' + n, 1)

    dec = codecs.decode_conv_phase_snap
    arm('I', 'Q', 'Phase')                                      # readouttesterIQ.py:43-54
    i = dec(roach.read('conv_phase_snapI_bram', 4 * 16))
    q = dec(roach.read('conv_phase_snapQ_bram', 4 * 16))
    p = dec(roach.read('conv_phase_snapPhase_bram', 4 * 16))
    assert calls == [16]                                        # one capture for the three
    assert np.array_equal(i, np.arange(16)) and np.array_equal(q, -i) and np.array_equal(p, i // 2)
    assert np.array_equal(dec(roach.read('conv_phase_snapQ_bram', 4 * 8)), -i[:8])   # held
    assert calls == [16]
    with pytest.raises(RuntimeError):
        roach.read('conv_phase_snapI_bram', 4 * 32)             # deeper than the capture
    arm('I', 'Q')                                               # ROACH_Pulses_IQ.py:376-386
    i2 = dec(roach.read('conv_phase_snapI_bram', 4 * 16))
    assert calls == [16, 16] and i2[0] == 1000
    assert np.array_equal(dec(roach.read('conv_phase_snapPhase_bram', 4 * 16)), p)   # not re-armed
    a, b = codecs.decode_iq_snap(roach.read('conv_phase_snapIQ_bram', 4 * 8))      # never armed
    b2, _ = codecs.decode_iq_snap(roach.read('conv_phase_snapIQ_bram', 4 * 8))
    assert calls == [16, 16, 4, 4] and a[0] == 2000 and b2[0] == 3000
    roach.progdev('x.bof')
    assert roach._armed == set() and roach._snaps == {}


def test_packet_codecs():
    from oracle.trigger_ref import pack_wide
    w = np.array([pack_wide(7, -3000, 1200, 123456789), pack_wide(200, 5000, -700, 17)], np.uint64)
    u = codecs.unpack_wide(w)
    assert list(u['ch']) == [7, 200]
    ref = codecs.wide_to_reference(w)
    b0, b1 = codecs.reference_bram_words(ref)
    buf0 = b0.astype('>u4').tobytes() + bytes(4 * (2 ** 14 - 2))
    buf1 = b1.astype('>u4').tobytes() + bytes(4 * (2 ** 14 - 2))
    dec = setup_ref.decode_pulses(buf0, buf1, 0, 2)
    assert dec[7][0][0] == 123456789 % 2 ** 20 and dec[7][0][2] == u['peak'][0]
    assert dec[200][0][1] == u['base'][1]
    with pytest.raises(ValueError):
        codecs.wide_to_reference(np.array([pack_wide(300, 0, 0, 0)], np.uint64))


def test_register_shim_decodes_setup_path():
    """RoachSetup/RoachPulses drive the FpgaClient exactly like the reference; the shim's decoded
    device configuration must equal the direct computation."""
    C = 256
    roach = FpgaClient(n_channels=C, gpu=False)
    roach.progdev('pulse_trigger_2022_Jan_24_1322.bof')
    freqs = [4.0e9 + d for d in (-91.3e6, 12.5e6, 100e6, 203.1e6)]
    rs = RoachSetup(roach, freqs, 4.0e9, n_channels=C)
    rs.define_LUTs()
    d = lut.define_dds_lut(freqs, 4.0e9, C)
    assert np.array_equal(roach.cfg.bins, d['bins'] % (2 * C))
    assert np.array_equal(roach.cfg.lut_i, d['lut_i']) and np.array_equal(roach.cfg.lut_q, d['lut_q'])
    I, Q, _, _, _ = lut.define_dac_lut(freqs, 4.0e9, np.ones(4))
    assert np.array_equal(roach.cfg.dac_i, I) and np.array_equal(roach.cfg.dac_q, Q)
    rs.iq_centers[:4] = [800 - 24j, -8000 + 16000j, -3 - 9j, 1000 + 1000j]
    rs.loadIQcenters()
    assert roach.cfg.ic[1] == -8000.0 and roach.cfg.qc[1] == 16000.0 and roach.cfg.qc[0] == -24.0
    fir = np.loadtxt(os.path.join(GOLD, 'fir', 'matched_30us.txt'))
    rp = RoachPulses(roach, 4, fir, n_channels=C)
    rp.zeroChannels[2] = 1
    rp.loadFIRcoeffs()
    q = codecs.fir_quantise(fir)
    assert np.array_equal(roach.cfg.fir[0], q) and np.array_equal(roach.cfg.fir[3], q)
    assert not roach.cfg.fir[2].any() and not roach.cfg.fir[4:].any()
    for ch, thr in ((0, -5913), (3, -120)):
        roach.write_int('capture_threshold', thr)
        roach.write_int('capture_load_thresh', (ch << 1) + 1)
        roach.write_int('capture_load_thresh', ch << 1)
    assert roach.cfg.thr[0] == -5913 and roach.cfg.thr[3] == -120
    roach.write_int('capture_Baseline_alpha', 41)
    roach.write_int('capture_base_Kf', 82)
    assert roach.cfg.baseline['kf'] == 82
    with pytest.raises(RuntimeError):
        roach.read_int('no_such_register')
    assert roach.read_int('DRAM_LUT_rd_valid') == 0


def test_replay_triggers_restated():
    """Host replays (pulse_triggering*.py) on a synthetic phase trace: hits at the injected
    pulses, skip semantics as in the reference loops."""
    rng = np.random.default_rng(5)
    x = rng.normal(10.0, 1.0, 20000)
    starts = [3000, 3500, 9000, 15000]
    for s in starts:
        t = np.arange(600)
        x[s:s + 600] -= 60 * np.exp(-t / 65.0)
    h = replay.rolling_mean_trigger(x)
    assert h == [3000, 9000, 15000]   # 3500 falls inside the 1000-sample skip after 3000
    h2 = replay.block_mean_trigger(x, averagelength=128, start=100, need=300, skip=200,
                                   wrap_negative=False)
    assert h2[0] == 3000 and 3500 in h2


def test_lds_layouts_linear():
    """st_read/st_write use base + compile-time offsets: every layout/pass pair must be linear
    (a wrong layout would silently scramble the FFT)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import lds_layouts as L
    for N in L.FRONT_PLANS:
        for name, Rw, NS, Rr, p in L.front_exchanges(N):
            assert L.exchange(N, Rw, NS, Rr, p)[0], ('k_front', N, name)
    for N in L.CHAN_PLANS:
        for name, Rw, NS, Rr, p in L.chan_exchanges(N):
            assert L.exchange(N, Rw, NS, Rr, p)[0], ('k_channelize', N, name)
    # the conflict-free claim for the headline geometry
    assert L.exchange(2048, 8, 8, 8, L.PADB)[1:] == (32, 16)


@pytest.mark.parametrize('N', [128, 512, 2048, 4096])
def test_pfb_tap_quantisation_matches_oracle(N):
    """The device's 16-bit PFB tap rule (mkid_pfb_effective_taps, host-only ABI call) equals the
    oracle's restatement and the product Python mirror, bit for bit."""
    import ctypes
    from mkids_sdr_amd import _lib, pfb
    from oracle.chain import pfb_prototype, quantize_pfb
    rng = np.random.default_rng(N)
    for h in (pfb_prototype(N), (rng.normal(size=4 * N) * 1e-3).astype(np.float32)):
        out = np.empty(4 * N, np.float32)
        S = ctypes.c_int32()
        L = _lib.load()
        assert L.mkid_pfb_effective_taps(h.ctypes.data_as(ctypes.c_void_p), 4, N,
                                         out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(S)) == 0
        ref, Sr = quantize_pfb(h, 4, N)
        mine, Sm = pfb.effective_taps(h)
        assert S.value == Sr == Sm
        assert np.array_equal(out.astype(np.float64), ref) and np.array_equal(mine, ref)


def test_pfb_rounding_cannot_overflow_the_int16_dot_products():
    """A prototype whose unrounded per-point sum sits just under 65535 * 2^-S but whose ROUNDED
    taps exceed it: the rule steps S down (full-scale -32768 samples aligned with the
    tap signs would otherwise wrap the int32 v_dot2 chain)."""
    import ctypes
    from mkids_sdr_amd import _lib, pfb
    from oracle.chain import quantize_pfb
    N = 16
    h = np.full(4 * N, 1e-3, np.float32)
    h[[0 * N + 3, 1 * N + 3, 2 * N + 3, 3 * N + 3]] = np.float32(16383.6)   # point 3: 4 x 16383.6
    out = np.empty(4 * N, np.float32)
    S = ctypes.c_int32()
    assert _lib.load().mkid_pfb_effective_taps(h.ctypes.data_as(ctypes.c_void_p), 4, N,
                                                out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(S)) == 0
    ref, Sr = quantize_pfb(h, 4, N)
    mine, Sm = pfb.effective_taps(h)
    assert S.value == Sr == Sm == -1
    hq = np.rint(np.ldexp(out.astype(np.float64), S.value)).reshape(4, N)
    assert np.abs(hq).sum(axis=0).max() <= 65535 and np.abs(hq).max() <= 32767
    assert 32768 * int(np.abs(hq).sum(axis=0).max()) <= 2 ** 31 - 1
    assert np.array_equal(out.astype(np.float64), ref) and np.array_equal(mine, ref)


def test_cpu_baseline_tool_runs(tmp_path):
    """tools/cpu_baseline.py (bench.py's CPU leg) on a tiny input: one-core, all-core and C1."""
    import json
    import subprocess
    import sys
    import signals
    c = signals.make_case(64, 1 << 16, seed=2, noise=30.0, pulses_per_ch=1.0)
    np.save(tmp_path / 'in.npy', c.iq)
    np.savez(tmp_path / 'cfg.npz', C=64, pfb=c.pfb, bins=c.bins, lut_i=c.lut_i, lut_q=c.lut_q,
             lpf=c.lpf12, fir=c.fir12, thr=np.full(64, -300))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, 'tools', 'cpu_baseline.py'), '--input',
                        str(tmp_path / 'in.npy'), '--cfg', str(tmp_path / 'cfg.npz'), '--one-core-samples',
                        str(1 << 15), '--all-core-samples', str(1 << 16), '--workers', '2'],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out['one_core']['value'] > 0 and out['all_cores']['cores'] == 2 and out['c1']['value'] > 0
    assert out['os_cpu_count'] >= 1 and out['cpu_model']


@pytest.mark.parametrize('N', [512, 1024, 2048, 4096])
def test_front_index_maps_and_lds_layouts(N):
    """k_front3.hip / k_front5.hip (N = 4096): the in-wave FFT staging reproduces numpy's FFT, the
    decimation combine of the select is exact (fp32 Horner form within 1e-6 of max |X| at 4096),
    and every LDS access pattern is bank-conflict free on gfx950."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location('front_layouts', os.path.join(root, 'tools', 'front_layouts.py'))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    assert m.fft_emulation() < 1e-10
    assert m.decimation_combine(N) < 1e-9
    ok = m.check_layouts(N)
    assert all(ok.values()), ok
    if N == 4096:
        assert m.horner_combine_f32() < 1e-6
        assert m.precombine_f32() < 1e-6     # k_front5's radix-2 pre-combination (round 5)
        dev, rec = m.pre_twiddle_errors()    # round 6: direct twiddles, not the W_16 recurrence
        assert dev < 1.2e-7 and rec > 3e-7


def test_resdiff_matches_reference_restatement():
    """The shim's vectorised resonator model equals iqsweep.RESDIFF (lib/iqsweep.py:824-858)."""
    from mkids_sdr_amd.roach import resdiff
    from oracle import setup_ref
    f = np.linspace(3.999e9, 4.001e9, 257)
    p = dict(Q=2.3e4, f0=4.0001e9, aleak=0.3, ph1=1.7e3, da=-0.2, ang1=0.7, Igain=1.1, Qgain=0.9,
             Ioff=0.05, Qoff=-0.12)
    ref = setup_ref.resdiff(f, **p)
    got = resdiff(f, **p)
    assert np.allclose(got.real, ref[:257], rtol=0, atol=1e-12)
    assert np.allclose(got.imag, ref[257:], rtol=0, atol=1e-12)


def test_loopback_resonator_source():
    """FpgaClient's loop-back source with resonators: a single DAC tone comes back multiplied by
    the resonator's complex transmission at the tone's RF frequency for the current LO."""
    from mkids_sdr_amd import lut
    from mkids_sdr_amd.roach import FpgaClient, resdiff
    fs, C, lo = 128e6, 64, 4.0e9
    roach = FpgaClient(n_channels=C, sample_rate=fs, gpu=False)
    f_rf = lo + 21 * fs / lut.LUT_LEN * 64
    I, Q, freqs, sf, ph = lut.define_dac_lut([f_rf], lo, np.zeros(1), fs)
    roach.cfg.dac_i, roach.cfg.dac_q = I, Q
    plain = roach._adc_lut().copy()
    r = dict(Q=1e4, f0=f_rf + 2e5, ang1=0.3, Ioff=0.1, Qoff=0.05)
    roach.set_resonators([r], lo)
    for lo_now in (lo, lo - 3e5, lo + 7e5):
        roach.set_lo(lo_now)
        h = resdiff(np.array([f_rf + (lo_now - lo)]), **r)[0]
        got = np.fft.fft(roach._adc_lut())
        ref = np.fft.fft(plain)
        k = int(np.argmax(np.abs(ref)))                 # the tone's bin: f_rf - lo at baseband
        assert abs(np.fft.fftfreq(lut.LUT_LEN, 1 / fs)[k] - (f_rf - lo)) < 1.0
        assert abs(got[k] - ref[k] * h) < 1e-9 * abs(ref[k])
        # the rest is the LUT's quantisation noise (each bin through its own transmission)
        assert np.abs(roach._adc_lut() - plain * h).max() < 0.01 * np.abs(plain).max()


def test_noise_spectrum_matches_reference_loop():
    """codecs.noise_spectrum (longsnapshot's phase-noise FFT, ROACH_Pulses.py:521-543) equals the
    loop-for-loop restatement, and at the reference's 2^20-sample capture its bins are the
    reference's saved ch_noifreqs_0.txt."""
    from oracle import replay as oreplay
    x = np.random.default_rng(3).normal(0, 5.0, 1 << 20) + 12.0
    f, s = codecs.noise_spectrum(x)
    f2, s2 = oreplay.noise_spectrum_loop(x)
    assert np.array_equal(f, f2)
    assert np.allclose(s, s2, rtol=1e-12, atol=1e-9)
    ref = np.loadtxt(os.path.join(GOLD, 'ch_noifreqs_0.txt'))
    assert np.allclose(f, ref, rtol=0, atol=1e-12)
    raw = np.array([-25736, -1, 0, 1, 25736, 12345], np.int64)
    assert np.array_equal(codecs.decode_qdr(raw.astype('>i2').tobytes()), raw)


def test_py2_str_reproduces_reference_text_files():
    """The reference writes its snapshot files with Python 2 str(q) per line (ROACH_Pulses.py:476-536);
    codecs.py2_str reproduces both of the reference's own saved files byte for byte."""
    from mkids_sdr_amd.codecs import py2_str
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for name in ('ch_noifreqs_0.txt', 'ch_snap_0.txt'):
        text = open(os.path.join(root, 'tests', 'golden', name)).read()
        lines = text.splitlines()
        assert ''.join(py2_str(float(v)) + '\n' for v in lines) == text
    assert py2_str(0.0) == '0.0' and py2_str(-3.0) == '-3.0' and py2_str(1e-20) == '1e-20'
