"""The reference's ChannelizerControls flow, unchanged in shape, driving the GPU through the
FpgaClient register shim on a DAC->ADC loop-back: define_LUTs -> toggleDAC -> rotateLoops
(ROACH_Setup.py:395-671) -> loadFIRcoeffs / loadThresholds (ROACH_Pulses.py:59-299) ->
snapshot / readPulses."""
import os

import numpy as np
import pytest

from mkids_sdr_amd import codecs
from mkids_sdr_amd.roach import FpgaClient, RoachPulses, RoachSetup

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def test_setup_rotate_threshold_flow(gpu):
    C = 256
    roach = FpgaClient(n_channels=C, noise_sigma=40.0, seed=3)
    roach.progdev('pulse_trigger_2022_Jan_24_1322.bof')
    rng = np.random.default_rng(9)
    freqs = list(4.0e9 + rng.choice(np.arange(-250, 250), 16, replace=False) * 1e6 + 15625.0)
    rs = RoachSetup(roach, freqs, 4.0e9, n_channels=C)
    rs.define_LUTs()
    rs.toggleDAC()
    I, Q = rs.read_avg_iq()
    amp = np.hypot(I[:16], Q[:16])
    assert np.all(amp > 50), amp               # every tone lands in its channel
    assert np.all(np.hypot(I[16:], Q[16:]) < 0.2 * amp.min())
    rs.rotateLoopsReady()
    phase, _ = roach.run(2048)
    tone_phase = np.angle(np.exp(1j * phase[64:, :16]).mean(0))
    assert np.abs(tone_phase).max() < 0.05, tone_phase   # loops rotated to phase 0

    rp = RoachPulses(roach, 16, np.loadtxt(os.path.join(GOLD, 'fir', 'matched_30us.txt')),
                     n_channels=C)
    rp.loadFIRcoeffs()
    thr = rp.loadThresholds()
    assert all(-25736 <= t < 0 for t in thr)
    assert np.array_equal(roach.cfg.thr[:16], thr)
    snap = rp.snapshot_raw(0, steps=2)
    assert len(snap) == 2 * 2 * 1024 and np.abs(snap).max() < 2000   # near 0 after rotation
    pulses = rp.readPulses(steps=2)
    assert sum(len(v) for v in pulses.values()) < 50   # noise only: few or no triggers


def _ref_iq_decode(buf):
    """pulse_triggering_IQ.py:121-147 verbatim in spirit: hex strings per byte, nibble slicing."""
    def twos_comp(val, bits):
        if (val & (1 << (bits - 1))) != 0:
            val = val - (1 << bits)
        return val
    hx = ["0x{:02x}".format(b) for b in buf]
    I, Q = [], []
    for k in range(len(buf) // 16):
        I.append(twos_comp(int(hx[6 + 16 * k][3] + hx[7 + 16 * k][2:4] + hx[8 + 16 * k][2], 16), 16))
        I.append(twos_comp(int(hx[11 + 16 * k][3] + hx[12 + 16 * k][2:4] + hx[13 + 16 * k][2], 16), 16))
        Q.append(twos_comp(int(hx[9 + 16 * k][2:4] + hx[10 + 16 * k][2:4], 16), 16))
        Q.append(twos_comp(int(hx[14 + 16 * k][2:4] + hx[15 + 16 * k][2:4], 16), 16))
    return np.array(I), np.array(Q)


def test_snapshot_registers_readback(gpu):
    """conv_phase_snapIQ_bram / conv_phase_snapPhase_bram / qdr0_memory served from the GPU and
    decoded the way the reference scripts decode them."""
    import struct
    C = 256
    roach = FpgaClient(n_channels=C, noise_sigma=20.0, seed=5)
    roach.progdev('pulse_trigger_2022_Jan_24_1322.bof')
    freqs = list(4.0e9 + np.array([-120, -40, 30, 95]) * 1e6 + 15625.0)
    rs = RoachSetup(roach, freqs, 4.0e9, n_channels=C)
    rs.define_LUTs()
    rs.toggleDAC()
    rs.read_avg_iq()
    rs.rotateLoopsReady()
    rs.loadIQcenters()
    ch = 1
    roach.write_int('conv_phase_ch_we_IQ', ch)
    L_IQ = 1024
    I, Q = _ref_iq_decode(roach.read('conv_phase_snapIQ_bram', 4 * L_IQ))
    assert len(I) == L_IQ // 2
    Ic, Qc = roach.cfg.ic[ch], roach.cfg.qc[ch]
    ph = -360 * np.arctan2(Q - Qc, I - Ic) / (2 * np.pi)     # pulse_triggering_IQ.py:152
    assert np.abs(np.hypot(I - Ic, Q - Qc)).mean() > 50       # on the loop, not at its centre
    assert np.abs(np.median(ph)) < 5.0                        # rotated loop: phase ~ 0
    roach.write_int('conv_phase_ch_we_Phase', ch)
    buf = roach.read('conv_phase_snapPhase_bram', 4 * 512)
    raw = [struct.unpack('>h', buf[4 * m + 2:4 * m + 4])[0] for m in range(512)]  # v2.py:93
    assert np.abs(np.median(raw)) < 1000
    roach.write_int('ch_we', ch)
    q = roach.read('qdr0_memory', 4 * 1024)
    vals = struct.unpack('>%dh' % 2048, q)                     # ROACH_Pulses.py:471
    assert len(vals) == 2048 and np.abs(np.median(vals)) < 1000


def _iq_tone_client(C=256, seed=7):
    """A loop-back feedline with four tones, LUTs defined and the DAC on; no rotation and no
    centres, so arctan2(Q, I) of the low-pass output is the phase the device computes."""
    roach = FpgaClient(n_channels=C, noise_sigma=40.0, seed=seed)
    roach.progdev('pulse_trigger_2022_Jan_24_1322.bof')
    freqs = list(4.0e9 + np.array([-120, -40, 30, 95]) * 1e6 + 15625.0)
    rs = RoachSetup(roach, freqs, 4.0e9, n_channels=C)
    rs.define_LUTs()
    rs.toggleDAC()
    roach.run(64)        # the DAC has been on a while: the filters are past their start-up rows
    return roach


def _readouttester(roach, ch_we, ch_we_phase, steps, L):
    """readouttesterIQ.py:34-83 through the shim: arm I, Q and phase together, read 4L bytes of
    each BRAM per step, one '>h' per word at bytes [2:4]; phase_cpu = arctan2(Qraw, Iraw),
    phase_fpga = phaseraw * 360 / 2^16 * 4 / pi (both returned in radians here)."""
    import struct
    roach.write_int('conv_phase_ch_we_IQ', ch_we)
    roach.write_int('conv_phase_ch_we_Phase', ch_we_phase)
    bin_i, bin_q, bin_p = b'', b'', b''
    for _ in range(steps):
        for name, v in (('conv_phase_startSnapI', 0), ('conv_phase_startSnapQ', 0),
                        ('conv_phase_startSnapPhase', 0), ('conv_phase_snapI_ctrl', 1),
                        ('conv_phase_snapQ_ctrl', 1), ('conv_phase_snapPhase_ctrl', 1),
                        ('conv_phase_snapI_ctrl', 0), ('conv_phase_snapQ_ctrl', 0),
                        ('conv_phase_snapPhase_ctrl', 0), ('conv_phase_startSnapI', 1),
                        ('conv_phase_startSnapQ', 1), ('conv_phase_startSnapPhase', 1)):
            roach.write_int(name, v)
        bin_i += roach.read('conv_phase_snapI_bram', 4 * L)
        bin_q += roach.read('conv_phase_snapQ_bram', 4 * L)
        bin_p += roach.read('conv_phase_snapPhase_bram', 4 * L)
    n = steps * L
    Iraw = np.array([struct.unpack('>h', bin_i[4 * m + 2:4 * m + 4])[0] for m in range(n)])
    Qraw = np.array([struct.unpack('>h', bin_q[4 * m + 2:4 * m + 4])[0] for m in range(n)])
    praw = np.array([struct.unpack('>h', bin_p[4 * m + 2:4 * m + 4])[0] for m in range(n)])
    phase_cpu = 360 * np.arctan2(Qraw, Iraw) / (2 * np.pi)
    phase_fpga = praw * 360. / 2 ** 16 * 4 / np.pi
    return Iraw, Qraw, praw, np.deg2rad(phase_cpu), np.deg2rad(phase_fpga)


@pytest.mark.parametrize('steps,L', [(15, 16), (1, 2 ** 15)])
def test_readouttester_iq_vs_phase(gpu, steps, L):
    """The reference's CPU-vs-firmware parity probe (readouttesterIQ.py:34-88) run
    unmodified in shape through FpgaClient: the I/Q snapshot and the phase snapshot of the same
    channel come from one capture, and the host's arctan2(Qraw, Iraw) equals the device's
    Fix16_13 phase within half an LSB (the device's rounding of its own float phase) + 1e-5 rad
    (the phase bar) + the int16 rounding of the I/Q snapshot (|dphi| <= 0.5 sqrt2 / |IQ|).
    (15, 16) is the script's own capture; (1, 2^15) is ROACH_Pulses_IQ.snapshot's depth."""
    roach = _iq_tone_client()
    ch = 1
    Iraw, Qraw, praw, cpu, fpga = _readouttester(roach, ch, ch, steps, L)
    mag = np.hypot(Iraw, Qraw)
    assert len(Iraw) == steps * L and mag.min() > 50           # a live tone in every row
    bar = 0.5 / 8192 + 1e-5 + 0.5 * np.sqrt(2) / (mag - 1)
    d = np.abs(np.angle(np.exp(1j * (cpu - fpga))))
    assert np.all(d <= bar), 'max %.3g rad over the bar (row %d)' % ((d - bar).max(), np.argmax(d - bar))
    # the probe has power: the noise moves the phase between rows by more than the bar, so a
    # phase snapshot from other rows than the I/Q (off by one) would fail it
    shifted = np.abs(np.angle(np.exp(1j * (cpu[1:] - fpga[:-1]))))
    print('rows off by one over the bar: %.3f' % (shifted > bar[1:]).mean())
    assert (shifted > bar[1:]).any()
    # the phase BRAM's channel selects independently (readouttesterIQ.py:29-30 uses 27 / 43)
    Iraw2, Qraw2, praw2, cpu2, fpga2 = _readouttester(roach, ch, 2, 1, 64)
    assert np.abs(np.angle(np.exp(1j * (cpu2 - fpga2)))).max() > 0.1


def test_roach_pulses_iq_snapshot(gpu):
    """ROACH_Pulses_IQ.snapshot (:357-407) through RoachPulses.snapshot_iq at L = 2^15: I and Q
    come from one capture (held by the BRAMs until the next strobe: a second Q read without a
    strobe returns the same words), on the tone's loop."""
    roach = _iq_tone_client(seed=8)
    rp = RoachPulses(roach, 4, np.loadtxt(os.path.join(GOLD, 'fir', 'matched_30us.txt')), n_channels=256)
    I, Q, phase = rp.snapshot_iq(ch_we=2, steps=1, L=2 ** 15)
    assert len(I) == len(Q) == len(phase) == 2 ** 15
    mag = np.hypot(I, Q)
    assert mag.min() > 50 and mag.std() < 0.2 * mag.mean()
    again = codecs.decode_conv_phase_snap(roach.read('conv_phase_snapQ_bram', 4 * 2 ** 15))
    assert np.array_equal(again, Q)
    # the same tone's phase from the device's phase stream agrees with the snapshot's median
    roach.write_int('conv_phase_ch_we_Phase', 2)
    raw = codecs.decode_conv_phase_snap(roach.read('conv_phase_snapPhase_bram', 4 * 4096))
    ph_dev = np.rad2deg(np.angle(np.exp(1j * raw / 8192.0).mean()))
    ph_snap = np.rad2deg(np.angle(np.exp(1j * np.deg2rad(phase)).mean()))
    assert abs((ph_dev - ph_snap + 180) % 360 - 180) < 2.0


def test_pulse_ring_packetmaster_seconds(gpu):
    """§8(f)1 end to end: the device trigger feeds the firmware wire stream (us since PPS,
    end-of-second markers) into the pulses ring while startBuffer is 1; PulseServer ships the
    ring halves (PulseServer.c:151-227, 318-386) and PacketMaster bins them per pixel per second
    (PacketMaster.c:304-397, 978-1023). Over >= 2 simulated seconds the binned rows equal the
    per-packet restatement (oracle/packet_ref.py) fed with the device's own packets."""
    from mkids_sdr_amd import packets
    from oracle import packet_ref
    C, fs = 64, 1 << 21                      # 16384 phase rows per second
    N = 2 * C
    roach = FpgaClient(n_channels=C, sample_rate=fs, noise_sigma=600.0, seed=11)
    roach.progdev('pulse_trigger_2022_Jan_24_1322.bof')
    roach.packet_log = []
    freqs = list(4.0e9 + np.array([-29, -21, -13, -6, 3, 9, 17, 26]) * (fs / N))
    rs = RoachSetup(roach, freqs, 4.0e9, n_channels=C, sample_rate=fs)
    rs.define_LUTs()
    rs.toggleDAC()
    rs.rotateLoopsReady()
    rp = RoachPulses(roach, len(freqs), np.loadtxt(os.path.join(GOLD, 'fir', 'matched_30us.txt')),
                     n_channels=C)
    rp.loadFIRcoeffs()
    rp.customThresholds[:len(freqs)] = 0.0   # threshold at the baseline: noise triggers often
    rp.loadThresholds()

    roach.write_int('startBuffer', 0)        # PulseServer.c:78-80
    roach.write_int('startBuffer', 1)
    k0 = roach._wire.next_sec                # first second the ring will carry in full
    server = packets.PulseServer(roach.ring)
    pm = packets.PacketMaster(1, C, exptime=2, dataset='t0')
    sent = []
    for _ in range(64):
        roach.read_int('pulses_addr')        # time passes: pulse_rows more phase rows
        blk = server.poll()
        if blk is not None:
            sent.append(blk)
            pm.receive(0, *blk)
        if pm.done():
            break
    roach.write_int('startBuffer', 0)
    diag = dict(written=roach.ring.written, halves=len(sent), sec=pm.sec, rows=roach._j, k0=k0,
                thr=roach.cfg.thr[:len(freqs)].tolist(), packets=sum(len(e) for e, _, _ in roach.packet_log))
    assert pm.done() and pm.corrupted_eos == 0 and pm.nonpixel == 0, diag
    assert pm.photon_counts[:, :len(freqs)].min() > 50         # every tone channel, both seconds
    assert pm.photon_counts[:, len(freqs):].max() == 0         # deleted channels stay silent

    # the restatement over the device's own packets
    truth = []
    for ev, j0, n in roach.packet_log:
        f = codecs.unpack_wide(ev)
        rows = j0 - 1 + ((f['ts'] - (j0 - 1)) % (1 << 28))
        truth += list(zip(rows.tolist(), f['ch'].tolist(), f['peak'].tolist(), f['base'].tolist()))
    words = packet_ref.wire_stream(truth, fs, N, roach._j)
    eos = [i for i, w in enumerate(words) if w == packet_ref.EOS]
    words = words[eos[k0 - 1] + 1:] if k0 > 0 else words
    ref_sent = packet_ref.pulse_server(words)
    assert len(ref_sent) >= len(sent)
    for (lo, hi), (rlo, rhi) in zip(sent, ref_sent):
        assert [int(x) for x in np.frombuffer(lo, '>u4')] == rlo
        assert [int(x) for x in np.frombuffer(hi, '>u4')] == rhi
    rows, counts, _, _ = packet_ref.packet_master(ref_sent[:len(sent)], C, 2)
    assert np.array_equal(pm.photon_counts, np.array(counts))
    for p in range(len(freqs)):
        for s in range(2):
            assert [int(x) for x in pm.rows[(0, p)][s]] == rows[p][s]
            us = packets.decode_wire(pm.rows[(0, p)][s])['us']
            assert np.all(np.diff(us) > 0) and us.max() < 10 ** 6
    # the reference readPulses decodes the same ring (EOS words appear as channel 255)
    got = rp.readPulses(steps=1)
    assert set(got) <= set(range(len(freqs))) | {255}


def test_lo_sweep_loop_calibration(gpu):
    """§8(f)3: resonator IQ loops (iqsweep.RESDIFF) on the loop-back feedline; sweepLOready
    (ROACH_Setup.py:699-810) steps the LO and reads the device avgIQ at each step, findIQcenters
    puts each centre in the middle of its swept loop, loadIQcenters loads it, and
    rotateLoopsReady (:645-671, re-sweeping as the reference does) rotates every loop so the
    on-resonance phase is 0. The synthetic loop centre in channel units is K (Ioff + i Qoff),
    K = the chain's response to the tone with the resonators off; radius 0.5 |K|."""
    C, fs, lo = 64, 128e6, 4.0e9
    roach = FpgaClient(n_channels=C, sample_rate=fs, noise_sigma=4.0, seed=8)
    roach.progdev('pulse_trigger_2022_Jan_24_1322.bof')
    res_hz = fs / 2 ** 16
    offs = np.array([-40e6, -12e6, 21e6, 50e6])
    freqs = list(lo + np.round(offs / res_hz) * res_hz)
    rs = RoachSetup(roach, freqs, lo, n_channels=C, sample_rate=fs)
    rng = np.random.default_rng(2)
    res = [dict(Q=2.0e4, f0=f + 20e3, ang1=float(rng.uniform(-3, 3)), Ioff=float(rng.uniform(-.3, .3)),
                Qoff=float(rng.uniform(-.3, .3))) for f in freqs]
    rs.define_LUTs()
    rs.toggleDAC()
    rs.programLOrev2board(lo, 0)

    def chain_gain():
        roach.set_resonators([], lo)
        I, Q = rs.read_avg_iq()
        roach.set_resonators(res, lo)
        return (I + 1j * Q)[:len(freqs)]

    def check_centres(K):
        want = K * np.array([r['Ioff'] + 1j * r['Qoff'] for r in res])
        err = np.abs(rs.iq_centers[:len(freqs)] - want) / (0.5 * np.abs(K))
        assert np.all(np.abs(K) > 300), K
        assert err.max() < 0.01, err

    K = chain_gain()
    span, steps = 1.2e6, 120                  # +-3 linewidths (f0/Q = 200 kHz), 10 kHz steps
    I, Q = rs.sweepLOready(span, steps)
    assert I.shape == (len(freqs), steps) and rs.IQ_vels.shape == (len(freqs), steps - 1)
    check_centres(K)
    # the sweep traces a circle of radius 0.5 |K| about the centre
    r = np.abs(I + 1j * Q - rs.iq_centers[:len(freqs), None])
    assert np.all(np.abs(r / (0.5 * np.abs(K)[:, None]) - 1) < 0.03), r
    rs.loadIQcenters()
    assert np.allclose(roach.cfg.ic[:len(freqs)], rs.iq_centers[:len(freqs)].real, atol=8)

    rs.rotateLoopsReady(sweep=(span, steps))  # DDS rotated, loops re-swept in the new frame
    check_centres(chain_gain())
    rs.loadIQcenters()
    phase, _ = roach.run(2048)
    tone_phase = np.angle(np.exp(1j * phase[64:, :len(freqs)]).mean(0))
    assert np.abs(tone_phase).max() < 0.05, tone_phase


def test_longsnapshot_and_contsnapshot(gpu, tmp_path):
    """ROACH_Pulses.py longsnapshot (433-551) and contsnapshot (557-762) through the shim on the
    GPU: 2^19 qdr0 words = 2^20 device phase samples of one channel; the noise-FFT bins equal the
    reference's saved ch_noifreqs_0.txt (fftfreq(10485)), the spectrum equals the loop-for-loop
    restatement on the same qdr phase, and contsnapshot's device block-mean hits, windows and
    pulse numbers equal the restated loop (failsafe included)."""
    from oracle import replay as oreplay
    C = 64
    roach = FpgaClient(n_channels=C, noise_sigma=60.0, seed=5)
    roach.progdev('pulse_trigger_2022_Jan_24_1322.bof')
    freqs = [4.0e9 + 37e6 + 15625.0 * 3, 4.0e9 - 120e6]
    rs = RoachSetup(roach, freqs, 4.0e9, n_channels=C)
    rs.define_LUTs()
    rs.toggleDAC()
    rs.rotateLoopsReady()
    rp = RoachPulses(roach, 2, None, n_channels=C)
    ls = rp.longsnapshot(0, steps=1, save_dir=str(tmp_path))
    assert len(ls['qdr_phase']) == 2 ** 20 and len(ls['phase']) == 2 * 1024
    ref_freqs = np.loadtxt(os.path.join(GOLD, 'ch_noifreqs_0.txt'))
    assert ls['noiseFFTFreqs'].shape == ref_freqs.shape == (10485,)
    assert np.allclose(ls['noiseFFTFreqs'], ref_freqs, rtol=0, atol=1e-12)
    f2, n2 = oreplay.noise_spectrum_loop(ls['qdr_phase'])
    assert np.array_equal(f2, ls['noiseFFTFreqs'])
    assert np.allclose(ls['noiseFFT'], n2, rtol=1e-12, atol=1e-9)
    assert np.isfinite(ls['noiseFFT'][1:]).all()
    # the saved files are the reference's text: str(q) per line, Python 2 (12 significant digits);
    # the bins file is byte-identical to the reference's own ch_noifreqs_0.txt
    assert open(str(tmp_path / 'ch_noifreqs_0.txt')).read() == open(os.path.join(GOLD, 'ch_noifreqs_0.txt')).read()
    assert np.allclose(np.loadtxt(ls['longsnapshot_file']), ls['qdr_phase'], rtol=0, atol=5e-9)
    # noise only: a threshold of a few degrees fires on the noise tails
    sd = float(np.std(ls['qdr_phase']))
    thr = 3.5 * sd
    for maxloops in (None, 200000, 3000):
        cs = rp.contsnapshot(0, steps=1, phase_threshold=thr, averagelength_power=10, maxloops=maxloops)
        qdr = cs['qdr_phase']
        hits, pn, fin = oreplay.contsnapshot_loop(qdr, thr, 1024, (1 << 40) if maxloops is None else maxloops)
        assert cs['hits'] == hits
        assert cs['pulsenumber'] == pn
        assert np.array_equal(np.asarray(cs['phase']), np.asarray(fin))
        assert len(hits) > 3 or maxloops == 3000
    # the reference's default threshold (-20: every pass hits) over 4 snapshots (2^22 samples, ~4190
    # hits, more than any fixed cap), and a failsafe of 0 / 1 pass (the first pass always runs,
    # ROACH_Pulses.py:747-750)
    for steps, maxloops in ((4, None), (1, 0), (1, 1)):
        cs = rp.contsnapshot(0, steps=steps, phase_threshold=-20.0, averagelength_power=10, maxloops=maxloops)
        hits, pn, fin = oreplay.contsnapshot_loop(cs['qdr_phase'], -20.0, 1024,
                                                 (1 << 40) if maxloops is None else maxloops)
        assert cs['hits'] == hits and cs['pulsenumber'] == pn
        assert np.array_equal(np.asarray(cs['phase']), np.asarray(fin))
        assert len(hits) == (1 if maxloops is not None else len(cs['qdr_phase']) // 1000 - 1)
