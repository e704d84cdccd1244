"""Reference-held pins of the device path: data and vectors the reference itself
holds, run through the GPU.

* dac_lut.npz — the reference's own saved DAC/DDS LUTs (written by ROACH_Setup.py:558) written
  into dram_memory through the FpgaClient shim (ROACH_Setup.py:552-570), DAC LUT as the
  loop-back source, DDS de-interleaved with DDS_LAG 154 (setEnvironment.sh:24), C = 256,
  N = 512 (ROACH_Setup.py:507, 515): the single tone lands in the channel select_bins gives it
  (bin 100) with constant phase, equal to the float64 oracle chain within 1e-5 rad.
* ch_snap_0.txt — the reference's only real phase record (ROACH_Pulses.py:482-484) through the
  device replay trigger (pulse_triggering_v2.py:104-174 defaults) and through k_trigger
  (mkid_trigger_phase, thresholds by loadThresholds' rule, ROACH_Pulses.py:259-278), both equal
  to the oracle.
* bin_vectors.json peakfit — outputs of the reference's Utils/bin.py peakfit (bin.py:12-16),
  recorded by executing it: the device's integer peak fit, packed into the 12-bit packet field
  (ROACH_Pulses.py:852-859), is within 1 LSB of the reference's float fit.
"""
import json
import os

import numpy as np
import pytest

from mkids_sdr_amd import codecs, lut
from oracle import chain as ochain
from oracle import replay as oreplay
from oracle import trigger as otrig

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def test_reference_dac_lut_through_fpgaclient(gpu):
    from mkids_sdr_amd.roach import FpgaClient
    d = np.load(os.path.join(GOLD, 'dac_lut.npz'))
    C, N, fs = 256, 512, 512e6
    roach = FpgaClient(n_channels=C, sample_rate=fs)
    roach.progdev('pulse_trigger_2022_Jan_24_1322.bof')
    # the fixture's tone: DAC at f_base + (f_base - f) (ROACH_Setup.py:485-487) = -100 MHz, i.e.
    # readout f - f_base = +100 MHz; select_bins: round(100e6 * 512 / 512e6) = bin 100
    bins, resid = lut.select_bins([100e6] + [0.0] * (C - 1), N, fs)
    assert bins[0] == 100 and resid[0] == 0.0
    for i, b in enumerate(bins):                          # ROACH_Setup.py:545-547
        roach.write_int('bins', int(b))
        roach.write_int('load_bins', (i << 1) + 1)
        roach.write_int('load_bins', i << 1)
    roach.write('dram_memory', codecs.pack_luts(d['I_dac'], d['Q_dac'], d['I_dds'], d['Q_dds']))
    rows = 3000
    phase, _ = roach.run(rows)
    # oracle on the same loop-back samples (conj of the DAC LUT, tiled)
    idx = np.arange(rows * N) % lut.LUT_LEN
    iq = np.stack([d['I_dac'][idx], -d['Q_dac'][idx].astype(np.int64)], axis=1).astype(np.int16)
    li, lq = lut.deinterleave_dds(d['I_dds'].astype(np.int64), d['Q_dds'].astype(np.int64), C, lut.DDS_LAG)
    assert np.all(li == 32767) and np.all(lq == 0)
    lpf = codecs.fir_quantise(np.loadtxt(os.path.join(GOLD, 'fir', 'BlackmanFilter_250kHz.txt')))
    r = ochain.OracleChain(C, ochain.pfb_prototype(N), bins, li, lq, lpf).process(iq)
    err = np.abs((phase[:, 0].astype(np.float64) - r['phase'][:, 0] + np.pi) % (2 * np.pi) - np.pi)
    assert err.max() < 1e-5, err.max()
    settled = phase[64:, 0].astype(np.float64)
    assert np.ptp(settled) < 1e-4                          # a constant phase: the tone at DC
    amp = np.abs(r['y'][64:]).mean(axis=0)
    assert amp[0] > 100 * amp[1:].max()                    # only channel 0 (bin 100) sees it


def _snap_raw():
    deg = np.loadtxt(os.path.join(GOLD, 'ch_snap_0.txt'))
    raw = np.rint(deg / codecs.SCALE_TO_ANGLE).astype(np.int64)
    assert np.abs(raw * codecs.SCALE_TO_ANGLE - deg).max() < 1e-6   # exact Fix16_13 samples
    return raw


def test_ch_snap0_through_device_replay(gpu):
    import torch
    from mkids_sdr_amd import replay
    from mkids_sdr_amd.channelizer import Channelizer
    raw = _snap_raw()
    n = len(raw)
    ch = Channelizer(64, max_chunk=1 << 16)
    try:
        d = torch.from_numpy(raw.astype(np.int16).reshape(n, 1).copy()).cuda()
        deg = raw * codecs.SCALE_TO_ANGLE
        for m, L, T in [(20, 1000, 25.0), (20, 100, 5.0), (10, 50, 2.0)]:
            got = replay.rolling_mean_trigger(ch, d, n, 1, 1, meanlength=m, pulselength=L, threshold=T, cap=64)
            assert got == [oreplay.rolling_mean_trigger(deg, meanlength=m, pulselength=L, threshold=T)]
        for A, T in [(128, 25.0), (128, 5.0), (64, 2.0)]:
            got = replay.block_mean_trigger(ch, d, n, 1, 1, averagelength=A, threshold=T, cap=64)
            assert got == [oreplay.block_mean_trigger(deg, averagelength=A, threshold=T)]
    finally:
        ch.close()


def test_ch_snap0_through_device_trigger(gpu):
    from mkids_sdr_amd.channelizer import Channelizer
    raw = _snap_raw()
    C = 64
    thr0, _ = codecs.threshold_from_phase(raw)
    assert thr0 == -5913
    mf = codecs.fir_quantise(np.loadtxt(os.path.join(GOLD, 'fir', 'matched_30us.txt')))
    # the snapshot in every channel, each rotated in time and offset so the channels differ;
    # thresholds per channel from the rule, some tightened so the record's excursions fire
    block = np.stack([np.roll(raw, 37 * c) - (c % 7) * 300 for c in range(C)], axis=1)
    thr = np.array([codecs.threshold_from_phase(block[:, c])[0] // (1 + c % 4) for c in range(C)], np.int32)
    taps = np.tile(mf, (C, 1))
    for mode in (1, 0, 2):
        ch = Channelizer(C, max_chunk=1 << 20)
        try:
            ch.set_fir(taps)
            ch.set_thresholds(thr)
            ch.set_baseline(mode, 41, 82, 93623, 8192)
            got = np.concatenate([ch.trigger_phase(block[:1000]), ch.trigger_phase(block[1000:])])
        finally:
            ch.close()
        tr = otrig.Trigger(C, taps, thr, mode=mode)
        e1, _, _ = tr.run(block[:1000])
        e2, _, _ = tr.run(block[1000:])
        exp = np.concatenate([e1, e2])
        assert np.array_equal(got, exp), mode
        if mode == 1:
            assert len(exp) > 10


def test_peakfit_vectors_through_device_trigger(gpu):
    """Utils/bin.py peakfit vectors (executed reference outputs): a stream per channel shaped so
    that the trigger fires on y1 and emits on the upturn y3 with (f2, f1, f) = (y1, y2, y3)."""
    from mkids_sdr_amd.channelizer import Channelizer
    vec = json.load(open(os.path.join(GOLD, 'bin_vectors.json')))['peakfit']
    vs = [v for v in vec if v['y'][1] <= v['y'][0] and v['y'][2] > v['y'][1]
          and all(abs(int(y)) < 30000 for y in v['y'])]
    assert len(vs) >= 40
    C = 256
    vs = vs[:C]
    rows = 200
    f = np.full((rows, C), 30000, np.int64)   # armed: e = f >= thr (no baseline: mode NONE)
    thr = np.full(C, -(1 << 30), np.int32)
    for c, v in enumerate(vs):
        y1, y2, y3 = (int(y) for y in v['y'])
        f[100:103, c] = (y1, y2, y3)
        f[103:, c] = 30000
        thr[c] = y1 + 1                       # y1 < thr fires; 30000 >= thr stays armed
    taps = np.zeros((C, 26), np.int64)
    taps[:, 0] = -2048                        # f_j = clamp16((-2048 raw_j) >> 11) = -raw_j
    ch = Channelizer(C, max_chunk=1 << 20)
    try:
        ch.set_fir(taps)
        ch.set_thresholds(thr)
        ch.set_baseline(0, 41, 82, 93623, 0)
        ev = ch.trigger_phase((-f).astype(np.int16))
    finally:
        ch.close()
    u = codecs.unpack_wide(ev)
    assert len(ev) == len(vs)
    for c, v in enumerate(vs):
        k = np.flatnonzero(u['ch'] == c)
        assert len(k) == 1 and u['ts'][k[0]] == 101        # stamped at the peak sample y2
        ref_field = min(max((int(np.floor(v['out'])) >> 4) + 2048, 0), 4095)
        assert abs(int(u['peak'][k[0]]) - ref_field) <= 1, (v, u['peak'][k[0]], ref_field)
