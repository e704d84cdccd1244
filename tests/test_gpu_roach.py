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
