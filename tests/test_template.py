"""MakeTemplate (a18) and the optimal filter: oracle restatement (CPU) and device parity (GPU).

Input pulses follow the reference's own generator FakeTemplateData (pulses.py:429-481): I = 2 -
noise + 0.25 s(t), Q = s(t) + noise, s = (1 - e^{-t/0.1}) e^{-t/65} after sample 1000, I and Q
rolled independently by round(N(0,1)*10) (as the reference does), float32 rows of 2000.
"""
import numpy as np
import pytest

from oracle import template_ref


def fake_pulses(n, seed, bad_every=0, big_every=0):
    rng = np.random.default_rng(seed)
    I = np.zeros((n, 2000), np.float32)
    Q = np.zeros((n, 2000), np.float32)
    idx = np.arange(1000, dtype='float32')
    shape = (1.0 - np.exp(-idx / 0.1)) * np.exp(-idx / 65.0)
    for j in range(n):
        i = np.zeros(2000)
        q = np.zeros(2000)
        amp = 10.0 if (big_every and j % big_every == 3) else 1.0
        i[1000:2000] = shape * 0.25 * amp
        q[1000:2000] = shape * amp
        i += 2.0 - rng.normal(size=2000) * .01
        q += rng.normal(size=2000) * .01
        if bad_every and j % bad_every == 5:      # baseline step: fails the baseline check
            q[1500:] += 0.3
        i = np.roll(i, int((rng.normal() * 10.0) + 0.5))
        q = np.roll(q, int((rng.normal() * 10.0) + 0.5))
        I[j], Q[j] = i, q
    return I, Q


def test_oracle_template_on_fake_pulses():
    I, Q = fake_pulses(300, 1, bad_every=50, big_every=40)
    r = template_ref.make_template(I, Q)
    assert 20.0 < r['pm'] < 28.0                 # atan2(1, 2.25) = 24 deg peak
    assert 0 < r['count'] <= 300 and r['count1'] > 200
    assert abs(r['pstart'] - 1000) < 15 and 0.9 < r['template'].max() <= 1.0 + 1e-12
    assert r['flag'] == 1                        # count < 500
    g = template_ref.optimal_filter(r['template'], r['noise'])
    assert g.shape == (100,) and np.isfinite(g).all()


@pytest.mark.gpu
@pytest.mark.parametrize('n,seed', [(1200, 2), (257, 3)])
def test_device_template_matches_oracle(gpu, n, seed):
    from mkids_sdr_amd import template
    from mkids_sdr_amd.channelizer import Channelizer
    I, Q = fake_pulses(n, seed, bad_every=97, big_every=61)
    ref = template_ref.make_template(I, Q)
    ch = Channelizer(64, max_chunk=1 << 14)
    try:
        got = template.make_template(ch, I, Q)
        assert got['count1'] == ref['count1'] and got['count'] == ref['count']
        assert got['flag'] == ref['flag'] and got['pstart'] == ref['pstart']
        assert abs(got['pm'] - ref['pm']) < 1e-4 and abs(got['pdev'] - ref['pdev']) < 1e-4
        np.testing.assert_allclose(got['template'], ref['template'], rtol=0, atol=2e-5)
        np.testing.assert_allclose(got['noise'], ref['noise'], rtol=2e-4, atol=1e-9 * ref['noise'].max())
        g_ref = template_ref.optimal_filter(ref['template'], ref['noise'])
        g = template.optimal_filter(ch, got['d_template'], got['d_noise'])
        np.testing.assert_allclose(g, g_ref, rtol=0, atol=1e-3 * np.abs(g_ref).max())
        taps, taps12 = template.matched_fir_taps(g)
        assert len(taps12) == 26 and np.abs(taps12).max() <= 2047
        # exactness of the device arithmetic itself, independent of the oracle
        g2 = template.optimal_filter(ch, ref['template'], ref['noise'])
        np.testing.assert_allclose(g2, g_ref, rtol=1e-9, atol=1e-12 * np.abs(g_ref).max())
    finally:
        ch.close()


@pytest.mark.gpu
def test_device_template_no_pulses_is_loud(gpu):
    from mkids_sdr_amd import _lib, template
    from mkids_sdr_amd.channelizer import Channelizer
    I = np.full((20, 2000), 2.0, np.float32)
    Q = np.zeros((20, 2000), np.float32)
    ch = Channelizer(64, max_chunk=1 << 14)
    try:
        with pytest.raises(_lib.MkidError):
            template.make_template(ch, I, Q)
    finally:
        ch.close()
