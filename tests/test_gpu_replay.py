"""Device replay triggers (a12/a13) vs the oracle restatement of the reference's numpy loops."""
import numpy as np
import pytest

from oracle import replay as oreplay

pytestmark = pytest.mark.gpu


def make_phase(n, nch, seed, base_deg=10.0, noise_deg=3.0, rate=1.0 / 1500, amp_deg=60.0,
               wander=True):
    """Fix16_13 phase [n][nch]: baseline (+ slow wander) + noise + negative-going pulses."""
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    x = np.empty((n, nch), np.float64)
    for c in range(nch):
        b = base_deg + (rng.normal(0, 0.05, n).cumsum() if wander else 0)
        v = b + rng.normal(0, noise_deg, n)
        for s in np.flatnonzero(rng.random(n) < rate):
            tau = t[s:] - s
            v[s:] -= amp_deg * rng.uniform(0.5, 1.5) * np.exp(-tau / 40.0) * (1 - np.exp(-tau / 2.0))
        x[:, c] = v
    raw = np.clip(np.rint(x / (360. / 2 ** 16 * 4 / np.pi)), -25736, 25736).astype(np.int16)
    return raw


def oracle_hits(raw, fn, **kw):
    deg = raw.astype(np.float64) * 360. / 2 ** 16 * 4 / np.pi
    return [fn(deg[:, c], **kw) for c in range(raw.shape[1])]


@pytest.fixture(scope='module')
def ch(gpu):
    from mkids_sdr_amd.channelizer import Channelizer
    c = Channelizer(64, max_chunk=1 << 16)
    yield c
    c.close()


@pytest.mark.parametrize('n,nch,m,L,T,seed', [
    (16384, 64, 20, 1000, 25.0, 1),    # pulse_triggering_v2.py defaults, snapshot length
    (16384, 37, 7, 300, 12.5, 2),
    (5000, 256, 20, 1000, 8.0, 3),     # low threshold: noise hits, many skips
    (119, 5, 20, 10, 1.0, 4),          # n < start: no hits
])
def test_rolling_matches_reference_loop(ch, n, nch, m, L, T, seed):
    import torch
    from mkids_sdr_amd import replay
    raw = make_phase(n, nch, seed)
    d = torch.from_numpy(raw).cuda()
    got = replay.rolling_mean_trigger(ch, d, n, nch, nch, meanlength=m, pulselength=L, threshold=T,
                                      cap=max(64, n // L + 2))
    exp = oracle_hits(raw, oreplay.rolling_mean_trigger, meanlength=m, pulselength=L, threshold=T)
    assert got == exp
    assert sum(len(h) for h in exp) > 0 or n < 200


@pytest.mark.parametrize('n,nch,A,start,need,skip,wrap,base,seed', [
    (16384, 64, 128, 100, 300, 200, True, 170.0, 5),    # pulse_triggering.py; phase near +-180
    (32768, 16, 1024, 500, 1500, 1000, False, 10.0, 6),  # ROACH_Pulses.py contsnapshot, A > 128
    (20000, 33, 256, 100, 50, 200, True, -20.0, 7),      # need < A: stops at the last full block
])
def test_block_matches_reference_loop(ch, n, nch, A, start, need, skip, wrap, base, seed):
    import torch
    from mkids_sdr_amd import replay
    raw = make_phase(n, nch, seed, base_deg=base)
    d = torch.from_numpy(raw).cuda()
    got = replay.block_mean_trigger(ch, d, n, nch, nch, averagelength=A, threshold=25.0, start=start,
                                    need=need, skip=skip, wrap_negative=wrap, cap=n // skip + 2)
    exp = []
    deg = raw.astype(np.float64) * 360. / 2 ** 16 * 4 / np.pi
    for c in range(nch):
        try:
            exp.append(oreplay.block_mean_trigger(deg[:, c], averagelength=A, threshold=25.0, start=start,
                                                  need=need, skip=skip, wrap_negative=wrap))
        except IndexError:  # the reference loop would raise once bob // A passes the last mean
            exp.append(None)
    for c in range(nch):
        if exp[c] is not None:
            assert got[c] == exp[c], c
        else:
            nmeans = n // A
            assert all(h // A < nmeans for h in got[c])
    assert sum(len(h) for h in got) > 0


def test_replay_on_chain_raw_phase(gpu):
    """The device's own raw phase block (mkid_last_raw_phase) as replay input, no host copy."""
    import torch
    import signals
    from mkids_sdr_amd import replay
    from mkids_sdr_amd.channelizer import Channelizer
    C, S = 64, 2 ** 18
    case = signals.make_case(C, S, seed=9, pulses_per_ch=8.0)
    ch = Channelizer(C, max_chunk=S)
    try:
        ch.set_bins(case.bins)
        ch.set_dds(case.lut_i, case.lut_q)
        ch.set_lpf(case.lpf12)
        ch.set_centers(case.ic, case.qc)
        x = torch.from_numpy(np.ascontiguousarray(case.iq).reshape(-1)).cuda()
        ev = torch.empty(1 << 16, dtype=torch.int64, device='cuda')
        cnt = torch.zeros(2, dtype=torch.int64, device='cuda')
        ch.process_device(x, S, None, ev, ev.numel(), cnt)
        p, rows = ch.raw_phase_ptr()
        got = replay.rolling_mean_trigger(ch, p, rows, C, C, pulselength=200, threshold=5.0, cap=rows)
        host = ch.raw_phase()
        exp = oracle_hits(host, oreplay.rolling_mean_trigger, pulselength=200, threshold=5.0)
        assert got == exp
        assert sum(len(h) for h in exp) > 0
    finally:
        ch.close()
