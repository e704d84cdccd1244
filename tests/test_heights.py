"""Per-packet optimal-filter pulse height (BASELINE config 5; include/mkidgpu.h
mkid_set_pulse_filter / mkid_pulse_heights, k_heights.hip) against oracle/heights.py.

CPU: the oracle against a plain double loop, including 28-bit stamp unwrapping and windows that
leave the rows. GPU: the device heights on the device's own phase and packets, config-5 geometry
(2048 channels, N = 4096) and streamed 1024-channel fused cases with j0 > 0 and with the phase
history carried across calls;
fp32 accumulation of <= 128 products, so the bar is relative 1e-5 of sum |coeff * phase|.
"""
import numpy as np
import pytest

from oracle import heights as oh


def _pack(ch, ts):
    return np.uint64((int(ch) << oh.CH_SHIFT) | (int(ts) & oh.TS_MASK))


def _loop(phase, events, coeff, pre, j0):
    out = []
    for w in events.tolist():
        ch, ts = w >> 52, w & oh.TS_MASK
        base = max(j0 - (1 << 27), 0)
        jg = base + ((ts - (base & oh.TS_MASK)) & oh.TS_MASK)
        r0 = jg - j0 - pre
        if r0 < 0 or r0 + coeff.shape[1] > phase.shape[0]:
            out.append(np.nan)
            continue
        out.append(sum(float(coeff[ch, i]) * float(phase[r0 + i, ch]) for i in range(coeff.shape[1])))
    return np.array(out)


@pytest.mark.parametrize('j0', [0, 1000, (1 << 28) - 7, 3 << 28])
def test_oracle_heights_match_loop(j0):
    rng = np.random.default_rng(5)
    rows, C, nco, pre = 300, 8, 20, 6
    phase = rng.normal(size=(rows, C)).astype(np.float32)
    coeff = rng.normal(size=(C, nco))
    ts = j0 + np.array([0, 5, 6, 50, 200, 273, 274, 299, 320])
    ch = rng.integers(0, C, ts.size)
    ev = np.array([_pack(c, t) for c, t in zip(ch, ts)], np.uint64)
    ref = _loop(phase, ev, coeff, pre, j0)
    got = oh.pulse_heights(phase, ev, coeff, pre, j0)
    assert np.array_equal(np.isnan(ref), np.isnan(got))
    assert np.isnan(got).sum() == 4  # windows starting before row 0 (ts 0, 5) or past the end
    ok = ~np.isnan(ref)
    assert np.allclose(got[ok], ref[ok], rtol=1e-12, atol=1e-12)


def _check(phase, ev, coeff, pre, j0, got):
    ref = oh.pulse_heights(phase, ev, coeff, pre, j0)
    assert np.array_equal(np.isnan(ref), np.isnan(got))
    ok = ~np.isnan(ref)
    assert ok.sum() > 20
    chs = (ev[ok] >> np.uint64(52)).astype(np.int64)
    scale = np.array([np.abs(coeff[c]).sum() for c in chs]) * np.abs(phase).max()
    assert np.all(np.abs(got[ok] - ref[ok]) <= 1e-5 * scale + 1e-6)


def _noise_iq(S, seed):
    """Random int16 I/Q: the chain turns it into noise-like phase that crosses the thresholds
    often, which is all the pulse-height check needs (it runs on the device's own phase and
    packets; the chain itself is checked in test_gpu_parity.py)."""
    rng = np.random.default_rng(seed)
    return rng.integers(-12000, 12000, size=(S, 2), dtype=np.int16)


@pytest.mark.gpu
def test_heights_config5_fused(gpu):
    from mkids_sdr_amd.channelizer import Channelizer
    C, S = 2048, 2 ** 20                       # config 5 geometry: N = 4096, fused k_front5
    ch = Channelizer(C, max_chunk=S)
    try:
        ch.set_fir(np.tile(np.arange(26, dtype=np.int16) * 40 - 500, (C, 1)))
        ch.set_thresholds(np.full(C, -200, np.int32))
        phase, ev = ch.process(_noise_iq(S, 61))
        rng = np.random.default_rng(62)
        coeff = rng.normal(size=(C, 100)).astype(np.float32)
        ch.set_pulse_filter(coeff, pre=20)
        got = ch.pulse_heights(phase, ev)
    finally:
        ch.close()
    assert ev.size > 100
    _check(phase, ev, coeff.astype(np.float64), 20, 0, got)


@pytest.mark.gpu
def test_heights_streamed_fused_j0(gpu):
    """Two device calls through the fused front end; heights of the second call's packets on its
    own phase rows (j0 = the first call's rows), with a 128-tap filter (two passes per lane)."""
    import torch
    from mkids_sdr_amd.channelizer import Channelizer
    C, S = 1024, 2 ** 20
    ch = Channelizer(C, max_chunk=S)
    try:
        ch.set_fir(np.tile(np.arange(26, dtype=np.int16) * 40 - 500, (C, 1)))
        ch.set_thresholds(np.full(C, -200, np.int32))
        J = S // (2 * C)
        x = torch.from_numpy(_noise_iq(2 * S, 63)).cuda()
        d_ph = torch.empty((J, C), dtype=torch.float32, device='cuda')
        cap = J * C
        d_ev = torch.empty(cap, dtype=torch.int64, device='cuda')
        d_cnt = torch.zeros(2, dtype=torch.int64, device='cuda')
        torch.cuda.synchronize()
        ch.process_device(x[:S], S, d_ph, d_ev, cap, d_cnt)
        ch.process_device(x[S:], S, d_ph, d_ev, cap, d_cnt)
        rng = np.random.default_rng(64)
        coeff = rng.normal(size=(C, 128)).astype(np.float32)
        ch.set_pulse_filter(coeff, pre=40)
        torch.cuda.synchronize()
        n = int(d_cnt[0].item())
        d_h = torch.empty(max(n, 1), dtype=torch.float32, device='cuda')
        ch.pulse_heights_device(d_ph, J, J, d_ev, n, d_h)
        torch.cuda.synchronize()
        got = d_h[:n].cpu().numpy()
        phase = d_ph.cpu().numpy()
        ev = d_ev[:n].cpu().numpy().view(np.uint64)
    finally:
        ch.close()
    assert n > 100
    _check(phase, ev, coeff.astype(np.float64), 40, J, got)


@pytest.mark.gpu
def test_heights_history_across_calls(gpu):
    """Heights after every call of a stream: windows that start before a call's first row read
    the context's carried copy of the previous call's last rows, so every packet of the second
    call whose window ends inside the stream equals the oracle on the concatenated phase. The
    first call's packets whose windows ran past its last row come back NaN; passed again with the
    second call (include/mkidgpu.h: deferral) they get their heights too."""
    import torch
    from mkids_sdr_amd.channelizer import Channelizer
    C, S, pre, nco = 1024, 2 ** 20, 20, 100
    J = S // (2 * C)
    ch = Channelizer(C, max_chunk=S)
    try:
        ch.set_fir(np.tile(np.arange(26, dtype=np.int16) * 40 - 500, (C, 1)))
        ch.set_thresholds(np.full(C, -200, np.int32))
        coeff = np.random.default_rng(65).normal(size=(C, nco)).astype(np.float32)
        ch.set_pulse_filter(coeff, pre=pre)
        x = torch.from_numpy(_noise_iq(2 * S, 66)).cuda()
        phases, evs, hs = [], [], []
        deferred = np.zeros(0, np.uint64)
        for k in range(2):
            d_ph = torch.empty((J, C), dtype=torch.float32, device='cuda')
            d_ev = torch.empty(J * C, dtype=torch.int64, device='cuda')
            d_cnt = torch.zeros(2, dtype=torch.int64, device='cuda')
            ch.process_device(x[k * S:(k + 1) * S], S, d_ph, d_ev, J * C, d_cnt)
            torch.cuda.synchronize()
            n = int(d_cnt[1].item())
            ev = np.concatenate([deferred, d_ev[:n].cpu().numpy().view(np.uint64)])
            d_all = torch.from_numpy(ev.view(np.int64).copy()).cuda()
            d_h = torch.empty(max(len(ev), 1), dtype=torch.float32, device='cuda')
            torch.cuda.synchronize()
            ch.pulse_heights_device(d_ph, J, k * J, d_all, len(ev), d_h)
            torch.cuda.synchronize()
            h = d_h[:len(ev)].cpu().numpy()
            phases.append(d_ph.cpu().numpy())
            nd = len(deferred)
            evs.append(ev[nd:])
            hs.append(h[nd:])
            if k == 0:
                ts1 = (ev & np.uint64(oh.TS_MASK)).astype(np.int64)
                tail = ts1 - pre + nco > J
                assert tail.sum() > 5
                assert np.array_equal(np.isnan(h), tail | (ts1 - pre < 0))
                deferred = ev[tail]
            else:
                h_def, ev_def = h[:nd], ev[:nd]
    finally:
        ch.close()
    phase = np.concatenate(phases)
    ev2 = evs[1]
    ts = (ev2 & np.uint64(oh.TS_MASK)).astype(np.int64)
    early = (ts - pre >= J - nco) & (ts - pre < J)      # windows reaching into the first call
    assert early.sum() > 5
    assert np.all(np.isfinite(hs[1][early]))
    _check(phase, ev2, coeff.astype(np.float64), pre, 0, hs[1])
    assert np.all(np.isfinite(h_def))
    _check(phase, ev_def, coeff.astype(np.float64), pre, 0, h_def)


@pytest.mark.gpu
def test_heights_errors(gpu):
    from mkids_sdr_amd import _lib
    from mkids_sdr_amd.channelizer import Channelizer
    ch = Channelizer(64, max_chunk=2 ** 14)
    try:
        with pytest.raises(_lib.MkidError):
            ch.pulse_heights(np.zeros((4, 64), np.float32), np.zeros(1, np.uint64))  # no filter yet
        with pytest.raises(_lib.MkidError):
            ch.set_pulse_filter(np.zeros((64, 10), np.float32), pre=-1)  # negative pre-trigger
    finally:
        ch.close()
