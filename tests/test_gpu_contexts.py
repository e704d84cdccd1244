"""Context hygiene of the C ABI: several contexts in one process (and from several host threads)
on the same GPU give the results one context gives alone; the device entry point rejects calls
larger than its workspace; packets of a call are channel-major over the whole call."""
import threading

import numpy as np
import pytest

import signals
from test_gpu_parity import configure, quiet_thresholds, sort_events

pytestmark = pytest.mark.gpu


def _run(case, thr, out, key, max_chunk, splits):
    from mkids_sdr_amd.channelizer import Channelizer
    ch = Channelizer(case.C, max_chunk=max_chunk)
    try:
        configure(ch, case, thr)
        ph, ev = [], []
        for a, b in zip(splits[:-1], splits[1:]):
            p, e = ch.process(case.iq[a:b])
            ph.append(p)
            ev.append(e)
        out[key] = (np.concatenate(ph), np.concatenate(ev))
    finally:
        ch.close()


def test_two_contexts_two_threads_same_gpu(gpu):
    C, S = 256, 1 << 20
    cases = [signals.make_case(C, S, seed=s, pulses_per_ch=3.0, noise=100.0) for s in (31, 32)]
    thrs = [quiet_thresholds(C, S // 4, s) for s in (31, 32)]
    splits = [0, S // 2, S]
    alone = {}
    for i in range(2):
        _run(cases[i], thrs[i], alone, i, S, splits)
    both = {}
    ts = [threading.Thread(target=_run, args=(cases[i], thrs[i], both, i, S, splits)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for i in range(2):
        assert np.array_equal(alone[i][0], both[i][0])
        assert np.array_equal(alone[i][1], both[i][1])
        assert len(alone[i][1]) > 0
    # the two feedlines are different streams
    assert not np.array_equal(alone[0][0], alone[1][0])


def test_device_call_larger_than_workspace_is_rejected(gpu):
    import torch
    from mkids_sdr_amd import _lib
    from mkids_sdr_amd.channelizer import Channelizer
    C = 64
    ch = Channelizer(C, max_chunk=1 << 14)
    try:
        ch.set_iq_tap(3)
        n = 1 << 15
        x = torch.zeros(2 * n, dtype=torch.int16, device='cuda')
        ev = torch.empty(1024, dtype=torch.int64, device='cuda')
        cnt = torch.zeros(2, dtype=torch.int64, device='cuda')
        with pytest.raises(_lib.MkidError):
            ch.process_device(x, n, None, ev, 1024, cnt)
        ch.process_device(x, n // 2, None, ev, 1024, cnt)   # at the limit: fine
        torch.cuda.synchronize()
        assert ch.iq_tap().shape == (n // 2 // (2 * C), 2)
    finally:
        ch.close()


@pytest.mark.parametrize('front', ['auto', 'split'])
def test_packets_channel_major_over_whole_call(gpu, front):
    """The split front end cuts a call into sub-chunks; packets still come out channel-major and
    time-ascending over the whole call (one compaction per call)."""
    from mkids_sdr_amd.channelizer import Channelizer
    C = 256
    S = 600 * 2 * C          # >= 512 N: four pipeline sub-chunks on the split path
    case = signals.make_case(C, S, seed=41, pulses_per_ch=4.0, noise=100.0)
    thr = quiet_thresholds(C, S // 4, 41)
    ch = Channelizer(C, max_chunk=S, front=front)
    try:
        configure(ch, case, thr)
        _, ev = ch.process(case.iq)
    finally:
        ch.close()
    assert len(ev) > 100
    assert np.array_equal(ev, sort_events(ev))


def test_host_call_longer_than_max_chunk_is_channel_major(gpu):
    """mkid_process cuts a call longer than cfg.max_chunk into max_chunk pieces; the pieces'
    lists are merged on the host, so the whole call is channel-major and time-ascending, and the
    packets equal one call through a context whose workspace holds the whole stream."""
    from mkids_sdr_amd.channelizer import Channelizer
    C = 256
    S = 600 * 2 * C
    case = signals.make_case(C, S, seed=43, pulses_per_ch=6.0, noise=100.0)
    thr = quiet_thresholds(C, S // 4, 43)
    out = {}
    for mc in (S, S // 4):
        ch = Channelizer(C, max_chunk=mc)
        try:
            configure(ch, case, thr)
            out[mc] = ch.process(case.iq)
        finally:
            ch.close()
    ev = out[S // 4][1]
    assert len(ev) > 100
    assert np.array_equal(ev, sort_events(ev))
    assert np.array_equal(ev, out[S][1])
    assert np.array_equal(out[S // 4][0], out[S][0])


def test_adc_and_phase_streams_do_not_mix(gpu):
    """A context carries one stream: mkid_trigger_phase on a context mid-ADC-stream (or the
    reverse) fails with MKID_E_STATE instead of shifting the live stream's stamps; after
    mkid_reset_stream either kind may start."""
    from mkids_sdr_amd import _lib
    from mkids_sdr_amd.channelizer import Channelizer
    C, S = 64, 1 << 14
    case = signals.make_case(C, S, seed=44, pulses_per_ch=0.0)
    ch = Channelizer(C, max_chunk=S)
    try:
        configure(ch, case, np.full(C, -(1 << 30)))
        ch.process(case.iq)
        with pytest.raises(_lib.MkidError) as e:
            ch.trigger_phase(np.zeros((8, C), np.int16))
        assert e.value.code == _lib.MKID_E_STATE
        ch.reset()
        ch.trigger_phase(np.zeros((8, C), np.int16))
        with pytest.raises(_lib.MkidError) as e:
            ch.process(case.iq)
        assert e.value.code == _lib.MKID_E_STATE
        ch.reset()
        ch.process(case.iq)
    finally:
        ch.close()


def test_failed_call_after_planning_marks_the_stream(gpu, monkeypatch):
    """a process call that fails after its first launch was enqueued (here an injected
    failure, MKID_FAULT_LAUNCH=1) has advanced the context's stream, so the context is marked as
    carrying an ADC stream: a following mkid_trigger_phase fails with MKID_E_STATE. A call refused in
    planning (a bad size) leaves the stream kind unchanged."""
    from mkids_sdr_amd import _lib
    from mkids_sdr_amd.channelizer import Channelizer
    C, S = 64, 1 << 14
    case = signals.make_case(C, S, seed=45, pulses_per_ch=0.0)
    monkeypatch.setenv('MKID_FAULT_LAUNCH', '1')
    ch = Channelizer(C, max_chunk=S)
    monkeypatch.delenv('MKID_FAULT_LAUNCH')
    try:
        configure(ch, case, np.full(C, -(1 << 30)))
        with pytest.raises(_lib.MkidError) as e:
            ch.process(case.iq[:100])              # not a multiple of N: refused before planning
        assert e.value.code == _lib.MKID_E_ARG
        ch.trigger_phase(np.zeros((8, C), np.int16))   # still a fresh context: allowed
        ch.reset()
        with pytest.raises(_lib.MkidError) as e:
            ch.process(case.iq)                    # the injected failure after the first launch
        assert e.value.code == _lib.MKID_E_HIP and 'injected' in str(e.value)
        with pytest.raises(_lib.MkidError) as e:
            ch.trigger_phase(np.zeros((8, C), np.int16))
        assert e.value.code == _lib.MKID_E_STATE
        ch.reset()
        ch.process(case.iq)                        # the hook fires once
    finally:
        ch.close()


def test_accumulator_rearm_and_failed_call(gpu, monkeypatch):
    """every mkid_set_accumulator(1) restarts the sums (the reference strobes avgIQ_ctrl
    before each startAccumulator 1), armed or not; a process call that fails while the accumulator
    is armed invalidates it (its sums may hold part of that call): mkid_avg_iq then fails with
    MKID_E_STATE until it is re-armed."""
    from mkids_sdr_amd import _lib
    from mkids_sdr_amd.channelizer import Channelizer
    C, S = 64, 1 << 14
    case = signals.make_case(C, S, seed=46, pulses_per_ch=0.0)
    monkeypatch.setenv('MKID_FAULT_LAUNCH', '3')
    ch = Channelizer(C, max_chunk=S)
    monkeypatch.delenv('MKID_FAULT_LAUNCH')
    try:
        configure(ch, case, np.full(C, -(1 << 30)))
        ch.set_accumulator(True)
        ch.process(case.iq[:S // 2])               # launch 1: fine
        a1 = ch.avg_iq()
        ch.set_accumulator(True)                   # re-arm while armed: the sums restart
        with pytest.raises(_lib.MkidError) as e:
            ch.avg_iq()
        assert e.value.code == _lib.MKID_E_STATE   # no rows since the re-arm
        ch.process(case.iq[S // 2:])
        a2 = ch.avg_iq()
        assert not np.array_equal(a1[0], a2[0])    # the second half's own mean, not both halves'
        with pytest.raises(_lib.MkidError) as e:
            ch.process(case.iq[:S // 2])           # launch 3: the injected failure (hook = 3)
        assert e.value.code == _lib.MKID_E_HIP
        with pytest.raises(_lib.MkidError) as e:
            ch.avg_iq()
        assert e.value.code == _lib.MKID_E_STATE and 're-arm' in str(e.value)
        ch.reset()
        ch.set_accumulator(True)
        ch.process(case.iq)
        mi, mq = ch.avg_iq()
        assert np.isfinite(mi).all() and np.isfinite(mq).all()
    finally:
        ch.close()


def test_timing_mask_and_counts_written_per_call(gpu):
    """mkid_set_timing_mask with MKID_TIMING_ONLY bits times only the named kernels (bench.py's timed
    steps record events around the front end alone); d_counts is written by each call's
    compaction (no zeroing launch), so stale values in it do not leak into the next call."""
    import torch
    from mkids_sdr_amd import _lib
    from mkids_sdr_amd.channelizer import Channelizer
    C, S = 256, 1 << 20
    case = signals.make_case(C, S, seed=51, pulses_per_ch=3.0, noise=100.0)
    thr = quiet_thresholds(C, S // 4, 51)
    x = torch.from_numpy(case.iq.reshape(-1)).to('cuda')
    cap = 1 << 16
    res = []
    for junk in (0, 123456789):
        ch = Channelizer(C, max_chunk=S)
        try:
            configure(ch, case, thr)
            ev = torch.empty(cap, dtype=torch.int64, device='cuda')
            cnt = torch.full((2,), junk, dtype=torch.int64, device='cuda')
            ch.set_timing(True, kernels=['k_front'])
            ch.process_device(x, S, None, ev, cap, cnt)
            torch.cuda.synchronize()
            t = ch.timing()
            assert t['k_front'][1] == 1 and t['k_front'][0] > 0
            assert t['k_trigger'][1] == 0 and t['k_compact'][1] == 0
            ch.set_timing(True)
            c = cnt.cpu().numpy().copy()
            ch.process_device(x, S, None, ev, cap, cnt)
            torch.cuda.synchronize()
            t = ch.timing()
            assert t['k_front'][1] == 1 and t['k_trigger'][1] == 1 and t['k_compact'][1] == 1
            with pytest.raises(_lib.MkidError):   # a bit past the last kernel
                ch._chk(ch._L.mkid_set_timing_mask(ch._h, 1 << _lib.K_COUNT))
            # mkid_set_timing keeps its round-1..3 meaning, any non-zero value times
            # every kernel (the mask moved to its own entry point)
            ch._chk(ch._L.mkid_set_timing(ch._h, -1))
            ch._chk(ch._L.mkid_set_timing(ch._h, 2))
            ch.process_device(x, S, None, ev, cap, cnt)
            torch.cuda.synchronize()
            t = ch.timing()
            assert t['k_front'][1] == 1 and t['k_trigger'][1] == 1 and t['k_compact'][1] == 1
            ch.set_timing(False)
            with pytest.raises(ValueError):
                ch.set_timing(True, kernels=['no_such_kernel'])
            res.append((c, ev[:int(c[1])].cpu().numpy()))
        finally:
            ch.close()
    assert res[0][0][0] > 0 and np.array_equal(res[0][0], res[1][0])
    assert np.array_equal(res[0][1], res[1][1])
