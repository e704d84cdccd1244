"""The N > 1 feedline path on real hardware, world_size 2 over gloo: each rank runs its own
synthetic feedline (different seed) at config 3/4's per-feedline geometry (1024 ch, N = 2048)
through the HIP channeliser + trigger on cuda:0, checks its packets against the oracle trigger on
its own Fix16_13 phase, and the packet lists are gathered to rank 0 with
mkids_sdr_amd.feedlines.gather_packets. gloo's gather takes host tensors, so the lists cross as
CPU tensors here; bench.py's pipelined gather (test_gpu_bench_multi.py) moves device buffers
with backend nccl. Both ranks share the box's single GPU (2 processes, well inside the per-card
limit)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    for p in (ROOT, os.path.join(ROOT, 'tests')):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import signals
    from oracle import trigger as otrig
    from mkids_sdr_amd.channelizer import Channelizer
    from mkids_sdr_amd.feedlines import gather_packets

    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        C, S = 1024, 2 ** 20
        case = signals.make_case(C, S, seed=11 + rank, pulses_per_ch=0.5, window_phase=60)
        quiet = signals.make_case(C, S, seed=11 + rank, pulses_per_ch=0)
        thr = signals.thresholds_from_quiet(quiet, signals.oracle_chain(quiet).process(quiet.iq)['raw'])
        ch = Channelizer(C, device=0, max_chunk=S)
        try:
            ch.set_pfb(case.pfb)
            ch.set_bins(case.bins)
            ch.set_dds(case.lut_i, case.lut_q)
            ch.set_lpf(case.lpf12)
            ch.set_fir(case.fir12)
            ch.set_centers(case.ic, case.qc)
            ch.set_thresholds(thr)
            _, ev = ch.process(case.iq)
            raw = ch.raw_phase()
        finally:
            ch.close()
        ev_ref, _, _ = otrig.Trigger(C, case.fir12, thr).run(raw.astype(np.int64))
        local_ok = sorted(int(e) for e in ev) == sorted(int(e) for e in ev_ref) and len(ev) > 0
        mine = ev.view(np.int64)
        out = gather_packets(torch.from_numpy(mine.copy()), len(mine))
        gathered = None if out is None else [o.numpy().tolist() for o in out]
        q.put((rank, local_ok, mine.tolist(), gathered))
    finally:
        dist.destroy_process_group()


def test_two_feedlines_gather_gloo():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=100) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, local_ok, _, _ in res:
        assert local_ok, 'rank %d packets differ from the oracle trigger' % rank
    gathered = res[0][3]
    assert res[1][3] is None
    assert gathered == [res[r][2] for r in range(world)]
    assert gathered[0] != gathered[1]  # different feedlines
