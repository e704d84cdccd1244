"""The N > 1 path on CPU: world_size-2 gloo process group, one synthetic feedline per rank,
packet lists gathered to rank 0 exactly (mkids_sdr_amd.feedlines.gather_packets — the same code
bench.py runs over RCCL)."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _rank_packets(rank):
    from oracle.trigger_ref import pack_wide
    rng = np.random.default_rng(100 + rank)
    n = 5 + 7 * rank
    return np.array([pack_wide(int(c), int(p), int(b), int(t)) for c, p, b, t in
                     zip(rng.integers(0, 1024, n), rng.integers(-9000, 0, n),
                         rng.integers(-500, 500, n), np.sort(rng.integers(0, 1 << 20, n)))],
                    np.uint64).view(np.int64)


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from mkids_sdr_amd.feedlines import gather_packets
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        pk = torch.from_numpy(_rank_packets(rank))
        padded = torch.cat([pk, torch.full((3,), -1, dtype=torch.int64)])  # junk past `count`
        out = gather_packets(padded, len(pk))
        if rank == 0:
            q.put([o.numpy().tolist() for o in out])
        else:
            q.put(None if out is None else 'unexpected')
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_gather_packets_gloo(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = [r for r in res if r is not None]
    assert len(got) == 1
    lists = got[0]
    assert len(lists) == world
    for r in range(world):
        assert lists[r] == _rank_packets(r).tolist()


def _stream_worker(rank, world, port, q, steps):
    """bench.py's streaming protocol on CPU: per step a new packet list is written into the
    step's slot (the slot the gather of step k-1 may still hold), the gather of step k-1 runs
    after step k is written, flush() after the last step."""
    import torch
    import torch.distributed as dist
    from mkids_sdr_amd.feedlines import PacketGather
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        cap = 64
        ev = [torch.full((cap,), -7, dtype=torch.int64) for _ in range(2)]
        cnt = [torch.zeros(2, dtype=torch.int64) for _ in range(2)]
        g = PacketGather(ev, cnt, 'gloo', 'cpu', keep_last=True)
        seen = []
        for k in range(steps):
            g.before_step(k)
            rng = np.random.default_rng(1000 * rank + k)
            n = int(rng.integers(0, 40))          # empty lists included
            vals = torch.from_numpy(rng.integers(0, 1 << 62, n))
            s = k % 2
            ev[s][:n] = vals
            cnt[s][0] = cnt[s][1] = n
            g.after_step(k)
            if rank == 0 and k >= 1:
                seen.append([t.tolist() for t in g.last])   # step k-1's lists
        g.flush()
        if rank == 0:
            seen.append([t.tolist() for t in g.last])
        q.put((rank, seen, g.total))
    finally:
        dist.destroy_process_group()


def _expected(rank, k):
    rng = np.random.default_rng(1000 * rank + k)
    n = int(rng.integers(0, 40))
    return rng.integers(0, 1 << 62, n).tolist()


@pytest.mark.parametrize('world', [2, 3])
def test_packet_gather_pipelined_gloo(world):
    import torch.multiprocessing as mp
    steps = 5
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stream_worker, args=(r, world, port, q, steps)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seen = res[0][1]
    assert len(seen) == steps
    for k in range(steps):
        assert seen[k] == [_expected(r, k) for r in range(world)], k
    assert res[0][2] == sum(len(_expected(r, k)) for r in range(world) for k in range(steps))
