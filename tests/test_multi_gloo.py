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
