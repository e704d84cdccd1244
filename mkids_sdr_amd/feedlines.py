"""Multi-feedline orchestration: one feedline (ADC stream, C channels) per GPU, one process per
GPU, and the path's single exchange step — the photon-packet gather to rank 0.

The reference runs one ROACH per feedline with no inter-board traffic and funnels every board's
packet stream into one PacketMaster on the host (PacketMaster.c:245-405, 577-625). Here each rank
processes its own feedline end to end on its own GPU; `gather_packets` then moves the per-rank
uint64 packet lists to rank 0 over torch.distributed (RCCL over xGMI with backend 'nccl', gloo
on CPU). The volume is ~MB/s per GPU, so this is latency-, not bandwidth-bound: one all_gather of
the counts and one gather of the lists padded to the longest.
"""


def gather_packets(packets, count, group=None, dst=0):
    """packets: 1-D int64 tensor with `count` valid entries (device or CPU, matching the process
    group's backend). Returns [per-rank tensors] on `dst` (index = rank = feedline), else None."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    cnt = torch.tensor([int(count)], dtype=torch.int64, device=packets.device)
    allc = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(allc, cnt, group=group)
    counts = [int(c.item()) for c in allc]
    width = max(max(counts), 1)
    buf = torch.zeros(width, dtype=torch.int64, device=packets.device)
    buf[:count] = packets[:count]
    bufs = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    return [b[:n] for b, n in zip(bufs, counts)]
