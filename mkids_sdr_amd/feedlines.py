"""Multi-feedline orchestration: one feedline (ADC stream, C channels) per GPU, one process per
GPU, and the path's single exchange step — the photon-packet gather to rank 0.

The reference runs one ROACH per feedline with no inter-board traffic and funnels every board's
packet stream into one PacketMaster on the host (PacketMaster.c:245-405, 577-625). Here each rank
processes its own feedline end to end on its own GPU; the per-rank uint64 packet lists then move
to rank 0 over torch.distributed (RCCL over xGMI with backend 'nccl', gloo on CPU). The volume is
~MB/s per GPU, so this is latency-, not bandwidth-bound: one exchange of the counts and one gather
of the lists padded to the longest.

`gather_packets` is the blocking one-shot form. `PacketGather` is the streaming form bench.py
runs: the gather of step k is issued on a side stream after step k+1's kernels are queued, so it
overlaps the next step's DSP instead of draining the GPU between steps (the reference's
PacketMaster likewise reads one ROACH's finished BRAM half while the board fills the other,
PulseServer.c:318-386).
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


class PacketGather:
    """Pipelined per-step photon-list gather for a feedline-per-GPU run.

    The caller owns `slots` (>= 2) packet buffers and count pairs on the device (the d_events /
    d_counts of mkid_process_device). Per step k:

        gather.before_step(k)        # the main stream waits until slot k's previous gather is done
        ch.process_device(..., events[k % slots], ..., counts[k % slots])
        gather.after_step(k)         # counts -> pinned host copy, event recorded; then gathers
                                     # step k-1 (its kernels finished before step k's started)
    and gather.flush() after the last step.

    Host side, the only wait is on step k-1's completion event (the GPU is already running step
    k). The counts are exchanged over a CPU (gloo) group; the lists move with `backend`:
      'nccl': device buffers gathered by RCCL on a side stream (the NCCL stream waits on the side
              stream, which waits on step k-1's event, not on the main stream);
      'gloo': the valid prefix is copied to pinned host memory on the side stream and gathered
              over gloo (a one-GPU box can run N ranks this way: RCCL needs one GPU per rank).
    On `dst`, `last` holds the most recent gathered lists (CPU int64 tensors, index = rank) and
    `total` the packets gathered so far.
    """

    def __init__(self, events, counts, backend, device, dst=0, ctrl_group=None, keep_last=True):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.events, self.counts = list(events), list(counts)
        self.slots = len(self.events)
        if self.slots < 2 or len(self.counts) != self.slots:
            raise ValueError('PacketGather needs >= 2 equally many event and count slots')
        if backend not in ('nccl', 'gloo'):
            raise ValueError('backend must be nccl or gloo')
        self.backend = backend
        self.device = torch.device(device)
        self.cuda = self.device.type == 'cuda'
        if backend == 'nccl' and not self.cuda:
            raise ValueError('the nccl gather moves device buffers')
        self.dst = dst
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        # CPU control channel for the counts (the default group when it is gloo already)
        self.ctrl = ctrl_group
        self.h_counts = torch.zeros((self.slots, 2), dtype=torch.int64)
        if self.cuda:
            self.h_counts = self.h_counts.pin_memory()
            self.done_ev = [torch.cuda.Event() for _ in range(self.slots)]   # step k finished
            self.side = torch.cuda.Stream(self.device)
        self.free_ev = [None] * self.slots                                   # slot k's gather done
        self.pending = []          # steps queued but not yet gathered
        self.keep_last = keep_last
        self._last = None
        self.last_counts = None
        self.total = 0
        self.host_buf = None

    @property
    def last(self):
        """The most recently gathered lists on `dst` (CPU int64 tensors, index = rank), else None."""
        if self._last is None:
            return None
        if self.cuda:
            self.side.synchronize()
        return [t.cpu() for t in self._last]

    def before_step(self, k):
        s = k % self.slots
        if self.free_ev[s] is not None:
            self.torch.cuda.current_stream(self.device).wait_event(self.free_ev[s])
            self.free_ev[s] = None

    def after_step(self, k):
        s = k % self.slots
        if self.cuda:
            self.h_counts[s].copy_(self.counts[s], non_blocking=True)
            self.done_ev[s].record(self.torch.cuda.current_stream(self.device))
        else:
            self.h_counts[s].copy_(self.counts[s])
        self.pending.append(k)
        while len(self.pending) > 1:
            self._gather(self.pending.pop(0))

    def flush(self):
        while self.pending:
            self._gather(self.pending.pop(0))
        if self.cuda:
            self.side.synchronize()

    def _gather(self, k):
        torch, dist = self.torch, self.dist
        s = k % self.slots
        if self.cuda:
            self.done_ev[s].synchronize()
        produced, written = (int(v) for v in self.h_counts[s].tolist())
        if produced > written:
            raise RuntimeError('rank %d step %d: %d packets produced, only %d fit the buffer'
                               % (self.rank, k, produced, written))
        cnt = torch.tensor([written], dtype=torch.int64)
        allc = [torch.zeros_like(cnt) for _ in range(self.world)]
        dist.all_gather(allc, cnt, group=self.ctrl)
        counts = [int(c.item()) for c in allc]
        width = max(max(counts), 1)
        ev = self.events[s]
        if width > ev.numel():
            raise RuntimeError('gather width %d exceeds the packet buffer (%d)' % (width, ev.numel()))
        if not self.cuda:                     # CPU feedlines (tests): gloo on the buffers directly
            recv = [torch.empty(width, dtype=torch.int64) for _ in range(self.world)] \
                if self.rank == self.dst else None
            dist.gather(ev[:width].contiguous(), recv, dst=self.dst)
            if recv is not None and self.keep_last:
                self._last = [r[:n].clone() for r, n in zip(recv, counts)]
        else:
            with torch.cuda.stream(self.side):
                self.side.wait_event(self.done_ev[s])
                if self.backend == 'nccl':
                    recv = [torch.empty(width, dtype=torch.int64, device=self.device)
                            for _ in range(self.world)] if self.rank == self.dst else None
                    dist.gather(ev[:width], recv, dst=self.dst)
                    if recv is not None and self.keep_last:
                        self._last = [r[:n] for r, n in zip(recv, counts)]   # device; copied on demand
                else:
                    if self.host_buf is None or self.host_buf.numel() < width:
                        self.host_buf = torch.empty(max(width, 1 << 16), dtype=torch.int64).pin_memory()
                    send = self.host_buf[:width]
                    send.copy_(ev[:width], non_blocking=True)
                    self.side.synchronize()
                    recv = [torch.empty(width, dtype=torch.int64) for _ in range(self.world)] \
                        if self.rank == self.dst else None
                    dist.gather(send, recv, dst=self.dst)
                    if recv is not None and self.keep_last:
                        self._last = [r[:n].clone() for r, n in zip(recv, counts)]
                fe = torch.cuda.Event()
                fe.record(self.side)
                self.free_ev[s] = fe
        self.last_counts = counts
        self.total += sum(counts)
