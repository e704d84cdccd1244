#!/usr/bin/env python3
"""Select-wave channel assignment for k_front3 (N = 2048) and k_front5 (N = 4096) that minimises LDS bank conflicts of
the per-channel Y gather: a ds_read_b64 group of 32 lanes costs one LDS cycle per distinct address
on its busiest bank pair (MI355X_MICROARCH.md §LDS; Y entry i sits on bank pair i mod 32), so the
32 channels a group reads should fall on distinct pairs. Greedy: channels by class (pair) size,
each into the group whose cost rises least, then the one it leaves lowest, then the emptiest.
`python tools/lds_assign.py` prints the modelled cost; tools/kbench.py's `lib.so#a` / `lib.so#b`
relabel the bench feedline in these orders (the same physical tones, channels renumbered), which
times the gather at the reduced conflict level with the kernel unchanged (round-3 A/B:
profiles/r03/r03_h_kbench_f3_slot_order.json)."""
import numpy as np


def yswz(k):
    return k ^ ((k >> 2) & 14)


def group_cost(groups, yoff):
    tot = 0
    for g in groups:
        a = np.unique(yoff[np.asarray(g)])
        tot += int(np.bincount(a % 32, minlength=32).max())
    return tot


def assign(yoff, ng=32, gs=32):
    yoff = np.asarray(yoff)
    cls = yoff % 32
    cnt = np.bincount(cls, minlength=32)
    order = sorted(range(len(yoff)), key=lambda c: (-cnt[cls[c]], cls[c], yoff[c]))
    groups = [[] for _ in range(ng)]
    mult = np.zeros((ng, 32), int)
    seen = [set() for _ in range(ng)]
    gmax = np.zeros(ng, int)
    for c in order:
        k = cls[c]
        best = None
        for g in range(ng):
            if len(groups[g]) >= gs:
                continue
            same = int(yoff[c]) in seen[g]
            m = mult[g, k] + (0 if same else 1)
            newmax = max(gmax[g], m)
            key = (newmax - gmax[g], newmax, len(groups[g]))
            if best is None or key < best[0]:
                best = (key, g, same)
        _, g, same = best
        groups[g].append(c)
        if not same:
            seen[g].add(int(yoff[c]))
            mult[g, k] += 1
        gmax[g] = max(gmax[g], mult[g, k])
    return groups


def slot_order(bins, C=1024):
    """slot -> channel for the select threads: slot st + (C/2) q (st = 64 w + 32 h + l) is lane l
    of half h of wave w, read instruction q (the k_front3 layout: C = 1024, 8 select waves), with
    the groups chosen over all channels; group index g = (q, w, h)."""
    bins = np.asarray(bins)
    yoff = np.array([yswz(int(b) & 511) for b in bins])
    ng = C // 32
    groups = assign(yoff, ng=ng)
    perm = np.empty(C, np.int64)
    for g, members in enumerate(groups):
        q, w, h = g // (ng // 2), (g // 2) % (ng // 4), g % 2
        for l, c in enumerate(members):
            perm[64 * w + 32 * h + l + (C // 2) * q] = c
    return perm


def slot_order_blocks(bins, B=128, C=1024):
    """as slot_order, but each select wave keeps the 128 channels 128 w' .. 128 w' + 127 (its
    output stores and LO loads stay within 2-4 cache lines per instruction): the 4 read groups of
    a wave (2 halves x 2 read instructions) are chosen among its own channels."""
    bins = np.asarray(bins)
    yoff = np.array([yswz(int(b) & 511) for b in bins])
    perm = np.empty(C, np.int64)
    for blk in range(C // B):
        ch = np.arange(blk * B, (blk + 1) * B)
        groups = assign(yoff[ch], ng=B // 32, gs=32)
        for j, members in enumerate(groups):
            for l, c in enumerate(members):
                # group j of wave blk: read instruction q = j >> 1, half h = j & 1
                slot = 64 * blk + 32 * (j & 1) + l + (C // 2) * (j >> 1)
                perm[slot] = ch[c]
    return perm


def f5_groups():
    """k_front5's read groups (C = 2048): waves 0-7 of the select waves read channels
    64 w + 32 h + l + 512 q (q < 3), waves 8-11 read 1536 + 64 w' + 32 h + l + 256 q (q < 2); one group
    per (wave, half, q)."""
    g = [[64 * w + 32 * h + l + 512 * q for l in range(32)] for w in range(8) for h in range(2) for q in range(3)]
    g += [[1536 + 64 * w + 32 * h + l + 256 * q for l in range(32)] for w in range(4) for h in range(2)
          for q in range(2)]
    return g


def slot_order_f5(bins):
    """natural channel -> feedline channel for a relabelled feedline whose k_front5 read groups
    are the conflict-minimising ones (tools/kbench.py lib.so#c: the bound of the select-order
    effect with the kernel unchanged)."""
    bins = np.asarray(bins)
    yoff = np.array([yswz(int(b) & 511) for b in bins])
    groups = assign(yoff, ng=64)
    perm = np.empty(2048, np.int64)
    for members, slots in zip(groups, f5_groups()):
        for c, s in zip(members, slots):
            perm[s] = c
    return perm


def f5_key(bins):
    """k_front5's Y entry per channel (round 5 radix-2 pre-combination): yswz(bin & 511) in the
    P^s regions, s = bit 9 of the bin, 4 REG = 2304 entries apart (same bank pair, another
    address)."""
    bins = np.asarray(bins, np.int64)
    return np.array([yswz(int(b) & 511) for b in bins]) + 2304 * ((bins >> 9) & 1)


def f5_waves():
    """k_front5's select waves as (slot base, q stride, reads per thread): waves 4-11 three
    channels per thread, 12-15 two."""
    return [(64 * w, 512, 3) for w in range(8)] + [(1536 + 64 * v, 256, 2) for v in range(4)]


def slot_order_f5_waves(bins):
    """mkid_slot_order at C = 2048 (mkid_plan.cpp slot_order): each k_front5 select wave spreads
    its own channels (the natural channels of its slots) over its read groups (group j: read
    instruction j >> 1, half j & 1) with the conflict-minimising greedy on f5_key."""
    key = f5_key(bins)
    perm = np.empty(2048, np.int64)
    for base, stride, nq in f5_waves():
        ch = np.array([base + l + stride * q for q in range(nq) for l in range(64)])
        groups = assign(key[ch], ng=2 * nq, gs=32)
        for j, members in enumerate(groups):
            for l, c in enumerate(members):
                perm[base + 32 * (j & 1) + l + stride * (j >> 1)] = ch[c]
    return perm


def natural_groups(C=1024):
    return [[64 * w + 32 * h + l + (C // 2) * q for l in range(32)] for q in range(2) for w in range(C // 128)
            for h in range(2)]


if __name__ == '__main__':
    rng = np.random.default_rng(0)
    for trial in range(4):
        bins = rng.permutation(np.arange(1, 2048))[:1024]
        yoff = np.array([yswz(int(b) & 511) for b in bins])
        perm = slot_order(bins)
        pb = slot_order_blocks(bins)
        print('natural %d  assigned %d  per-wave blocks %d  (ideal 32 cycles per 32 group-reads)' % (
            group_cost(natural_groups(), yoff), group_cost(natural_groups(), yoff[perm]),
            group_cost(natural_groups(), yoff[pb])))
    bins = rng.permutation(np.arange(1, 4096))[:2048]
    yoff = np.array([yswz(int(b) & 511) for b in bins])
    print('C = 2048: natural %d  assigned %d' % (group_cost(natural_groups(2048), yoff),
                                                group_cost(natural_groups(2048), yoff[slot_order(bins, 2048)])))
    key = f5_key(bins)
    print('k_front5 (P^s key): natural %d  per-wave order %d  relabel bound %d' % (
        group_cost(f5_groups(), key), group_cost(f5_groups(), key[slot_order_f5_waves(bins)]),
        group_cost(f5_groups(), key[slot_order_f5(bins)])))
