#!/usr/bin/env python3
"""CPU checks of k_front3.hip's pair ring (run by tests/test_host.py).

1. Integer emulation of the ring over a stream: the prologue and per-iteration refills exactly as
   the kernel stages them (refill thread -> plane index pair_owner_index(g'), `prev` kept in
   registers, P(s) written into slot s mod 9 after the iteration's reads), then every PFB point of
   every frame evaluated from the pair words the transform lanes read (ds_read_b128 at entry
   ring3_idx, taps (h0, h1) against P(s), (h2, h3) against P(s + 4)) must equal the direct
   definition sum_tau h_tau x[(k + 1) M - T N + tau N + p] (K1) bit for bit, and no
   slot may be overwritten while an iteration still reads it.
2. gfx950 bank-conflict freedom (MI355X_MICROARCH.md §LDS) of the refill's ds_write_b64 (4 x 16
   contiguous lanes, bank (a/4) mod 32) and the PFB's ds_read_b128 (its 4 x 16 lane groups, bank
   (a/4) mod 64).
"""
import numpy as np

N, M, NW, T, RS = 2048, 1024, 4, 4, 9


def ring3_idx(i):
    return 128 * (i >> 7) + 2 * (i & 63) + ((i >> 6) & 1)


def pair_owner_index(g):
    return 128 * (g >> 7) + ((g >> 1) & 63) + 64 * (g & 1)


def pair_ring_emulation(n_iter=12, seed=0):
    """Returns (max |PFB(pair ring) - PFB(direct)|, hazard count). Hops are indexed relative to
    k_start; hop h covers samples h M .. h M + M - 1 of x (x[0] = sample -8 M)."""
    rng = np.random.default_rng(seed)
    H0 = 8                                          # x index of hop h is (h + H0) M
    nh = 2 * n_iter + 16
    I = rng.integers(-32768, 32768, size=nh * M)
    Q = rng.integers(-32768, 32768, size=nh * M)
    taps = rng.integers(-32768, 32768, size=(N, T))  # int16 taps per point (any values: exact)

    def hop(h):
        return (h + H0) * M

    ring = np.zeros((RS, M, 2, 2), np.int64)         # [slot][entry][I/Q pair][lo, hi]
    written = {}                                     # slot -> pair-hop it holds

    def pair_put(s, prev_h, cur_h, qh):
        slot = s % RS
        for g in range(256):
            i = pair_owner_index(g)
            assert ring3_idx(i) == g
            for u in range(4):
                o = 4 * i + u
                ring[slot, u * 256 + g, 0] = (I[hop(prev_h) + o], I[hop(cur_h) + o])
                ring[slot, u * 256 + g, 1] = (Q[hop(prev_h) + o], Q[hop(cur_h) + o])
        written[slot] = s

    # prologue (both refill hops qh = 0, 1), kernel's m loop
    for qh in (0, 1):
        prev = None
        for m in range(5):
            if qh == 0 and m == 0:
                continue
            h = -8 + 2 * m + qh
            s = h - 2
            if m > 0 and s >= -7:
                pair_put(s, prev, h, qh)
            prev = h
    err, hazards = 0, 0
    for t in range(n_iter):
        k = 2 * t                                    # frames k, k + 1 (relative to k_start)
        reads = set()
        for slot_ in range(2):
            kk = k + slot_
            for w in range(NW):
                for L in range(64):
                    for r in range(8):
                        hi, j = r >> 2, r & 3
                        s0 = kk - 7 + hi
                        e = ring3_idx(64 * j + L)
                        p = NW * (64 * r + L) + w
                        got = []
                        for comp in range(2):
                            acc = 0
                            for half, s in enumerate((s0, s0 + 4)):
                                reads.add(s)
                                if written.get(s % RS) != s:
                                    hazards += 1
                                lo, hiw = ring[s % RS, w * 256 + e, comp]
                                acc += taps[p, 2 * half] * lo + taps[p, 2 * half + 1] * hiw
                            got.append(acc)
                        ref = [0, 0]
                        for tau in range(T):
                            xs = hop(kk + 1) - T * N + tau * N + p
                            ref[0] += taps[p, tau] * I[xs]
                            ref[1] += taps[p, tau] * Q[xs]
                        err = max(err, abs(got[0] - ref[0]), abs(got[1] - ref[1]))
        # the iteration's refill: P(k + qh) from hops k + qh (kept) and k + 2 + qh (loaded)
        for qh in (0, 1):
            s = k + qh
            assert (s % RS) not in {x % RS for x in reads}, 'refill overwrites a slot read this iteration'
            pair_put(s, k + qh, k + 2 + qh, qh)
    return err, hazards


def _conflict_degree(addr_dw, ndw, groups, nbanks):
    deg = 1
    for g in groups:
        banks = {}
        for L in g:
            for d in range(ndw):
                a = addr_dw(L) + d
                banks.setdefault(a % nbanks, set()).add(a)
        deg = max(deg, max(len(v) for v in banks.values()))
    return deg


def layout_ok():
    w64 = [range(16 * g, 16 * g + 16) for g in range(4)]
    r128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
            list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
    r128 += [[x + 32 for x in g] for g in r128]
    ok = {}
    # refill: wave (rw & 3) lane L writes entry g' = (rw & 3) 64 + L of plane u (8 B each)
    ok['pair_write'] = max(_conflict_degree(lambda L, b=b, u=u: 2 * (u * 256 + b * 64 + L), 2, w64, 32)
                           for b in range(4) for u in range(4)) == 1
    # PFB: lane L reads entries 2 L, 2 L + 1 (+ 128 for j = 2, 3) of plane w (16 B)
    ok['pair_read'] = max(_conflict_degree(lambda L, w=w, jp=jp: 2 * (w * 256 + 128 * jp + 2 * L), 4, r128, 64)
                          for w in range(4) for jp in range(2)) == 1
    ok['owner_bijective'] = sorted(pair_owner_index(g) for g in range(256)) == list(range(256))
    return ok


if __name__ == '__main__':
    print('pair ring emulation (max error, hazards):', pair_ring_emulation())
    print(layout_ok())
