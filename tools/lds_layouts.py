#!/usr/bin/env python3
"""LDS layout checker for the Stockham exchanges of k_front / k_channelize (fft_common.h).

A layout maps float2 index i to i + (i >> SH) * MUL. Two properties are checked per exchange:
  * linearity (CORRECTNESS): st_read / st_write address every point as one per-thread base plus
    a compile-time offset, pad(base + K) = pad(base) + pad(K); this must hold for every offset a
    pass adds, for every thread;
  * bank cycles (PERFORMANCE): LDS-array cycles of the wave instructions under the gfx950 banking
    rules of MI355X_MICROARCH.md §LDS (ds_write_b64: 4 groups of 16 lanes, bank = dword mod 32;
    ds_read_b64: 2 groups of 32 lanes, bank = dword mod 64).

    python tools/lds_layouts.py          # report for the kernels' plans
"""
import itertools

PTS = 8
FRONT_PLANS = {128: [8, 4, 4], 256: [8, 8, 4], 512: [8, 4, 4, 4], 1024: [8, 8, 4, 4], 2048: [8, 8, 8, 4]}
CHAN_PLANS = {128: [8, 4, 4], 256: [8, 8, 4], 512: [8, 8, 8], 1024: [8, 8, 4, 4], 2048: [8, 8, 8, 4],
              4096: [8, 8, 8, 8]}
PAD16 = (4, 1)
PADB = (5, 4)


def pad(i, p):
    return i + (i >> p[0]) * p[1]


def write_addrs(N, R, NS, q, r, ts, p):
    NT = N // PTS
    out = []
    for t in ts:
        j = t + q * NT
        out.append(pad((j // NS) * NS * R + (j % NS) + r * NS, p))
    return out


def read_addrs(N, R, q, r, ts, p):
    NT, NR = N // PTS, N // R
    return [pad(t + q * NT + r * NR, p) for t in ts]


def write_linear(N, R, NS, p):
    NT = N // PTS
    for q in range(PTS // R):
        for r in range(R):
            d = set()
            for t in range(NT):
                j = t + q * NT
                base = (j // NS) * NS * R + (j % NS)
                d.add(pad(base + r * NS, p) - pad(base, p))
            if d != {pad(r * NS, p)}:
                return False
    return True


def read_linear(N, R, p):
    NT, NR = N // PTS, N // R
    for q in range(PTS // R):
        for r in range(R):
            if {pad(t + q * NT + r * NR, p) - pad(t, p) for t in range(NT)} != {pad(q * NT + r * NR, p)}:
                return False
    return True


def cyc_write_b64(addr):
    tot = 0
    for g in range(0, len(addr), 16):
        banks = {}
        for a in addr[g:g + 16]:
            for d in (0, 1):
                banks.setdefault((2 * a + d) % 32, set()).add(2 * a + d)
        tot += max(len(v) for v in banks.values())
    return tot


def cyc_read_b64(addr):
    tot = 0
    for g in range(0, len(addr), 32):
        banks = {}
        for a in addr[g:g + 32]:
            for d in (0, 1):
                banks.setdefault((2 * a + d) % 64, set()).add(2 * a + d)
        tot += max(len(v) for v in banks.values())
    return tot


def exchange(N, Rw, NS, Rr, p):
    """(linear, write cycles, read cycles) per wave for one exchange; Rr = None: select reads."""
    NT = N // PTS
    waves = [range(w, min(w + 64, NT)) for w in range(0, NT, 64)]
    wc = sum(cyc_write_b64(write_addrs(N, Rw, NS, q, r, ts, p))
             for ts in waves for q in range(PTS // Rw) for r in range(Rw)) // len(waves)
    lin = write_linear(N, Rw, NS, p)
    rc = 0
    if Rr is not None:
        rc = sum(cyc_read_b64(read_addrs(N, Rr, q, r, ts, p))
                 for ts in waves for q in range(PTS // Rr) for r in range(Rr)) // len(waves)
        lin = lin and read_linear(N, Rr, p)
    return lin, wc, rc


def front_exchanges(N):
    """Exchanges of k_front<N>: (name, write radix, NS, read radix or None, layout)."""
    R = FRONT_PLANS[N]
    padb = PADB
    ex = [('A', R[0], 1, R[1], PAD16)]
    if len(R) == 4:
        ex.append(('B', R[1], R[0], R[2], padb))
        ex.append(('C', R[2], R[0] * R[1], None, PAD16))
    else:
        ex.append(('C', R[1], R[0], None, PAD16))
    return ex


def chan_exchanges(N):
    R = CHAN_PLANS[N]
    ex, NS = [], 1
    for k in range(len(R)):
        ex.append(('P%d' % (k + 1), R[k], NS, R[k + 1] if k + 1 < len(R) else None, PAD16))
        NS *= R[k]
    return ex


def main():
    for N in sorted(FRONT_PLANS):
        for name, Rw, NS, Rr, p in front_exchanges(N):
            print('k_front<%d> %s' % (N, name), 'layout', p, 'linear/write/read', exchange(N, Rw, NS, Rr, p))
    for N in sorted(CHAN_PLANS):
        for name, Rw, NS, Rr, p in chan_exchanges(N):
            print('k_channelize<%d> %s' % (N, name), 'linear/write/read', exchange(N, Rw, NS, Rr, p))
    # candidate search for exchange B at N = 2048
    best = []
    for sh, mul in itertools.product(range(3, 8), range(1, 9)):
        lin, wc, rc = exchange(2048, 8, 8, 8, (sh, mul))
        if lin:
            best.append((max(wc, 48) + rc, wc, rc, (sh, mul)))
    print('exchange B candidates (cost, write, read, layout):', sorted(best)[:5])


if __name__ == '__main__':
    main()
