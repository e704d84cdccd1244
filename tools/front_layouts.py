#!/usr/bin/env python3
"""Checks of the fused front ends' index maps and LDS layouts (k_front3.hip at N = 512 / 1024 /
2048, k_front5.hip at N = 4096; run by tests/test_host.py on the CPU).

1. numpy emulation of one wave's 512-point FFT exactly as the kernel stages it (radix-8 over
   registers, twiddle, T1 bit swaps register<->lane bits 3-5, radix-8, twiddle, T2 through LDS
   with the i + (i >> 3) layout, radix-8): lane L, register r must end holding
   Y[(L >> 3) + 8 (L & 7) + 64 r]; and the NW-way decimation combine of the select.
2. gfx950 bank-conflict freedom (MI355X_MICROARCH.md §LDS) of every LDS access pattern:
   ds_read_b32 ring reads, ds_read_b64 tap reads, ds_write_b32/b64/b128 ring writes, the
   ds_write_b64 / ds_read_b64 T2 exchange and the ds_write_b64 Y write.
"""
import numpy as np


def fft_emulation(seed=0):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=512) + 1j * rng.normal(size=512)
    W = lambda n, e: np.exp(-2j * np.pi * e / n)
    V = np.array([[x[64 * r + L] for r in range(8)] for L in range(64)])
    dft8 = lambda V: np.fft.fft(V, axis=1)
    V = dft8(V)
    V *= W(512, np.outer(np.arange(64), np.arange(8)))
    def bitswap(V, i, j):
        U = V.copy()
        for L in range(64):
            for r in range(8):
                if ((r >> i) & 1) != ((L >> j) & 1):
                    U[L, r] = V[L ^ (1 << j), r ^ (1 << i)]
        return U
    for i in range(3):
        V = bitswap(V, i, 3 + i)
    V = dft8(V)
    V *= W(64, np.outer(np.arange(64) & 7, np.arange(8)))
    mem = np.zeros(576, complex)
    f = lambda i: i + (i >> 3)
    for L in range(64):
        for r in range(8):
            mem[f(64 * (L >> 3) + 8 * r + (L & 7))] = V[L, r]
    U = np.array([[mem[f(64 * (L >> 3) + 8 * (L & 7) + r)] for r in range(8)] for L in range(64)])
    V = dft8(U)
    Y = np.fft.fft(x)
    return max(abs(V[L, r] - Y[(L >> 3) + 8 * (L & 7) + 64 * r]) for L in range(64) for r in range(8))


def decimation_combine(N, seed=1):
    rng = np.random.default_rng(seed)
    u = rng.normal(size=N) + 1j * rng.normal(size=N)
    NW = N // 512
    Ys = [np.fft.fft(u[w::NW]) for w in range(NW)]
    k = np.arange(N)
    X = sum(np.exp(-2j * np.pi * w * k / N) * Ys[w][k % 512] for w in range(NW))
    return np.abs(X - np.fft.fft(u)).max()


def horner_combine_f32(N=4096, seed=2):
    """The 8-way select combine as two Horner chains (k_front5 before its round-5 radix-2
    pre-combination): X[b] = (Y_0 + t (Y_1 + t (Y_2 + t Y_3))) + t4 (Y_4 + t (... + t Y_7)),
    t = W_N^b and t4 = W_N^{4b} (both rounded from float64), in complex64 as the device's fp32 cmac
    chains; returns the max error relative to max |X|."""
    rng = np.random.default_rng(seed)
    u = (rng.normal(size=N) + 1j * rng.normal(size=N)) * 3e4
    NW = N // 512
    Ys = [np.fft.fft(u[w::NW]).astype(np.complex64) for w in range(NW)]
    k = np.arange(N)
    t = np.exp(-2j * np.pi * k / N).astype(np.complex64)
    t4 = np.exp(-2j * np.pi * ((4 * k) % N) / N).astype(np.complex64)
    lo, hi = Ys[3][k % 512], Ys[7][k % 512]
    for w in (2, 1, 0):
        lo = (Ys[w][k % 512] + lo * t).astype(np.complex64)
        hi = (Ys[w + 4][k % 512] + hi * t).astype(np.complex64)
    X = (lo + hi * t4).astype(np.complex64)
    ref = np.fft.fft(u)
    return float(np.abs(X - ref).max() / np.abs(ref).max())


def pre_twiddles(recurrence=False):
    """[8][64] complex64: k_front5's pre-combination twiddle for output 64 r + e, e = kl + 8 la, in
    the device's fp32 arithmetic (pre_twiddles in k_front5.hip; recurrence=True: round 5's
    wk *= W_16)."""
    f = np.float32
    a, b, h = f(0.92387953251128675613), f(0.38268343236508977173), f(0.70710678118654752440)
    e = np.arange(64)
    w0 = np.exp(-2j * np.pi * e / 1024).astype(np.complex64)
    out = np.empty((8, 64), np.complex64)
    if recurrence:
        w16 = np.complex64(np.exp(-2j * np.pi / 16))
        wk = w0.copy()
        for r in range(8):
            out[r] = wk
            wk = (wk * w16).astype(np.complex64)
        return out
    x, y = w0.real.astype(np.float64), w0.imag.astype(np.float64)
    mx, my = (x * a).astype(f), (y * a).astype(f)
    fma = lambda p, q, c: (p * np.float64(q) + np.float64(c)).astype(f)
    u1 = fma(y, b, mx) + 1j * fma(-x, b, my)
    vv = fma(-y, b, mx) + 1j * fma(x, b, my)
    u2 = ((x + y).astype(f) * h).astype(f) + 1j * ((y - x).astype(f) * h).astype(f)
    for r, t in enumerate((w0, u1, u2, -1j * vv, -1j * w0, -1j * u1, -1j * u2, -vv)):
        out[r] = t
    return out


def pre_twiddle_errors():
    """max |twiddle - exact| of the device construction and of round 5's recurrence."""
    k = 64 * np.arange(8)[:, None] + np.arange(64)[None, :]
    ex = np.exp(-2j * np.pi * k / 1024)
    return (float(np.abs(pre_twiddles() - ex).max()), float(np.abs(pre_twiddles(True) - ex).max()))


def precombine_f32(N=4096, seed=3):
    """k_front5.hip: the transform wave that holds sub-FFTs r and r + 4 writes
    P_r^s[k] = Y_r[k] + (-1)^s W_1024^k Y_{r+4}[k], k = 64 r' + e (e = kl + 8 la), with the twiddle
    W_1024^k = w0 W_16^{r'} built as k_front5's pre_twiddles (round 6): w0 = W_1024^e and
    u1 = w0 W_16, vv = w0 conj(W_16), u2 = w0 W_16^2 from fp32 constants, the quarter turns exact
    (round 5 stepped wk *= W_16, 3.5e-7 at r' = 7: pre_twiddle_errors); the select evaluates
    X[b] = (P_0 + t^2 P_2) + t (P_1 + t^2 P_3), t = W_N^b, s = bit 9 of b; complex64 throughout as
    the device; returns the max error relative to max |X|."""
    rng = np.random.default_rng(seed)
    u = (rng.normal(size=N) + 1j * rng.normal(size=N)) * 3e4
    Ys = [np.fft.fft(u[w::8]).astype(np.complex64) for w in range(8)]
    k = np.arange(512)
    tw = pre_twiddles()[k // 64, k % 64]
    P = {}
    for r in range(4):
        d = (Ys[r + 4] * tw).astype(np.complex64)
        P[(r, 0)] = (Ys[r] + d).astype(np.complex64)
        P[(r, 1)] = (Ys[r] - d).astype(np.complex64)
    b = np.arange(N)
    s = (b >> 9) & 1
    kk = b % 512
    t = np.exp(-2j * np.pi * b / N).astype(np.complex64)
    t2 = (t * t).astype(np.complex64)
    g = lambda r: np.where(s == 0, P[(r, 0)][kk], P[(r, 1)][kk])
    xa = (g(0) + t2 * g(2)).astype(np.complex64)
    xb = (g(1) + t2 * g(3)).astype(np.complex64)
    X = (xa + t * xb).astype(np.complex64)
    ref = np.fft.fft(u)
    return float(np.abs(X - ref).max() / np.abs(ref).max())


def _groups(width):
    """lane groups (one LDS cycle each) and bank count of an instruction (MI355X_MICROARCH.md)."""
    if width == 'r32':
        return [range(0, 32), range(32, 64)], 32
    if width == 'r64':
        return [range(0, 32), range(32, 64)], 64
    if width == 'w32':
        return [range(0, 32), range(32, 64)], 32
    if width == 'w64':
        return [range(16 * g, 16 * g + 16) for g in range(4)], 32
    if width == 'w128':
        return [range(8 * g, 8 * g + 8) for g in range(8)], 32
    raise ValueError(width)


def conflict_degree(dword_addr_of_lane, ndw, width):
    """max distinct dwords any bank serves within one lane group (1 = conflict-free)."""
    groups, nb = _groups(width)
    deg = 1
    for g in groups:
        banks = {}
        for L in g:
            a = dword_addr_of_lane(L)
            for d in range(ndw):
                banks.setdefault((a + d) % nb, set()).add(a + d)
        deg = max(deg, max(len(v) for v in banks.values()))
    return deg


def conflict_free(dword_addr_of_lane, ndw, width):
    groups, nb = _groups(width)
    for g in groups:
        banks = {}
        for L in g:
            a = dword_addr_of_lane(L)
            for d in range(ndw):
                b = (a + d) % nb
                banks.setdefault(b, set()).add(a + d)
        if any(len(s) > 1 for s in banks.values()):
            return False
    return True


def check_layouts(N):
    NW, M = N // 512, N // 2
    Q = M // NW
    ok = {}
    # ring reads: point NW (64 r + L) + w at w Q + 64 (r & 3) + L (4-byte samples)
    ok['ring_read'] = all(conflict_free(lambda L, w=w, r=r: w * Q + 64 * (r & 3) + L, 1, 'r32')
                          for w in range(NW) for r in range(8))
    ok['tap_read'] = all(conflict_free(lambda L, w=w, r=r: 2 * (w * 512 + 64 * r + L), 2, 'r64')
                         for w in range(NW) for r in range(8))
    # ring writes: thread t writes samples 4t'..4t'+3 (t' = t mod M/4) of one hop (8t'..8t'+7
    # at NW = 8: one dword in each plane)
    if NW == 8:
        # k_front5: select waves 12-15 (256 threads) refill a hop, 8 samples per thread, one
        # dword in each plane
        ok['ring_write8'] = all(conflict_free(lambda L, j=j, b=b: j * Q + b + L, 1, 'w32')
                                for j in range(8) for b in range(0, M // 8, 64))
        ok['tap_read'] = True   # k_front5 holds the PFB taps in VGPRs
    elif NW == 4:
        ok['ring_write'] = all(conflict_free(lambda L, j=j, b=b: j * Q + b + L, 1, 'w32')
                               for j in range(4) for b in range(0, M // 4, 64))
    elif NW == 2:
        ok['ring_write'] = all(conflict_free(lambda L, j=j, b=b: j * Q + 2 * (b + L), 2, 'w64')
                               for j in range(2) for b in range(0, M // 4, 64))
    else:
        ok['ring_write'] = all(conflict_free(lambda L, b=b: 4 * (b + L), 4, 'w128') for b in range(0, M // 4, 64))
    f = lambda i: i + (i >> 3)
    ok['t2_write'] = all(conflict_free(lambda L, r=r: 2 * f(64 * (L >> 3) + 8 * r + (L & 7)), 2, 'w64')
                         for r in range(8))
    ok['t2_read'] = all(conflict_free(lambda L, r=r: 2 * f(64 * (L >> 3) + 8 * (L & 7) + r), 2, 'r64')
                        for r in range(8))
    g = lambda k: k ^ ((k >> 2) & 14)
    ok['y_write'] = all(conflict_free(lambda L, r=r: 2 * g((L >> 3) + 8 * (L & 7) + 64 * r), 2, 'w64')
                        for r in range(8))
    ok['y_bijective'] = len({g(k) for k in range(512)}) == 512 and max(g(k) for k in range(512)) < 576
    ok['t2_fits'] = max(f(i) for i in range(512)) < 576
    return ok


if __name__ == '__main__':
    print('fft emulation max error', fft_emulation())
    for N in (512, 1024, 2048, 4096):
        print(N, 'combine error', decimation_combine(N), check_layouts(N))
    print('4096 Horner combine (fp32) relative error', horner_combine_f32())
