"""PFB prototype filter (build decision: the firmware's PFB taps are absent from the reference,
.MISSING_LARGE_BLOBS:1-27). Hamming-windowed sinc of T*N taps, cutoff at the bin spacing,
normalised to unit DC gain so a bin-centred tone of amplitude A gives |X[b]| = A. The device
applies the taps as 16-bit integers h_q = rint(h 2^S) (mkid_set_pfb): `effective_taps` returns
h_q 2^-S, the coefficients the device's PFB actually uses."""
import numpy as np


def pfb_prototype(N, T=4):
    L = T * N
    n = np.arange(L, dtype=np.float64)
    h = np.sinc((n - (L - 1) / 2.0) / N) * (0.54 - 0.46 * np.cos(2 * np.pi * n / (L - 1)))
    h = h / h.sum()
    return h.astype(np.float32)


def effective_taps(h, T=4):
    """(h_q * 2^-S as float64 [T*N], S): the rule of mkid_set_pfb (include/mkidgpu.h)."""
    h = np.asarray(h, np.float32).astype(np.float64).reshape(T, -1)
    ms = float(np.max(np.abs(h).sum(axis=0)))
    ma = float(np.max(np.abs(h)))
    S = 0
    if ms > 0.0:
        S = -64
        while S < 64 and np.ldexp(ms, S + 1) <= 65535.0 and np.ldexp(ma, S + 1) <= 32767.0:
            S += 1
    while True:   # step S down until the rounded taps obey both bounds (mkid_set_pfb)
        hq = np.rint(np.ldexp(h, S))
        if (np.abs(hq).sum(axis=0).max() <= 65535 and np.abs(hq).max() <= 32767) or S <= -64:
            break
        S -= 1
    return np.ldexp(hq, -S).reshape(-1), int(S)
