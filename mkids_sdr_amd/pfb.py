"""PFB prototype filter (build decision: the firmware's PFB taps are absent from the reference,
.MISSING_LARGE_BLOBS:1-27). Hamming-windowed sinc of T*N taps, cutoff at the bin spacing,
normalised to unit DC gain so a bin-centred tone of amplitude A gives |X[b]| = A; rounded to
float32, which are the exact coefficients the device uses."""
import numpy as np


def pfb_prototype(N, T=4):
    L = T * N
    n = np.arange(L, dtype=np.float64)
    h = np.sinc((n - (L - 1) / 2.0) / N) * (0.54 - 0.46 * np.cos(2 * np.pi * n / (L - 1)))
    h = h / h.sum()
    return h.astype(np.float32)
