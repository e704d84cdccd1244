"""CPU study: how long two exact SVF baseline trajectories (the int64 Chamberlin update of
k_trig_spec, trig_common.h base_update_svf, bench.py's kf = 82, kq = 93623, base_thr = 8192) take to
become bit-identical when one starts from the speculative cold guess (low = f0 * 2^16, band = 0) or
from the true state perturbed by +-P in low (+-P/16 in band) -- i.e. how much a better segment-start
guess (e.g. a float scan of the linear filter) could shorten the SVF warm-up W.
Gaussian filtered-phase input of sigma 50 / 300 / 1000 LSB, 4096 trials each.
    python tools/svf_merge_study.py      (prints one line per (sigma, start))"""
import numpy as np, sys
kf, kq, bt = 82, 93623, 8192
def step(low, band, f):
    e = f - (low >> 16)
    gate = np.abs(e) < bt
    high = f.astype(np.int64) * 65536 - low - ((kq * band) >> 16)
    nb = band + ((kf * high) >> 16)
    nl = low + ((kf * nb) >> 16)
    return np.where(gate, nl, low), np.where(gate, nb, band)
rng = np.random.default_rng(1)
T = 4096; Nmax = 120000
for sigma in (50, 300, 1000):
    for pert in ('cold', 2**20, 2**12, 2**8, 2**4, 1):
        # true trajectory: start from a settled state (run 200k samples first)
        low = np.zeros(T, np.int64); band = np.zeros(T, np.int64)
        for i in range(30000):
            low, band = step(low, band, np.rint(rng.normal(0, sigma, T)).astype(np.int64))
        if pert == 'cold':
            f0 = np.rint(rng.normal(0, sigma, T)).astype(np.int64)
            l2 = f0 * 65536; b2 = np.zeros(T, np.int64)
        else:
            l2 = low + rng.integers(-pert, pert + 1, T); b2 = band + rng.integers(-max(pert >> 4, 1), max(pert >> 4, 1) + 1, T)
        merged = np.full(T, -1)
        for i in range(Nmax):
            f = np.rint(rng.normal(0, sigma, T)).astype(np.int64)
            low, band = step(low, band, f); l2, b2 = step(l2, b2, f)
            m = (low == l2) & (band == b2) & (merged < 0)
            merged[m] = i
            if i % 1000 == 0 and (merged >= 0).all(): break
        ok = merged[merged >= 0]
        print(sigma, pert, 'merged %.3f' % (len(ok) / T), 'p50 %d p90 %d p99 %d max %d' % tuple(np.percentile(ok, [50, 90, 99, 100])) if len(ok) else '', flush=True)
