#!/usr/bin/env python3
"""Fit of the degree-7 (in t^2) atan polynomial used by phase_atan2 (fft_common.h), evaluated in
float32 arithmetic against float64 atan2: max error and Fix16_13 rounding-flip rate.

    python tools/atan_fit.py
"""
import numpy as np
from numpy.polynomial import chebyshev as Ch
# fit atan(t)/t as polynomial in u = t^2 on [0,1], minimax-ish via Chebyshev least squares + Remez-lite
def fit(deg):
    u = (1 - np.cos(np.linspace(0, np.pi, 4000))) / 2  # cheb nodes on [0,1]
    t = np.sqrt(u)
    f = np.where(t > 0, np.arctan(t) / np.where(t > 0, t, 1), 1.0)
    # weighted least squares for absolute error of atan: weight by t
    w = np.maximum(t, 1e-3)
    A = np.vander(u, deg + 1, increasing=True) * w[:, None]
    c, *_ = np.linalg.lstsq(A, f * w, rcond=None)
    # iterate reweighting (Lawson) towards minimax
    for it in range(60):
        err = (np.vander(u, deg + 1, increasing=True) @ c - f) * t
        w = w * (np.abs(err) / np.abs(err).max() + 1e-3) ** 0.5
        A = np.vander(u, deg + 1, increasing=True) * w[:, None]
        c, *_ = np.linalg.lstsq(A, f * w, rcond=None)
    return c
def atan2_f32(y, x, c):
    y = y.astype(np.float32); x = x.astype(np.float32)
    ax, ay = np.abs(x), np.abs(y)
    mx = np.maximum(ax, ay); mn = np.minimum(ax, ay)
    t = (mn / mx).astype(np.float32)          # ~correctly rounded division
    u = (t * t).astype(np.float32)
    p = np.float32(c[-1])
    for k in range(len(c) - 2, -1, -1):
        p = (p * u + np.float32(c[k])).astype(np.float32)
    r = (p * t).astype(np.float32)
    r = np.where(ay > ax, (np.float32(np.pi / 2) - r).astype(np.float32), r)
    r = np.where(x < 0, (np.float32(np.pi) - r).astype(np.float32), r)
    r = np.where(y < 0, -r, r)
    return r
rng = np.random.default_rng(1)
ang = rng.uniform(-np.pi, np.pi, 2_000_000)
rad = rng.uniform(100, 30000, ang.size)
x = (rad * np.cos(ang)).astype(np.float32); y = (rad * np.sin(ang)).astype(np.float32)
ref = np.arctan2(y.astype(np.float64), x.astype(np.float64))
ref32 = np.arctan2(y, x)  # numpy float32 atan2 (correctly rounded-ish)
print('numpy f32 atan2 max err', np.abs(ref32 - ref).max())
for deg in (7, 8, 9, 10):
    c = fit(deg)
    r = atan2_f32(y, x, c)
    e = np.abs(r.astype(np.float64) - ref)
    flips = np.mean(np.rint(r.astype(np.float64) * 8192) != np.rint(ref * 8192))
    flips32 = np.mean(np.rint(ref32.astype(np.float64) * 8192) != np.rint(ref * 8192))
    print(deg, 'max err %.3g' % e.max(), 'flips %.2e (f32 atan2 %.2e)' % (flips, flips32))
    if deg == 9: print(repr(c))
print('---')
for deg in (5, 6, 7):
    c = fit(deg)
    r = atan2_f32(y, x, c)
    e = np.abs(r.astype(np.float64) - ref)
    flips = np.mean(np.rint(r.astype(np.float64) * 8192) != np.rint(ref * 8192))
    print(deg, 'max err %.3g' % e.max(), 'flips %.2e' % flips, repr(c.astype(np.float32)))
