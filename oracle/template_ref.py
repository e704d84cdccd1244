"""Restatement of the reference's MakeTemplate (DataReadout/ReadoutControls/lib/pulses.py:239-427)
— TEST INFRASTRUCTURE (oracle for k_template.hip).

Input: one resonator's pulses as the reference's RawPulse table holds them (pulses.py:30-43):
I, Q float32 [P][2000]. The PyTables file I/O is replaced by arrays; the arithmetic follows the
reference line by line in numpy with the reference's dtypes (float32 pulses, float64 fit and
template), including its quirk that `I = dat['I'][j]; I += ...` edits the table in place, so the
first 1000 pulses are re-referenced twice (once per pass).

Parity: the reference is Python 2 + PyTables and cannot run here; this restatement is pinned by
the reference's own FakeTemplateData generator (pulses.py:429-481, restated in
tests/test_template.py), not by reference outputs ("parity unpinned" for a18 in DESIGN.md).

The optimal filter is a stub in the reference (pulses.py:398 "calculate optimal filter
parameters", PulseAnalysis.coeff = Float32Col(100), pulses.py:59): `optimal_filter` below is this
repository's definition, the frequency-domain matched filter S*/J.
"""
import numpy as np

NPTS = 2000
NNOISE = 800


def make_template(I, Q, xc=0.0, yc=0.0):
    dat_I = np.array(I, np.float32, copy=True)   # the table read into memory (pulses.py:263)
    dat_Q = np.array(Q, np.float32, copy=True)
    N = len(dat_I)
    tP = np.zeros(NPTS, dtype='float64')
    tPf = np.zeros(NPTS, dtype='float64')
    noise = np.zeros(NNOISE, dtype='float64')
    count = 0.0
    peaklist = []
    idx = np.arange(NPTS) * 2.0                                          # :269
    fitidx = np.concatenate((idx[:900], idx[1800:]))                     # :270
    I1m = np.median(dat_I[:100, :900])                                   # :277
    Q1m = np.median(dat_Q[:100, :900])
    if N > 1000:                                                         # :281
        N = 1000

    def prep(j):
        Ij = dat_I[j]                 # views: the += below edits the table (pulses.py:287-292)
        Qj = dat_Q[j]
        Ij += (I1m - np.median(Ij[1:900]))
        Qj += (Q1m - np.median(Qj[1:900]))
        P1 = np.arctan2(Qj - yc, Ij - xc)                                # :295
        P2 = np.rad2deg(np.unwrap(P1))                                   # :299
        fit = np.poly1d(np.polyfit(fitidx, np.concatenate((P2[:900], P2[1800:])), 1))  # :302
        P3 = P2 - fit(idx)
        stdev = np.std(P3[:100])                                         # :306
        bad = np.abs(np.mean(P3[:100]) - np.mean(P3[1900:])) > stdev * 2.0
        return P3, bad

    for j in range(N):                                                   # first pass :285
        P3, bad = prep(j)
        if bad:
            continue
        peak = np.max(P3[980:1050])                                      # :313
        peaklist.append(peak)
        if peak < 15.0 or peak > 120.0:
            continue
        ploc = int(np.where(P3 == peak)[0][0])                           # :319
        if ploc < 980 or ploc > 1020:
            continue
        P4 = np.roll(P3, 1000 - ploc)                                    # :324
        tP += P4 / np.max(P4)
        count += 1
    count1 = count
    tP /= count                                                          # :330

    peaklist = np.asarray(peaklist)                                      # :334
    pm = np.median(peaklist[np.where(peaklist > 15)])
    pdev = np.std(peaklist[np.where(peaklist > 15)])

    N = len(dat_I)                                                       # :339
    count = 0.0
    for j in range(N):                                                   # second pass
        P3, bad = prep(j)
        if bad:
            continue
        conv = np.convolve(tP[900:1500], P3)                             # :366
        ploc = int(np.where(conv == np.max(conv))[0][0] - 1160.0)
        peak = np.max(P3[1000 + ploc])
        if peak < pm - 4.0 * pdev or peak > pm + 4.0 * pdev:             # :372
            continue
        if ploc < -30 or ploc > 30:                                      # :376
            continue
        P4 = np.roll(P3, -ploc)                                          # :380
        tPf += P4 / np.max(P4)
        count += 1
        noise += np.abs(np.fft.fft(np.deg2rad(P4[50:850]))) ** 2         # :387
    tPf /= count
    noise /= count
    noiseidx = np.fft.fftfreq(len(noise), d=0.000002)                    # :391
    flag = 1 if (count < 500 or pm < 10 or pm > 150) else 0              # :409
    pstart = int(np.where(tPf == np.max(tPf))[0][0])
    return dict(template=tPf, noise=noise, noiseidx=noiseidx, count1=count1, count=count,
                pm=pm, pdev=pdev, flag=flag, pstart=pstart, template1=tP)


def optimal_filter(template, noise, ncoeff=100, pre=100):
    """S*/J matched filter from the template and the noise PSD (this repository's definition; the
    reference's step is a stub): s = template[pstart - pre : pstart - pre + 800] (deg -> rad),
    H = S / J with H[0] = 0 (baseline-insensitive), g = real(ifft(H)) read as correlation weights
    (y_j = sum_m g[m] x_{j+m} = ifft(conj(S) X / J)_j: white noise gives g = s, the plain matched
    filter); normalised so that sum_m g[m] s[m] = 1 (unit gain for a template-shaped pulse); the
    ncoeff weights starting pre-10 samples before the peak."""
    t = np.asarray(template, np.float64)
    J = np.asarray(noise, np.float64)
    pstart = int(np.argmax(t))
    s = np.deg2rad(t[pstart - pre:pstart - pre + NNOISE])
    S = np.fft.fft(s)
    H = S / J            # applied to data as conj(H) X: the S*/J filter
    H[0] = 0.0
    g = np.real(np.fft.ifft(H))
    g /= np.dot(g, s)
    k0 = pre - 10
    return g[k0:k0 + ncoeff].copy()
