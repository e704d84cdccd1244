#!/usr/bin/env python3
"""Where does the fp32 chain's phase error come from? (CPU study)

Runs the float64 oracle chain (oracle/chain.py) and variants of it in which ONE stage is computed
in float32 (numpy complex64: PFB-output conversion, FFT, DDC mix, IQ low-pass — uncentred 'lpf' or the
device's centred form 'lpfc' — centre + atan2), on a
feedline with unequal per-resonator attenuation (ROACH_Setup.py:499-502) and off-origin IQ loop
centres (ROACH_Setup.py:595-667), and reports each variant's max phase error against the float64
chain, binned by the channel's loop radius |y - centre| relative to the strongest tone's |y|.
numpy's float32 FFT is not the device's radix-8 decomposition, so this attributes orders of
magnitude, not the device's exact numbers (tests/test_gpu_parity.py measures those).

    python tools/precision_study.py [--channels 1024] [--log2 18] [--span 20] [--ratio-min 0.1]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

import signals  # noqa: E402
from oracle import chain  # noqa: E402


class Chain32(chain.OracleChain):
    """The oracle chain with selected stages rounded to float32."""

    def __init__(self, *a, stages=(), **k):
        super().__init__(*a, **k)
        self.stages = set(stages)

    def channelize(self, iq, block=256):
        x = iq[:, 0].astype(np.float64) + 1j * iq[:, 1].astype(np.float64)
        xx = np.concatenate([self.xhist, x])
        K = len(x) // self.M
        z = np.empty((K, self.C), np.complex128)
        span = np.arange(self.T * self.N)
        cidx = np.arange(self.C)
        lo32 = self.lo.astype(np.complex64)
        for kb in range(0, K, block):
            ke = min(K, kb + block)
            ks = np.arange(kb, ke)
            seg = xx[ks[:, None] * self.M + span[None, :]].reshape(ke - kb, self.T, self.N)
            u = (seg * self.h[None]).sum(axis=1)            # exact (int16 x 16-bit taps)
            if 'pfb' in self.stages or 'fft' in self.stages:
                u = u.astype(np.complex64)
            X = np.fft.fft(u, axis=1)
            if 'fft' not in self.stages:
                X = np.fft.fft(u.astype(np.complex128), axis=1)
            kg = self.k0 + ks
            sign = 1.0 - 2.0 * ((self.bins[None, :] * (kg[:, None] + 1)) & 1)
            if 'ddc' in self.stages:
                Xb = X[:, self.bins].astype(np.complex64) * sign.astype(np.float32)
                z[kb:ke] = Xb * lo32[cidx[None, :], (kg[:, None] % self.P)]
            else:
                lo = self.lo[cidx[None, :], (kg[:, None] % self.P)]
                z[kb:ke] = X[:, self.bins] * sign * lo
        self.xhist = xx[len(xx) - len(self.xhist):].copy()
        self.k0 += K
        return z

    def lpf(self, z):
        if 'lpfc' in self.stages:
            return self.lpf_centred(z)
        if 'lpf' not in self.stages:
            return super().lpf(z)
        nt = len(self.g)
        zz = np.concatenate([self.zhist, z]).astype(np.complex64)
        J = z.shape[0] // 2
        y = np.zeros((J, self.C), np.complex64)
        g = self.g.astype(np.float32)
        for i in range(nt):
            start = (nt - 2) + 1 - i
            y = y + g[i] * zz[start:start + 2 * J:2]
        self.zhist = zz[len(zz) - (nt - 2):].astype(np.complex128)
        return y.astype(np.complex128)

    def lpf_centred(self, z):
        """The device's centred low-pass (mkid_internal.h Centring): fp32
        y' = sum_i g_i (z_i - c') with c' = fp32(c / G), and r = fp32(G c' - c) from float64; the
        chain carries y = y' + r + c onward (exact in float64), so the float64 phase stage sees
        the fp32 y' + r."""
        nt = len(self.g)
        G = float(self.g.sum())
        c = self.ic.astype(np.float64) + 1j * self.qc.astype(np.float64)
        cp = (c / G).astype(np.complex64)
        r = (G * cp.astype(np.complex128) - c).astype(np.complex64)
        zz = np.concatenate([self.zhist, z])
        J = z.shape[0] // 2
        y = np.zeros((J, self.C), np.complex64)
        g = self.g.astype(np.float32)
        for i in range(nt):
            start = (nt - 2) + 1 - i
            d = (zz[start:start + 2 * J:2].astype(np.complex64) - cp[None, :]).astype(np.complex64)
            y = (y + g[i] * d).astype(np.complex64)
        self.zhist = zz[len(zz) - (nt - 2):].copy()
        yc = (y + r[None, :]).astype(np.complex64)          # the fp32 y - c the device's atan2 sees
        return yc.astype(np.complex128) + c[None, :]

    def phase(self, y):
        if 'atan' not in self.stages:
            return super().phase(y)
        y32 = y.astype(np.complex64)
        ph = np.arctan2(y32.imag - self.qc.astype(np.float32)[None, :],
                        y32.real - self.ic.astype(np.float32)[None, :]).astype(np.float64)
        raw = np.clip(np.rint(ph * 8192.0), -chain.FIX16_13_PI, chain.FIX16_13_PI).astype(np.int16)
        return ph, raw


def combine_study(seeds=3, span=20.0):
    """k_front5's decimated combine (N = 4096, 8 sub-FFTs of 512, radix-2 pre-combination in the
    transform waves, 4-way Horner select) in complex64 on a 2048-tone comb spread over `span` dB:
    the error at the tone bins relative to the strongest tone, for the pre-combination twiddles of
    round 5 (wk *= W_16), of round 6 (tools/front_layouts.pre_twiddles), and directly rounded ones,
    beside a plain fp32 4096-point FFT. The sub-FFT outputs carry the comb's 8 aliased bins, so a
    twiddle error leaks the strong tones into the weak channels' bins."""
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import front_layouts as fl
    N, C = 4096, 2048
    k = np.arange(512)
    tws = {'round5_recurrence': fl.pre_twiddles(True)[k // 64, k % 64],
           'round6_device': fl.pre_twiddles()[k // 64, k % 64],
           'direct_rounded': np.exp(-2j * np.pi * k / 1024).astype(np.complex64)}
    out = {name: [] for name in list(tws) + ['numpy_fp32_fft4096']}
    for seed in range(seeds):
        rng = np.random.default_rng(seed)
        bins = rng.permutation(np.arange(1, N))[:C]
        amp = 10 ** (-rng.uniform(0, span, C) / 20)
        n = np.arange(N)
        x = (amp[None, :] * np.exp(2j * np.pi * (np.outer(n, bins) / N + rng.uniform(size=C)[None, :]))).sum(1)
        u = x * 3e4 / np.abs(x).max()
        ref = np.fft.fft(u)
        ymax = np.abs(ref[bins]).max()
        Ys = [np.fft.fft(u[w::8].astype(np.complex64)).astype(np.complex64) for w in range(8)]
        b = np.arange(N)
        s_, kk = (b >> 9) & 1, b % 512
        t = np.exp(-2j * np.pi * b / N).astype(np.complex64)
        t2 = (t * t).astype(np.complex64)
        for name, tw in tws.items():
            P = {}
            for r in range(4):
                d = (Ys[r + 4] * tw).astype(np.complex64)
                P[(r, 0)] = (Ys[r] + d).astype(np.complex64)
                P[(r, 1)] = (Ys[r] - d).astype(np.complex64)
            g = lambda r: np.where(s_ == 0, P[(r, 0)][kk], P[(r, 1)][kk])
            X = ((g(0) + t2 * g(2)).astype(np.complex64) + t * (g(1) + t2 * g(3)).astype(np.complex64)).astype(np.complex64)
            e = np.abs(X[bins] - ref[bins]) / ymax
            out[name].append((float(e.max()), float(np.sqrt((e ** 2).mean()))))
        e = np.abs(np.fft.fft(u.astype(np.complex64)).astype(np.complex64)[bins] - ref[bins]) / ymax
        out['numpy_fp32_fft4096'].append((float(e.max()), float(np.sqrt((e ** 2).mean()))))
    return {name: dict(max_rel_to_strongest=max(a for a, _ in v), rms_rel_to_strongest=float(np.mean([b for _, b in v])))
            for name, v in out.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--combine', action='store_true', help="k_front5's combine study only (combine_study)")
    p.add_argument('--channels', type=int, default=1024)
    p.add_argument('--log2', type=int, default=18)
    p.add_argument('--span', type=float, default=20.0, help='attenuation span (dB)')
    p.add_argument('--ratio-min', type=float, default=0.1, help='smallest loop radius / |centre|')
    p.add_argument('--seed', type=int, default=7)
    a = p.parse_args()
    if a.combine:
        print(json.dumps(dict(span_db=a.span, tones=2048, N=4096, combine=combine_study(span=a.span)), indent=1))
        return
    C, S = a.channels, 1 << a.log2
    rng = np.random.default_rng(a.seed)
    att = rng.uniform(0.0, a.span, C)
    ratio = np.exp(rng.uniform(np.log(a.ratio_min), np.log(10.0), C))
    ratio[rng.random(C) < 0.2] = np.inf
    case = signals.make_case(C, S, seed=a.seed, pulses_per_ch=2.0, atten_db=att, loop_ratio=ratio)
    args = (case.C, case.pfb, case.bins, case.lut_i, case.lut_q, case.lpf12, case.ic, case.qc)
    ref = chain.OracleChain(*args).process(case.iq)
    ymax = np.abs(ref['y'][64:]).mean(0).max()
    q = case.loop_radius / ymax
    edges = [0.0, 0.01, 0.03, 0.1, 0.3, 1.01]
    out = {'channels': C, 'samples': S, 'span_db': a.span, 'ratio_min': a.ratio_min,
           'bins_q': edges, 'n_per_bin': [int(((q >= lo) & (q < hi)).sum()) for lo, hi in zip(edges, edges[1:])]}
    for st in (('pfb',), ('fft',), ('ddc',), ('lpf',), ('lpfc',), ('atan',), ('fft', 'ddc', 'lpf', 'atan'),
               ('pfb', 'fft', 'ddc', 'lpfc')):
        r = Chain32(*args, stages=st).process(case.iq)
        err = np.abs(signals.wrap(r['phase'][64:] - ref['phase'][64:])).max(axis=0)
        out['+'.join(st)] = [float(err[(q >= lo) & (q < hi)].max()) if ((q >= lo) & (q < hi)).any() else None
                             for lo, hi in zip(edges, edges[1:])]
        # error x radius: an absolute IQ error in units of the strongest tone's |y|
        out['+'.join(st) + ':abs_iq'] = float((err * q).max())
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
