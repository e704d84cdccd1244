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


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--channels', type=int, default=1024)
    p.add_argument('--log2', type=int, default=18)
    p.add_argument('--span', type=float, default=20.0, help='attenuation span (dB)')
    p.add_argument('--ratio-min', type=float, default=0.1, help='smallest loop radius / |centre|')
    p.add_argument('--seed', type=int, default=7)
    a = p.parse_args()
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
