"""numpy float64 restatement of the absent firmware chain K1-K6 — TEST INFRASTRUCTURE.

The reference's DSP ran in ROACH firmware that is not in the reference (.MISSING_LARGE_BLOBS:1-27;
README.md:31 names a Firmware/ directory that is absent). What the host code pins, and what this
restatement follows:
  K2  N-point FFT, 2x oversampled: fft_len=2**9 with 256 channels and the DDS LUT synthesised at
      sampleRate/fft_len*2 (ROACH_Setup.py:507, 515, 525)  -> hop M = N/2, C = N/2 channels.
  K3  bin select: fft_bin = round(f*N/fs) (ROACH_Setup.py:540).
  K4  DDS/DDC: per-channel LO LUT of the freqCombLUT residual tone (ROACH_Setup.py:523-530);
      mixed by conj(LUT)/2^15 (build decision, sign chosen so a tone at the selected bin +
      residual lands at DC with the LUT's phase removed).
  K5  26-tap FIR, int(lpf*(2**11-1)) 12-bit taps (ROACH_Pulses.py:61-97); decimate by 2 so the
      phase stream runs at fs/N (ROACH_Pulses.py:225 "2048 samples = 2 msec" at fs=512 MHz, N=512;
      set_svf.py:11 sampleRate=1e6).
  K6  IQ-centre subtract + phase: atan2(Q-Qc, I-Ic) (pulse_triggering_IQ.py:152 host replay),
      quantised to int16 Fix16_13 rad, clamp +-25736 (ROACH_Pulses.py:274-278).
Build decisions: PFB with T=4 taps per branch, Hamming-windowed sinc prototype
normalised to unit DC gain, applied as 16-bit taps (quantize_pfb, the device's rule); frame k covers samples [(k+1)M - TN, (k+1)M); the 2x-oversampling
rotation (-1)^(b(k+1)) is removed so a bin-centred tone gives a constant channel output.
"""
import numpy as np

FIX16_13_PI = 25736
FIR_TAPS = 26


def pfb_prototype(N, T=4):
    """Hamming-windowed sinc, T*N taps, unit DC gain, rounded to float32 (the device's taps)."""
    L = T * N
    n = np.arange(L, dtype=np.float64)
    h = np.sinc((n - (L - 1) / 2.0) / N) * (0.54 - 0.46 * np.cos(2 * np.pi * n / (L - 1)))
    h = h / h.sum()
    return h.astype(np.float32)


def quantize_pfb(h, T, N):
    """The taps the device applies (mkid_set_pfb, include/mkidgpu.h): h_q = rint(h 2^S) int16 with
    the largest S such that every point's sum_tau |h_q| <= 65535 and every |h_q| <= 32767;
    effective taps h_q 2^-S (exact in float32/float64)."""
    h = np.asarray(h, np.float32).astype(np.float64).reshape(T, N)
    ms = float(np.max(np.abs(h[0]) + np.abs(h[1]) + np.abs(h[2]) + np.abs(h[3]))) if T == 4 else \
        float(np.max(np.abs(h).sum(axis=0)))
    ma = float(np.max(np.abs(h)))
    S = 0
    if ms > 0.0:
        S = -64
        while S < 64 and np.ldexp(ms, S + 1) <= 65535.0 and np.ldexp(ma, S + 1) <= 32767.0:
            S += 1
    # the device re-checks the ROUNDED taps and steps S down while a point's sum of |h_q|
    # exceeds 65535 or a |h_q| exceeds 32767 (int16 dot products of full-scale samples stay
    # inside int32, mkid_api.hip quantize_pfb)
    while True:
        hq = np.rint(np.ldexp(h, S))
        if (np.abs(hq).sum(axis=0).max() <= 65535 and np.abs(hq).max() <= 32767) or S <= -64:
            break
        S -= 1
    return np.ldexp(hq, -S).reshape(-1), int(S)


def lo_table(lut_i, lut_q):
    """[C][P] int16 LUT -> complex128 conj(LUT)/2^15 (K4 mixer)."""
    return (np.asarray(lut_i, np.float64) - 1j * np.asarray(lut_q, np.float64)) / 32768.0


class OracleChain:
    """Streaming float64 chain. process(iq) -> dict(z, y, phase, raw)."""

    def __init__(self, n_channels, pfb_coeffs, bins, lut_i, lut_q, lpf_taps12, ic=None, qc=None,
                 T=4):
        self.C = int(n_channels)
        self.N = 2 * self.C
        self.M = self.C
        self.T = T
        self.h = quantize_pfb(pfb_coeffs, T, self.N)[0].reshape(T, self.N)
        self.bins = np.asarray(bins, np.int64) % self.N
        self.lo = lo_table(lut_i, lut_q)
        self.P = self.lo.shape[1]
        self.g = np.asarray(lpf_taps12, np.float64) / 2048.0
        self.ic = np.zeros(self.C) if ic is None else np.asarray(ic, np.float32).astype(np.float64)
        self.qc = np.zeros(self.C) if qc is None else np.asarray(qc, np.float32).astype(np.float64)
        self.reset()

    def reset(self):
        self.xhist = np.zeros(self.T * self.N - self.M, np.complex128)
        self.zhist = np.zeros((len(self.g) - 2, self.C), np.complex128)
        self.k0 = 0

    def channelize(self, iq, block=256):
        iq = np.asarray(iq)
        x = iq[:, 0].astype(np.float64) + 1j * iq[:, 1].astype(np.float64)
        assert len(x) % self.N == 0
        xx = np.concatenate([self.xhist, x])
        K = len(x) // self.M
        z = np.empty((K, self.C), np.complex128)
        span = np.arange(self.T * self.N)
        cidx = np.arange(self.C)
        for kb in range(0, K, block):
            ke = min(K, kb + block)
            ks = np.arange(kb, ke)
            seg = xx[ks[:, None] * self.M + span[None, :]].reshape(ke - kb, self.T, self.N)
            u = (seg * self.h[None]).sum(axis=1)
            X = np.fft.fft(u, axis=1)
            kg = self.k0 + ks
            sign = 1.0 - 2.0 * ((self.bins[None, :] * (kg[:, None] + 1)) & 1)
            lo = self.lo[cidx[None, :], (kg[:, None] % self.P)]
            z[kb:ke] = X[:, self.bins] * sign * lo
        self.xhist = xx[len(xx) - len(self.xhist):].copy()
        self.k0 += K
        return z

    def lpf(self, z):
        nt = len(self.g)
        zz = np.concatenate([self.zhist, z])
        J = z.shape[0] // 2
        y = np.zeros((J, self.C), np.complex128)
        for i in range(nt):
            start = (nt - 2) + 1 - i
            y += self.g[i] * zz[start:start + 2 * J:2]
        self.zhist = zz[len(zz) - (nt - 2):].copy()
        return y

    def phase(self, y):
        ph = np.arctan2(y.imag - self.qc[None, :], y.real - self.ic[None, :])
        raw = np.clip(np.rint(ph * 8192.0), -FIX16_13_PI, FIX16_13_PI).astype(np.int16)
        return ph, raw

    def process(self, iq):
        z = self.channelize(iq)
        y = self.lpf(z)
        ph, raw = self.phase(y)
        return dict(z=z, y=y, phase=ph, raw=raw)
