"""Pulse template and near-optimal filter on the device.

`make_template` is the reference's MakeTemplate (DataReadout/ReadoutControls/lib/pulses.py:239-427)
for one resonator's pulse set — the RawPulse rows I, Q float32 [P][2000] — returning the
PulseAnalysis fields (pulses.py:44-51). `optimal_filter` fills the step the reference leaves as a
stub (pulses.py:398, PulseAnalysis.coeff Float32Col(100)). `matched_fir_taps` turns the filter
into the firmware's 26-tap matched filter (K7) that `loadFIRcoeffs` / `Channelizer.set_fir` load.
"""
import ctypes

import numpy as np

from . import _lib, codecs

NPTS = 2000
NNOISE = 800


def _dev(a, dtype):
    import torch
    if hasattr(a, 'data_ptr'):
        return a.to(dtype=dtype).contiguous()
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32 if dtype == torch.float32
                                                 else np.float64)).cuda()


def make_template(ch, I, Q):
    """I, Q: float32 [P][2000] (host arrays or device tensors). Returns a dict with template
    [2000], noise [800], noiseidx [800] (np.fft.fftfreq(800, d=2e-6), pulses.py:391) and the
    scalars count, count1, pm, pdev, flag, pstart."""
    import torch
    dI, dQ = _dev(I, torch.float32), _dev(Q, torch.float32)
    if dI.dim() != 2 or dI.shape[1] != NPTS or dQ.shape != dI.shape:
        raise ValueError('I, Q must be [P][2000]')
    tpl = torch.empty(NPTS, dtype=torch.float64, device=dI.device)
    noise = torch.empty(NNOISE, dtype=torch.float64, device=dI.device)
    info = _lib.TemplateInfo()
    torch.cuda.synchronize()
    ch._chk(ch._L.mkid_make_template(ch._h, ctypes.c_void_p(dI.data_ptr()), ctypes.c_void_p(dQ.data_ptr()),
                                     int(dI.shape[0]), ctypes.c_void_p(tpl.data_ptr()),
                                     ctypes.c_void_p(noise.data_ptr()), ctypes.byref(info)))
    return dict(template=tpl.cpu().numpy(), noise=noise.cpu().numpy(),
                noiseidx=np.fft.fftfreq(NNOISE, d=0.000002), count=info.count, count1=info.count1,
                pm=info.pm, pdev=info.pdev, flag=info.flag, pstart=info.pstart,
                d_template=tpl, d_noise=noise)


def optimal_filter(ch, template, noise, pre=100, ncoeff=100):
    """Correlation weights of the S/J optimal filter (see include/mkidgpu.h), float64 [ncoeff]."""
    import torch
    t = _dev(template, torch.float64)
    n = _dev(noise, torch.float64)
    out = torch.empty(ncoeff, dtype=torch.float64, device=t.device)
    torch.cuda.synchronize()
    ch._chk(ch._L.mkid_optimal_filter(ch._h, ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(n.data_ptr()),
                                      int(pre), int(ncoeff), ctypes.c_void_p(out.data_ptr())))
    return out.cpu().numpy()


def matched_fir_taps(coeff, ntaps=26, sign=-1.0):
    """Firmware FIR taps from correlation weights: the ntaps-long window of largest energy,
    reversed into convolution order (f_j = sum_i a_i raw_{j-i}), scaled to max |a| = 2047/2048
    and multiplied by `sign` (phase pulses are negative-going at the trigger, ROACH_Pulses.py:270).
    Returns (float taps for loadFIRcoeffs, int12 taps for Channelizer.set_fir)."""
    c = np.asarray(coeff, np.float64)
    e = np.convolve(c * c, np.ones(ntaps), mode='valid')
    k = int(np.argmax(e))
    a = sign * c[k:k + ntaps][::-1]
    a = a / np.max(np.abs(a)) * (2047.0 / 2048.0)
    return a, codecs.fir_quantise(a)
