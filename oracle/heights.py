"""Per-packet optimal-filter pulse height — TEST INFRASTRUCTURE (oracle for k_heights.hip).

BASELINE config 5 asks for "per-channel optimal-filter pulse-height estimation (fp32)". The
reference computes the template and noise PSD (pulses.py:239-427) and leaves the filter and its
application as a stub (pulses.py:398; PulseAnalysis.coeff Float32Col(100), pulses.py:59), so the
definition restated here is this repository's (include/mkidgpu.h): for a wide packet
(channel 12 bits at MKID_PKT_CH_SHIFT, 28-bit phase-sample stamp ts)
    h = sum_{i < ncoeff} coeff[ch][i] * phase[ts - pre + i][ch]
over phase rows holding global phase indices j0 .. j0 + rows - 1 (the 28-bit stamp unwrapped
into [j0 - 2^27, j0 + 2^27)); NaN when the window is not inside the rows (or, with the device's
carried history, its last rows before j0). Float64 accumulation: the device's
fp32 result is compared within a relative tolerance. Parity unpinned against the reference
(stub there).
"""
import numpy as np

CH_SHIFT = 52
TS_MASK = (1 << 28) - 1


def pulse_heights(phase, events, coeff, pre, j0=0):
    phase = np.asarray(phase)
    coeff = np.asarray(coeff, np.float64)
    rows, C = phase.shape
    ncoeff = coeff.shape[1]
    ev = np.asarray(events, np.uint64)
    out = np.full(ev.size, np.nan)
    for p, w in enumerate(ev.tolist()):
        ch = (w >> CH_SHIFT) & 0xFFF
        ts = w & TS_MASK
        base = max(j0 - (1 << 27), 0)                 # stamps unwrap into [j0 - 2^27, j0 + 2^27)
        jg = base + ((ts - (base & TS_MASK)) & TS_MASK)
        r0 = jg - j0 - pre
        if ch >= C or r0 < 0 or r0 + ncoeff > rows:
            continue
        out[p] = float(np.dot(coeff[ch], phase[r0:r0 + ncoeff, ch].astype(np.float64)))
    return out
