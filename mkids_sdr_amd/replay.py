"""Device versions of the reference's host-replay triggers.

The reference reads one channel's phase snapshot over katcp and walks it in a Python while-loop
(pulse_triggering_v2.py:104-174, pulse_triggering_IQ.py:159-200, pulse_triggering.py:109-208,
ROACH_Pulses.py:614-727). Here every channel of a device Fix16_13 phase block is walked at once
(mkid_replay_trigger, k_replay.hip) with the reference's own float64 arithmetic, so the hit lists
are the ones the numpy loops produce. Parameters keep the reference's names and defaults.
"""
import numpy as np

from . import _lib


def _hits_to_lists(d_hits, d_counts, cap):
    import torch
    torch.cuda.synchronize()  # the replay ran on the context stream, not torch's
    h = d_hits.cpu().numpy()
    n = d_counts.cpu().numpy()
    if (n > cap).any():
        raise _lib.MkidError(_lib.MKID_E_OVERFLOW, 'replay: more hits than cap=%d' % cap)
    return [h[c, :n[c]].tolist() for c in range(len(n))]


def rolling_mean_trigger(ch, d_raw, n, ld, nch, meanlength=20, pulselength=1000, threshold=25.0,
                         pre=100, cap=64):
    """pulse_triggering_v2.py:104-174: hits j where |mean(x[j-m:j]) - x[j]| > threshold, starting
    at pre + m, skipping pulselength after a hit, stopping at j + pulselength > n."""
    d_hits, d_counts = ch.replay_trigger(d_raw, n, ld, nch, _lib.REPLAY_ROLLING, meanlength,
                                         pre + meanlength, pulselength, pulselength, threshold,
                                         wrap_negative=False, cap=cap)
    return _hits_to_lists(d_hits, d_counts, cap)


def block_mean_trigger(ch, d_raw, n, ld, nch, averagelength=128, threshold=25.0, start=100,
                       need=300, skip=200, wrap_negative=True, cap=64):
    """pulse_triggering.py:109-208 (defaults) / ROACH_Pulses.py:614-727 (start=500, need=1500,
    skip=1000, no wrap): means over fixed blocks of averagelength."""
    d_hits, d_counts = ch.replay_trigger(d_raw, n, ld, nch, _lib.REPLAY_BLOCK, averagelength,
                                         start, need, skip, threshold,
                                         wrap_negative=wrap_negative, cap=cap)
    return _hits_to_lists(d_hits, d_counts, cap)


def raw_to_deg(raw):
    """Host decode used by the reference before the loops (pulse_triggering_v2.py:93-95)."""
    return np.asarray(raw, np.float64) * 360. / 2 ** 16 * 4 / np.pi
