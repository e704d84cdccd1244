"""Restatement of the reference's host-side numpy trigger replays — TEST INFRASTRUCTURE.

rolling_mean_trigger   pulse_triggering_v2.py:104-174 (same loop in pulse_triggering_IQ.py:159-200)
block_mean_trigger     pulse_triggering.py:109-208 (start 100, need 300 after, skip 200) and the
                       ROACH_Pulses.py:614-727 contsnapshot variant (start 500, 1500, skip 1000)
Both operate on phase in degrees and return the hit indices (the reference saves a window of
samples around each hit to text files; the indices are what determines them).
"""
import numpy as np


def rolling_mean_trigger(phase_deg, meanlength=20, pulselength=1000, threshold=25.0,
                         pre=100):
    x = np.asarray(phase_deg, np.float64)
    n = len(x)
    hits = []
    bob = pre + meanlength                                   # :104
    while bob < n:                                           # :108
        if bob + pulselength > n:                            # :111
            break
        rolling = np.mean(x[bob - meanlength:bob])           # :114
        if abs(rolling - x[bob]) > threshold:                # :118
            hits.append(bob)
            bob = bob + pulselength                          # :171
        else:
            bob = bob + 1                                    # :174
    return hits


def block_mean_trigger(phase_deg, averagelength=128, threshold=25.0, start=100, need=300,
                       skip=200, wrap_negative=True):
    x = np.array(phase_deg, np.float64)
    if wrap_negative:                                        # pulse_triggering.py:110-112
        x[x < 0] += 360
    n = len(x)
    nmeans = n // averagelength
    means = np.array([np.mean(x[averagelength * j:averagelength * (j + 1)])
                      for j in range(nmeans)])               # :119-120
    hits = []
    bob = start
    while bob < n:
        which = bob // averagelength                         # :125
        if bob + need > n:                                   # :127
            break
        if abs(means[which] - x[bob]) > threshold:           # :132
            hits.append(bob)
            bob += skip                                      # :205
        else:
            bob += 1
    return hits
