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


def contsnapshot_loop(qdr_phase_values, phase_threshold, averagelength, maxloops):
    """ROACH_Pulses.py:614-752 loop-for-loop: block means, the bob walk with its 2000-sample
    windows, and the failsafe that ends the walk after maxloops passes (747-750). Returns
    (hits, pulsenumberarray, finalphasearray)."""
    qdr_phase_values = np.asarray(qdr_phase_values, np.float64)
    total_pulses = 0
    pulsenumberarray = np.zeros(2000).tolist()              # :560-561
    finalphasearray = []
    bob = 500                                               # :611
    numberofaverages = len(qdr_phase_values) // averagelength
    phase_means = np.zeros(numberofaverages)
    for i in range(numberofaverages):                       # :626-627
        phase_means[i] = np.mean(qdr_phase_values[(averagelength * (i + 1) - averagelength):averagelength * (i + 1)])
    hits = []
    failsafe = 0
    while bob < len(qdr_phase_values):                      # :630
        whichmean = bob // averagelength
        if bob + 1500 > len(qdr_phase_values):              # :635
            break
        bob_array = qdr_phase_values[bob - 500:bob + 1500]  # :651
        if abs(phase_means[whichmean] - qdr_phase_values[bob]) > phase_threshold:   # :661
            hits.append(bob)
            pulsenumber = (total_pulses * np.ones(2000)).tolist()
            if total_pulses == 0:
                finalphasearray.extend(bob_array)
            else:
                finalphasearray.extend(bob_array)
                pulsenumberarray.extend(pulsenumber)
            total_pulses = total_pulses + 1
            bob = bob + 1000                                # :720
        else:
            bob = bob + 1
        failsafe = failsafe + 1                             # :747
        if failsafe > (maxloops - 1):
            break
    return hits, pulsenumberarray, [float(v) for v in finalphasearray]


def noise_spectrum_loop(qdr_phase_values, nFFTAverages=100, norm1=50.0):
    """ROACH_Pulses.py:521-532 loop-for-loop (Python-2 integer division of the sample count)."""
    nLongsnapSamples = len(qdr_phase_values)
    nSamplesPerFFT = nLongsnapSamples // nFFTAverages
    noiseFFT = np.zeros(nSamplesPerFFT)
    noiseFFTFreqs = np.fft.fftfreq(nSamplesPerFFT)
    for iAvg in range(nFFTAverages):
        noise = np.fft.fft(qdr_phase_values[iAvg * nSamplesPerFFT:(iAvg + 1) * nSamplesPerFFT])
        noise = np.abs(noise)
        noiseFFT += 20 * (np.log10(noise / norm1 / 1e-6))
    noiseFFT /= nFFTAverages
    return noiseFFTFreqs, noiseFFT
