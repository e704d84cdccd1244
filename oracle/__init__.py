"""CPU oracle for the MKID channeliser + pulse-trigger hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
anything under ``oracle/``, and only as the checker (or the timed CPU baseline), never as the
thing measured or shipped. The product path (``mkids_sdr_amd``) never imports this package and
fails loudly when its HIP library is missing.

Contents
  setup_ref.py  restatement of the reference's host setup math (ROACH_Setup.py / ROACH_Pulses.py /
                Utils/bin.py), written loop-for-loop after the reference so it can be pinned by the
                reference's own fixtures (dac.npy.npz bit-exact, castBin constants, peakfit).
  chain.py      numpy float64 restatement of the absent firmware chain K1-K6 (PFB, FFT, bin
                select, DDC, IQ low-pass /2, centre + atan2, Fix16_13 quantisation).
  trigger.c     C restatement of K7/K8 (matched filter, EMA/SVF baseline, threshold, peak fit,
                packets); trigger_ref.py is the pure-Python twin used to pin trigger.c.
  replay.py     the reference's host numpy replays (rolling-mean / block-mean triggers,
                pulse_triggering_v2.py:104-174, pulse_triggering.py:109-208).

Parity status: the LUT / bin / quantisation / threshold / trigger / packet layers are pinned by
reference fixtures and by the reference's importable Utils/bin.py (tests/golden/make_golden.py).
PFB -> phase arithmetic is pinned only against this restatement: the firmware is absent from the
reference (.MISSING_LARGE_BLOBS:1-27), so its taps/window are build decisions.
"""
