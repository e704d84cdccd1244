"""Generate the committed golden fixtures under tests/golden/ from the reference checkout.

Run in the build container only (the GPU box has no /root/reference):
    python tests/golden/make_golden.py [/root/reference]
What it writes (all data, no reference source):
  dac_lut.npz           the reference's own saved LUTs (DataReadout/ChannelizerControls/dac.npy.npz,
                        written by ROACH_Setup.py:558), re-stored as int16.
  ch_snap_0.txt         the reference's saved 2048-sample phase snapshot (ROACH_Pulses.py:482-484).
  ch_noifreqs_0.txt     the reference's saved noise-FFT frequency axis (ROACH_Pulses.py:532-534).
  fir/*.txt             the reference's FIR tap files (DataReadout/ChannelizerControls/LUT/).
  1tones.txt            the reference's frequency file (LUT/1tones.txt).
  bin_vectors.json      outputs of the reference's Utils/bin.py castBin / peakfit, imported and
                        executed here under Python 3 (uint path only: extractBin's line-22 `/` is
                        Python-2 integer division, see oracle/setup_ref.extract_bin), on inputs
                        that avoid exact .5 rounding ties (py2/py3 round() differ only there).
"""
import json
import os
import shutil
import sys

import numpy as np

REF = sys.argv[1] if len(sys.argv) > 1 else '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))
CC = os.path.join(REF, 'DataReadout', 'ChannelizerControls')


def main():
    d = np.load(os.path.join(CC, 'dac.npy.npz'), allow_pickle=False)
    np.savez_compressed(os.path.join(HERE, 'dac_lut.npz'),
                        **{k: d[k].astype(np.int16) for k in ('I_dac', 'Q_dac', 'I_dds', 'Q_dds')})
    for f in ('ch_snap_0.txt', 'ch_noifreqs_0.txt'):
        shutil.copy(os.path.join(CC, f), os.path.join(HERE, f))
    for f in os.listdir(os.path.join(CC, 'LUT')):
        if f.endswith('Filter_250kHz.txt') or f.startswith('matched'):
            shutil.copy(os.path.join(CC, 'LUT', f), os.path.join(HERE, 'fir', f))
    shutil.copy(os.path.join(CC, 'LUT', '1tones.txt'), os.path.join(HERE, '1tones.txt'))

    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    from Utils import bin as refbin  # the reference's own module

    rng = np.random.default_rng(20261015)
    cases = []
    for nbits, bp in ((12, 9), (16, 13), (18, 16), (12, 11)):
        for v in rng.uniform(-3.9, 3.9, 40):
            v = float(v)
            for q in ('Round', 'Truncate'):
                cases.append(dict(value=v, nBits=nbits, binaryPoint=bp, quantization=q,
                                  out=int(refbin.castBin(v, nBits=nbits, binaryPoint=bp,
                                                         quantization=q, format='uint'))))
    registers = dict(
        kf=int(refbin.castBin(2 * np.sin(np.pi * 200 / 1e6), quantization='Round', nBits=18,
                              binaryPoint=16, format='uint')),
        kq=int(refbin.castBin(1. / .7, quantization='Round', nBits=18, binaryPoint=16,
                              format='uint')),
        alpha=int(refbin.castBin(0.08, quantization='Round')),
        base_thresh=int(refbin.castBin(1., quantization='Round', nBits=16, binaryPoint=13)))
    peaks = []
    for _ in range(200):
        y = [float(v) for v in rng.integers(-3000, 3000, 3)]
        peaks.append(dict(y=y, out=float(refbin.peakfit(*y))))
    peaks.append(dict(y=[1.0, 3.0, 2.0], out=float(refbin.peakfit(1, 3, 2))))
    peaks.append(dict(y=[1.0, 2.0, 3.0], out=float(refbin.peakfit(1, 2, 3))))
    degs = [dict(x=int(x), out=float(refbin.bin12_9ToDeg(int(x)))) for x in (0, 1, 2047, 2048, 4095)]
    with open(os.path.join(HERE, 'bin_vectors.json'), 'w') as f:
        json.dump(dict(source='Utils/bin.py (reference), executed under Python 3 by make_golden.py',
                       castBin=cases, registers=registers, peakfit=peaks, bin12_9ToDeg=degs),
                  f, indent=0)
    print('golden fixtures written to', HERE)


if __name__ == '__main__':
    main()
