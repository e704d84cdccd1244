#!/usr/bin/env python3
"""Phase timing of k_front from in-kernel s_memtime stamps (a build with -DMKID_XP_STAMPS).

    make -C mkids_sdr_amd/csrc OUT=../variants/xp_stamps.so EXTRA=-DMKID_XP_STAMPS -B
    python tools/stamps.py mkids_sdr_amd/variants/xp_stamps.so

Lane 0 of each wave of the first 4 workgroups stamps before/after every barrier of iterations
8..15 (k_front.hip, MKID_XP_STAMPS). Prints the mean cycles per segment: work between barriers
and the wait inside each barrier. Timing only: the phase output of that build is garbage.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SEG = [('PFB (ring reads, taps, FMA, dft8)', 14, 0), ('wait S0', 0, 1),
       ('ring refill + pass-1 write', 1, 2), ('wait S1', 2, 3),
       ('pass-2 read', 3, 4), ('wait S2', 4, 5),
       ('pass-2 twiddle+dft8+write', 5, 6), ('wait S3', 6, 7),
       ('pass-3 read', 7, 8), ('wait S4', 8, 9),
       ('pass-3 twiddle+dft8+write', 9, 10), ('wait S5', 10, 11),
       ('select frame 0 (LDS reads, LO load)', 11, 12), ('frames 0-1 LPF + output 0', 12, 13),
       ('frames 2-3 + output 1 + loop', 13, 'next14')]


def main():
    import torch
    from mkids_sdr_amd.channelizer import Channelizer
    lib = os.path.abspath(sys.argv[1])
    C, N = 1024, 2048
    S = 1 << 28
    dev = torch.device('cuda', 0)
    ch = Channelizer(C, max_chunk=S, lib_path=lib)
    x = torch.randint(-2000, 2000, (2 * S,), dtype=torch.int16, device=dev)
    phase = torch.zeros(S // N * C, dtype=torch.float32, device=dev)
    ev = torch.empty(1 << 20, dtype=torch.int64, device=dev)
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    ch.set_thresholds(np.full(C, -(1 << 30), np.int32))
    for _ in range(2):
        phase.zero_()
        ch.process_device(x, S, phase, ev, ev.numel(), cnt)
        torch.cuda.synchronize()
    st = phase[:4 * 16 * 8 * 16 * 2].view(torch.int64).cpu().numpy().reshape(4, 16, 8, 16)
    tot = 0.0
    for name, a, b in SEG:
        if b == 'next14':
            d = st[:, :, 1:, 14] - st[:, :, :-1, a]
        else:
            d = st[:, :, :, b] - st[:, :, :, a]
        m = float(np.mean(d))
        tot += m
        print('%-36s %8.0f cycles  (min %6d max %6d)' % (name, m, int(d.min()), int(d.max())))
    it = st[:, :, 1:, 14] - st[:, :, :-1, 14]
    print('%-36s %8.0f cycles  (sum of segments %.0f)' % ('iteration', float(np.mean(it)), tot))
    ch.close()


if __name__ == '__main__':
    main()
