#!/usr/bin/env python3
"""Phase timing of the wave-specialised front ends (k_front3 'v3', k_front5 'v5') from in-kernel
s_memtime stamps (a build with -DMKID_XP_STAMPS): lane 0 of each wave of workgroups 0-3 stamps
the phase boundaries of iterations 8..15.

    bash tools/build_variant.sh f5_stamps -- -DMKID_XP_STAMPS
    python tools/stamps4.py build/variants/f5_stamps.so 2048 v5
Prints mean cycles per segment over waves and iterations. Timing only: the phase output of that
build holds the stamps.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SEG3 = [('transform waves: PFB + sub-FFT + ring write', 0, 1), ('transform waves: barrier wait', 1, 2),
        ('transform waves: loop back', 2, 'next0'),
        ('select waves: LO + select + DDC + low-pass + output', 3, 4), ('select waves: barrier wait', 4, 5),
        ('select waves: loop back', 5, 'next3')]


SEG5 = [('transform: sub-FFT 0 (ring reads .. Y write)', slice(0, 4), 0, 1, 0),
        ('transform: sub-FFT 1 (+ ring refill)', slice(0, 4), 1, 2, 0),
        ('transform: ring refill', slice(0, 4), 2, 3, 0),
        ('transform: barrier wait', slice(0, 4), 3, 4, 0),
        ('transform: loop back', slice(0, 4), 4, 'next0', 0),
        ('select: LO + select + DDC + low-pass + output', slice(4, 16), 8, 9, 8),
        ('select: barrier wait', slice(4, 16), 9, 10, 8),
        ('select: loop back', slice(4, 16), 10, 'next8', 8)]


def main():
    import torch
    from mkids_sdr_amd.channelizer import Channelizer
    lib = os.path.abspath(sys.argv[1])
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    N = 2 * C
    S = 1 << 28
    dev = torch.device('cuda', 0)
    ch = Channelizer(C, max_chunk=S, lib_path=lib)
    x = torch.randint(-2000, 2000, (2 * S,), dtype=torch.int16, device=dev)
    phase = torch.zeros(S // N * C, dtype=torch.float32, device=dev)
    ev = torch.empty(1 << 20, dtype=torch.int64, device=dev)
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    ch.set_thresholds(np.full(C, -(1 << 30), np.int32))
    for _ in range(3):
        phase.zero_()
        ch.process_device(x, S, phase, ev, ev.numel(), cnt)
        torch.cuda.synchronize()
    if len(sys.argv) > 3 and sys.argv[3] in ('v3', 'v3f4'):
        # k_front3: waves 0-7 transform, 8-15 select ('v3f4': 0-3 transform, 4-11 select)
        nx, nw = (8, 16) if sys.argv[3] == 'v3' else (4, 12)
        st = phase[:4 * 16 * 8 * 16 * 2].view(torch.int64).cpu().numpy().reshape(4, 16, 8, 16)[:, :nw]
        for name, a_, b_ in SEG3:
            w = slice(0, nx) if a_ < 3 else slice(nx, nw)
            top = 0 if a_ < 3 else 3
            x = st[:, w]
            d = x[:, :, 1:, top] - x[:, :, :-1, a_] if str(b_).startswith('next') else x[:, :, :, b_] - x[:, :, :, a_]
            print('%-52s %8.0f cycles  (min %6d max %6d)' % (name, float(np.mean(d)), int(d.min()), int(d.max())))
        if nx == 8 and st[:, :8, :, 7].any():   # decoupled build: the progress-word waits inside the work segments
            for name, w, a_, b_ in (('transform waves: progress-word wait (in segment 1)', slice(0, 8), 6, 7),
                                    ('select waves: progress-word wait (in segment 4)', slice(8, 16), 8, 9)):
                d = st[:, w, :, b_] - st[:, w, :, a_]
                print('%-52s %8.0f cycles  (min %6d max %6d)' % (name, float(np.mean(d)), int(d.min()), int(d.max())))
        work = st[:, :, :, 1] - st[:, :, :, 0] - (st[:, :, :, 7] - st[:, :, :, 6])
        swork = st[:, :, :, 4] - st[:, :, :, 3] - (st[:, :, :, 9] - st[:, :, :, 8])
        print('per-wave mean work cycles (waits excluded), transform waves:',
              ' '.join('%5.0f' % v for v in work[:, :nx].mean(axis=(0, 2))))
        print('per-wave mean work cycles (waits excluded), select waves:   ',
              ' '.join('%5.0f' % v for v in swork[:, nx:].mean(axis=(0, 2))))
        it = st[:, :nx, 1:, 0] - st[:, :nx, :-1, 0]
        print('%-52s %8.0f cycles' % ('iteration (2 frames)', float(np.mean(it))))
        ch.close()
        return
    if len(sys.argv) > 3 and sys.argv[3] == 'v5':   # k_front5: waves 0-3 transform, 4-15 select
        st = phase[:4 * 16 * 8 * 16 * 2].view(torch.int64).cpu().numpy().reshape(4, 16, 8, 16)
        for name, w, a_, b_, top in SEG5:
            x = st[:, w]
            d = x[:, :, 1:, top] - x[:, :, :-1, a_] if str(b_).startswith('next') else x[:, :, :, b_] - x[:, :, :, a_]
            print('%-52s %8.0f cycles  (min %6d max %6d)' % (name, float(np.mean(d)), int(d.min()), int(d.max())))
        it = st[:, :4, 1:, 0] - st[:, :4, :-1, 0]
        print('%-52s %8.0f cycles' % ('iteration (1 frame)', float(np.mean(it))))
        sw = st[:, 4:, :, 9] - st[:, 4:, :, 8]
        print('select work per wave 4..15:', ' '.join('%5.0f' % v for v in sw.mean(axis=(0, 2))))
        nb = (S // (N // 2) + 2047) // 2048
        bs = phase[2 * 8192:2 * (8192 + 4 * 4096)].view(torch.int64).cpu().numpy().reshape(-1, 4)
        bs = bs[:max(1, min(len(bs), int(sys.argv[4]) if len(sys.argv) > 4 else 256))]
        t0 = bs[:, 0].min()
        dur = bs[:, 1] - bs[:, 0]
        print('blocks %d: start offset min/med/max %d/%d/%d, duration min/med/max %d/%d/%d, span %d'
              % (len(bs), 0, int(np.median(bs[:, 0] - t0)), int((bs[:, 0] - t0).max()),
                 int(dur.min()), int(np.median(dur)), int(dur.max()), int(bs[:, 1].max() - t0)))
        np.save(os.path.join(ROOT, 'gpurun_out', 'f5_blocks.npy'), bs)
        ch.close()
        return
    raise SystemExit('usage: stamps4.py LIB [C] v3|v3f4|v5 (k_front3 / k_front5 stamp builds)')

if __name__ == '__main__':
    main()
