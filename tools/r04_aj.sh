#!/bin/bash
# round 4, call aj: EMA trigger warm-up at 4 waves per SIMD (kSegW 208 / 260 / 312 samples:
# shorter segments made the warm-up a larger share); reruns reported per variant
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04aj_kbench_c3|600|python -u tools/kbench.py --log2-samples 30 --rounds 8 $V/r04_final.so $V/segw208.so $V/segw312.so $V/r04_final.so > gpurun_out/r04aj_kbench_c3.json" \
  "r04aj_kbench_ch2048|600|python -u tools/kbench.py --channels 2048 --log2-samples 30 --rounds 6 $V/r04_final.so $V/segw208.so $V/segw312.so > gpurun_out/r04aj_kbench_ch2048.json"
