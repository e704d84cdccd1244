#!/bin/bash
# round 4, call ag: the EMA trigger at 4 waves per SIMD (launch bounds -> 128 VGPRs, 9 spilled
# dwords; the plan sizes segments from the occupancy, so 4/3 as many segments) vs 3 waves
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04ag_kbench_c3|600|python -u tools/kbench.py --log2-samples 30 --rounds 8 $V/r04_final.so $V/trig_w4.so $V/r04_final.so $V/trig_w4.so > gpurun_out/r04ag_kbench_c3.json" \
  "r04ag_kbench_c2|600|python -u tools/kbench.py --channels 256 --log2-samples 28 --rounds 10 $V/r04_final.so $V/trig_w4.so > gpurun_out/r04ag_kbench_c2.json" \
  "r04ag_kbench_ch2048|600|python -u tools/kbench.py --channels 2048 --log2-samples 30 --rounds 6 $V/r04_final.so $V/trig_w4.so > gpurun_out/r04ag_kbench_ch2048.json"
