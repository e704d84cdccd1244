#!/bin/bash
# round 4, call p: trigger issue priority by segment progress (s_setprio 3 -> 0 at the P1/P2/P3
# percent marks) on top of t_mb (zero-accumulator dot2, med3 clamp, buffer loads, kSegL 1024)
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04p_kbench_c3|600|python -u tools/kbench.py --log2-samples 30 --rounds 8 $V/base.so $V/t_mb.so $V/p_40.so $V/p_25.so $V/p_60.so > gpurun_out/r04p_kbench_c3.json" \
  "r04p_kbench_c2|600|python -u tools/kbench.py --channels 256 --log2-samples 28 --rounds 10 $V/base.so $V/t_mb.so $V/p_40.so $V/p_25.so $V/p_60.so > gpurun_out/r04p_kbench_c2.json"
