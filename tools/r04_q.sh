#!/bin/bash
# round 4, call q: trigger priority thresholds, second pass (P1/P2/P3 = 50/75/90, 60/80/95,
# 70/85/95, 80/90/97) at config 3 and at 2048 channels (config 5's trigger geometry)
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04q_kbench_c3|600|python -u tools/kbench.py --log2-samples 30 --rounds 8 $V/t_mb.so $V/p_50.so $V/p_60.so $V/p_70.so $V/p_80.so > gpurun_out/r04q_kbench_c3.json" \
  "r04q_kbench_ch2048|600|python -u tools/kbench.py --channels 2048 --log2-samples 30 --rounds 6 $V/base.so $V/t_mb.so $V/p_60.so $V/p_70.so > gpurun_out/r04q_kbench_ch2048.json"
