#!/bin/bash
# round 4, call c: split the pair-ring / buffer-I/O A/B into its two parts (same process, 12 rounds)
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04c_kbench|600|python -u tools/kbench.py --log2-samples 30 --rounds 12 $V/f3_r03.so $V/f3_r03_bufio.so $V/f3_pair_plainio.so $V/f3_pair.so > gpurun_out/r04c_kbench.json"
