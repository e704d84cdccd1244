#!/bin/bash
# round 4, call i: what-if bounds for k_front3's LDS ring (no ring reads / no refill writes)
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04i_kbench|600|python -u tools/kbench.py --log2-samples 30 --rounds 10 $V/f6a.so $V/wi_noring.so $V/wi_norefill.so $V/f6a.so > gpurun_out/r04i_kbench.json"
