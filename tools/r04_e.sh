#!/bin/bash
# round 4, call e: k_front3 stamps (phase-store guard fixed) and what-if builds (no LO loads / no
# raw+phase stores) against the round-3 kernel and the pair ring
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04e_stamps_r03|120|python -u tools/stamps4.py $V/st_r03.so 1024 v3" \
  "r04e_stamps_pair|120|python -u tools/stamps4.py $V/st_pair.so 1024 v3" \
  "r04e_kbench|600|python -u tools/kbench.py --log2-samples 30 --rounds 10 $V/f3_r03b.so $V/wi_r03_nolo.so $V/wi_r03_nost.so $V/f3_pair_plainio.so > gpurun_out/r04e_kbench.json"
