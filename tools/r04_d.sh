#!/bin/bash
# round 4, call d: why the pair ring does not pay: stamps + PMC of the round-3 k_front3 and the
# pair-ring build (plain select I/O)
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04d_stamps_r03|120|python -u tools/stamps4.py $V/st_r03.so 1024 v3" \
  "r04d_stamps_pair|120|python -u tools/stamps4.py $V/st_pair.so 1024 v3" \
  "r04d_pmc_r03|300|bash tools/pmc_variant.sh r03 $V/f3_r03b.so" \
  "r04d_pmc_pair|300|bash tools/pmc_variant.sh pair $V/f3_pair_plainio.so"
