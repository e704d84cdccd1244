#!/bin/bash
# round 4, call l: trigger with a whole group of raw rows in flight ahead (2 waves per SIMD) vs the
# half-group pipeline (3 waves per SIMD), configs 3 and 2
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04l_kbench_c3|600|python -u tools/kbench.py --log2-samples 30 --rounds 10 $V/base.so $V/trig_deep2.so $V/base.so $V/trig_deep2.so > gpurun_out/r04l_kbench_c3.json" \
  "r04l_kbench_c2|600|python -u tools/kbench.py --channels 256 --log2-samples 28 --rounds 10 $V/base.so $V/trig_deep2.so $V/base.so $V/trig_deep2.so > gpurun_out/r04l_kbench_c2.json"
