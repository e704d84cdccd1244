#!/bin/bash
# round 4, call s: SVF trigger after the call-r changes (16 ms vs 12 ms): A/B of the round-4 base,
# the adopted library and the same without the progress priority, SVF baseline at config 3
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04s_kbench_svf|600|python -u tools/kbench.py --baseline svf --log2-samples 30 --rounds 4 $V/base.so $V/r04_trig.so $V/noprio.so > gpurun_out/r04s_kbench_svf.json"
