#!/bin/bash
# round 4, call ai: roofline evidence for the final library: rocprofv3 trace + PMC of configs 3, 5
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04ai_prof_c3|600|bash tools/profile.sh r04_ai_c3 --config 3" \
  "r04ai_prof_c5|600|bash tools/profile.sh r04_ai_c5 --config 5"
# and the progress-priority thresholds at 4 waves per SIMD (P1/P2/P3 = 50/75/90, 70/85/95, 85/93/98)
V=build/variants
bash tools/gpu_steps.sh \
  "r04ai_kbench_prio_c3|600|python -u tools/kbench.py --log2-samples 30 --rounds 8 $V/r04_final.so $V/pr50.so $V/pr85.so $V/r04_final.so > gpurun_out/r04ai_kbench_prio_c3.json"
