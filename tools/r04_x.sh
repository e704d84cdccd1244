#!/bin/bash
# round 4, call x: roofline evidence for the current library at the new default warm-up (10 steps):
# rocprofv3 kernel trace + PMC passes for configs 3 and 5 (tools/profile.sh)
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04x_prof_c3|600|bash tools/profile.sh r04_x_c3 --config 3" \
  "r04x_prof_c5|600|bash tools/profile.sh r04_x_c5 --config 5"
