#!/bin/bash
# round 4, call g: full GPU suite on the current tree, the default bench line, rocprof trace + PMC
# passes for configs 3 and 5 (the roofline evidence chain: tools/profile.sh, pmc_summary --summary-out)
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04g_gputest|900|python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=10" \
  "r04g_bench_c3|300|python -u bench.py" \
  "r04g_prof_c3|600|bash tools/profile.sh r04_g_c3 --config 3" \
  "r04g_prof_c5|600|bash tools/profile.sh r04_g_c5 --config 5"
