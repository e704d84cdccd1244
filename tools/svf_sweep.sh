#!/bin/bash
# SVF trigger geometry sweep on the GPU box: bench.py --baseline svf under MKID_SVF_WARMUP /
# MKID_SVF_LANES (mkid_api.hip plan_sub), one short run each; prints ms/step, kernel times, re-runs.
#   bash tools/svf_sweep.sh "W1 W2 ..." "LANES1 LANES2 ..."
set -e
cd "${GRAFT_REPO_ROOT:-.}"
for w in $1; do for l in $2; do
  echo "W=$w LANES=$l $(MKID_SVF_WARMUP=$w MKID_SVF_LANES=$l timeout -k 10 120 python bench.py --baseline svf \
    --no-cpu-baseline --steps 3 --warmup 1 2>/dev/null | python3 -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["kernel_ms"], d["trigger_segments_rerun"])')"
done; done
