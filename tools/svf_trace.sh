#!/bin/bash
# Kernel trace of bench.py --baseline svf at a given MKID_SVF_LANES (spec vs fix-up split):
#   bash tools/svf_trace.sh LANES
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
MKID_SVF_LANES=$1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/svftr_$1 -o run --output-format csv \
  -- python3 bench.py --baseline svf --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/svftr_$1.log 2>&1
