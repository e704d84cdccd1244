#!/bin/bash
# Kernel trace of bench.py --baseline svf at a given MKID_SVF_LANES [and MKID_SVF_WARMUP]
# (spec vs fix-up split):
#   bash tools/svf_trace.sh LANES [WARMUP]
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
W=${2:-}
TAG=$1${W:+_w$W}
if [ -n "$W" ]; then export MKID_SVF_WARMUP=$W; fi
MKID_SVF_LANES=$1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/svftr_$TAG \
  -o run --output-format csv -- python3 bench.py --baseline svf --no-cpu-baseline --no-witness --steps 6 --warmup 4 \
  > gpurun_out/svftr_$TAG.log 2>&1
