#!/bin/bash
# rocprofv3 passes over bench.py on the GPU box (run through gpurun from the repo root):
#   bash tools/profile.sh TAG [extra bench.py args, e.g. --config 5]
# 1. kernel trace + stats of the default bench workload (per-kernel average durations);
# 2. PMC passes, each its own run (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950;
#    counters are never combined with runtime/sys traces), on one default (2^30-sample) step.
# Output: gpurun_out/prof_TAG/{kt,fetch,write,sq1,sq2}/...
set -euo pipefail
TAG=${1:-run}
shift || true
# one profiled rank per invocation: bench.py --gpus N > 1 would start its ranks from a process the
# profiler's preloaded library has already attached to the GPU
for a in "$@"; do
    if [ "$a" = "--gpus" ]; then echo "profile.sh: profile one rank (no --gpus)" >&2; exit 2; fi
done
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B="python3 $ROOT/bench.py --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv \
    -- $B --steps 10 --warmup 10 > "$OUT/kt.log" 2>&1
SMALL="--steps 1 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
    -- $B $SMALL > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
    -- $B $SMALL > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d "$OUT/sq1" -o run \
    --output-format csv -- $B $SMALL > "$OUT/sq1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES \
    SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d "$OUT/sq2" -o run \
    --output-format csv -- $B $SMALL > "$OUT/sq2.log" 2>&1
echo "profile passes done: $OUT"
