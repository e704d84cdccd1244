#!/bin/bash
# round 4, call af: rocprofv3 kernel trace of the SVF bench (where the 11.7 ms trigger goes:
# k_mf_rows / k_trig_spec<SVF> / k_trig_fix per launch)
cd "$GRAFT_REPO_ROOT"
ROOT=$(pwd)
mkdir -p gpurun_out/r04af
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r04af/svf" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline --baseline svf --steps 5 --warmup 3 > "$ROOT/gpurun_out/r04af/svf.log" 2>&1
