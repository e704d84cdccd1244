#!/bin/bash
# Effective clock of each dispatch (GRBM_GUI_ACTIVE / 8 XCDs / duration) for the EMA and SVF bench
# steps: one rocprofv3 pass with the counter and the kernel trace together.
set -e
ROOT=$(pwd)
export TMPDIR=/tmp
cd /tmp
for MODE in ema svf; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d "$ROOT/gpurun_out/clk_$MODE" -o run \
      --output-format csv -- python3 "$ROOT/bench.py" --no-cpu-baseline --baseline $MODE --steps 5 --warmup 1 \
      > "$ROOT/gpurun_out/clk_$MODE.log" 2>&1
done
