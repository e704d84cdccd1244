#!/bin/bash
# round 4, call v: (1) PMC of the adopted trigger at 2^30 (wave lifetime vs kernel after the
# progress priority); (2) why bench.py's config-2 front end (1.09-1.14 ms) is slower than
# kbench's (0.95 ms): rocprofv3 kernel traces of both harnesses on the same box
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
ROOT=$(pwd)
LOG2=30 bash tools/pmc_variant.sh trig_final30 build/variants/r04_trig2.so || exit $?
mkdir -p gpurun_out/r04v
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r04v/bench_c2" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline --config 2 --steps 10 --warmup 2 > "$ROOT/gpurun_out/r04v/bench_c2.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r04v/kbench_c2" -o run --output-format csv \
    -- python3 "$ROOT/tools/kbench.py" --channels 256 --log2-samples 28 --rounds 10 "$ROOT/mkids_sdr_amd/libmkidgpu.so" > "$ROOT/gpurun_out/r04v/kbench_c2.log" 2>&1 || exit $?
echo done
