#!/bin/bash
# PMC passes over one library build (tools/kbench.py, one variant, 2^LOG2 samples, default 28):
#   [LOG2=30] [CH=2048] bash tools/pmc_variant.sh NAME build/variants/NAME.so
# Output: gpurun_out/pmcv_NAME/{sq1,sq2}/...; summarise with
#   python tools/pmc_summary.py gpurun_out/pmcv_NAME --config 3 --samples-log2 28
set -euo pipefail
NAME=$1; LIB=$(cd "$(dirname "$2")" && pwd)/$(basename "$2")
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmcv_$NAME
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
K="python3 $ROOT/tools/kbench.py --log2-samples ${LOG2:-28} --channels ${CH:-1024} --rounds 2 $LIB"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d "$OUT/sq1" -o run \
    --output-format csv -- $K > "$OUT/sq1.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES \
    SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d "$OUT/sq2" -o run \
    --output-format csv -- $K > "$OUT/sq2.log" 2>&1
echo "pmc passes done: $OUT"
