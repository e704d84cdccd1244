set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/stamps.py build/kb/xp_stamps.so > gpurun_out/stamps_v23.txt 2>&1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_v23
mkdir -p $OUT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES -d $OUT/lds -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $OUT/lds.log 2>&1
