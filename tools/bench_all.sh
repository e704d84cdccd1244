#!/bin/bash
# Bench lines of every BASELINE config (run through gpurun from the repo root): configs 3/5/2 and
# SVF with CPU baselines + parity witness, SVF with a 49k-sample warm-up (no CPU leg).
#   bash tools/bench_all.sh TAG
TAG=${1:-r05}
bash tools/gpu_steps.sh \
  "${TAG}_bench_c3|280|python -u bench.py --steps 10 > gpurun_out/${TAG}_bench_c3.jsonl" \
  "${TAG}_bench_c5|280|python -u bench.py --config 5 --steps 10 > gpurun_out/${TAG}_bench_c5.jsonl" \
  "${TAG}_bench_c2|280|python -u bench.py --config 2 --steps 10 > gpurun_out/${TAG}_bench_c2.jsonl" \
  "${TAG}_bench_svf|280|python -u bench.py --baseline svf --steps 10 > gpurun_out/${TAG}_bench_svf.jsonl" \
  "${TAG}_bench_svf49k|200|MKID_SVF_WARMUP=49140 python -u bench.py --baseline svf --steps 10 --no-cpu-baseline > gpurun_out/${TAG}_bench_svf49k.jsonl"
