#!/bin/bash
# round 4, call w: trigger row offsets made uniform once per half group (no VALU add +
# readfirstlane per load): parity + SVF tests, same-box A/B, and bench lines with the new default
# warm-up of 10 steps
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04w_gputest_trig|600|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_svf.py -m gpu -x -v --timeout 300 --timeout-method thread" \
  "r04w_kbench_c3|600|python -u tools/kbench.py --log2-samples 30 --rounds 8 $V/base.so $V/r04_trig2.so $V/r04_trig3.so > gpurun_out/r04w_kbench_c3.json" \
  "r04w_bench_c3|300|python -u bench.py" \
  "r04w_bench_c2|300|python -u bench.py --config 2" \
  "r04w_bench_c5|300|python -u bench.py --config 5" \
  "r04w_bench_svf|300|python -u bench.py --baseline svf"
