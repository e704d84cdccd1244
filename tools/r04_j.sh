#!/bin/bash
# round 4, call j: the GPU tests after test_gpu_roach (the suite stopped there in call g), trigger
# warm-up length A/B (kSegW 520 / 260 / 130), bench lines for configs 2 and 5 and SVF
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04j_gputest_tail|600|python -u -m pytest tests/test_gpu_roach.py tests/test_gpu_svf.py tests/test_heights.py tests/test_template.py -m gpu -x -v --timeout 200 --timeout-method thread" \
  "r04j_kbench_segw|600|python -u tools/kbench.py --log2-samples 30 --rounds 10 $V/base.so $V/segw260.so $V/segw130.so $V/base.so > gpurun_out/r04j_kbench_segw.json" \
  "r04j_bench_c2|300|python -u bench.py --config 2" \
  "r04j_bench_c5|300|python -u bench.py --config 5" \
  "r04j_bench_svf|300|python -u bench.py --baseline svf"
