#!/bin/bash
# round 4, call z: fewer launches per call (history rolls into the spare buffer + pointer swap
# instead of device-to-device copies, the call's two rolls in one launch, packet counts written by
# the compaction instead of a zeroing memset): full GPU suite, same-box A/B at configs 2 and 3,
# bench lines
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04z_gputest|900|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=10" \
  "r04z_kbench_c2|600|python -u tools/kbench.py --channels 256 --log2-samples 28 --rounds 12 $V/r04_trig3.so $V/r04_launch.so $V/r04_trig3.so $V/r04_launch.so > gpurun_out/r04z_kbench_c2.json" \
  "r04z_kbench_c3|600|python -u tools/kbench.py --log2-samples 30 --rounds 8 $V/r04_trig3.so $V/r04_launch.so > gpurun_out/r04z_kbench_c3.json" \
  "r04z_bench_c2|300|python -u bench.py --config 2" \
  "r04z_bench_c3|300|python -u bench.py"
