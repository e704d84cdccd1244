#!/bin/bash
# round 4, call r: the trigger changes of calls n-q adopted (zero-accumulator dot2, med3 clamp,
# buffer loads with SGPR row offsets, progress-ordered issue priority, kSegL 1024): full GPU suite,
# bench lines for configs 3, 2, 5 and SVF
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04r_gputest|900|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=10" \
  "r04r_bench_c3|300|python -u bench.py" \
  "r04r_bench_c2|300|python -u bench.py --config 2" \
  "r04r_bench_c5|300|python -u bench.py --config 5" \
  "r04r_bench_svf|300|python -u bench.py --baseline svf"
