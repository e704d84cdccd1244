#!/bin/bash
# round 4, call ah: the trigger at 4 waves per SIMD adopted: full GPU suite, smoke, bench lines
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04ah_gputest|900|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=10" \
  "r04ah_smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "r04ah_bench_c3|300|python -u bench.py" \
  "r04ah_bench_c2|300|python -u bench.py --config 2" \
  "r04ah_bench_c5|300|python -u bench.py --config 5" \
  "r04ah_bench_svf|300|python -u bench.py --baseline svf"
