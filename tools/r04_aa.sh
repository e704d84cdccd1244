#!/bin/bash
# round 4, call aa: bench.py times only the front end inside the timed steps (per-kernel
# breakdown from the last warm-up steps); timing-mask / per-call counts test; smoke; bench lines
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04aa_gputest_ctx|600|python -u -m pytest tests/test_gpu_contexts.py tests/test_gpu_bench_multi.py -m gpu -x -v --timeout 300 --timeout-method thread" \
  "r04aa_smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "r04aa_bench_c3|300|python -u bench.py" \
  "r04aa_bench_c2|300|python -u bench.py --config 2" \
  "r04aa_bench_c5|300|python -u bench.py --config 5" \
  "r04aa_bench_svf|300|python -u bench.py --baseline svf"
