#!/bin/bash
# round 4, call ac: the round's final library (SVF filter pre-pass, rows allocated on first SVF
# use): full GPU suite, smoke, bench lines for configs 3, 2, 5 and SVF
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04ac_gputest|900|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=10" \
  "r04ac_smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "r04ac_bench_c3|300|python -u bench.py" \
  "r04ac_bench_c2|300|python -u bench.py --config 2" \
  "r04ac_bench_c5|300|python -u bench.py --config 5" \
  "r04ac_bench_svf|300|python -u bench.py --baseline svf"
