#!/bin/bash
# round 4, call a: GPU suite (incl. the self-launched 2-rank bench and the world-1 RCCL gather),
# the default bench line, and the gather's cost at config 3 (plain vs --force-gather, alternating)
cd "$GRAFT_REPO_ROOT"
B="python -u bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline --copy-mib 256"
bash tools/gpu_steps.sh \
  "r04a_gputest|900|python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=15" \
  "r04a_bench_c3|300|python -u bench.py" \
  "r04a_plain1|120|$B" \
  "r04a_force1|120|$B --force-gather --backend nccl --check-gather" \
  "r04a_plain2|120|$B" \
  "r04a_force2|120|$B --force-gather --backend nccl --check-gather"
