#!/bin/bash
# round 4, call k: k_front3<512> (wave-specialised, config 2) behind MKID_FRONT_V3=1: parity at
# C = 256 (streamed, deleted channels / modes), same-process A/B against k_front2<512>, bench lines
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04k_parity512|600|MKID_FRONT_V3=1 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k '256'" \
  "r04k_kbench512|600|python -u tools/kbench.py --channels 256 --log2-samples 28 --rounds 12 $V/f3n512.so $V/f3n512.so#MKID_FRONT_V3=1 $V/f3n512.so $V/f3n512.so#MKID_FRONT_V3=1 > gpurun_out/r04k_kbench512.json" \
  "r04k_bench_c2_v3|300|MKID_FRONT_V3=1 python -u bench.py --config 2 --no-cpu-baseline" \
  "r04k_bench_c2|300|python -u bench.py --config 2 --no-cpu-baseline"
