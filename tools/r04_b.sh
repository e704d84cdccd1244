#!/bin/bash
# round 4, call b: k_front3 pair ring + buffer-descriptor select I/O: parity subset on the new
# library, same-process A/B against the round-3 kernel (build/variants/f3_r03.so, tools/build_rev.sh),
# bench line
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04b_parity|600|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_refpins.py tests/test_gpu_roach.py -x -v --timeout 200 --timeout-method thread" \
  "r04b_kbench|600|python -u tools/kbench.py --log2-samples 30 --rounds 10 build/variants/f3_r03.so build/variants/f3_pair.so > gpurun_out/r04b_kbench.json" \
  "r04b_bench_c3|300|python -u bench.py"
