#!/bin/bash
# round 4, call h: k_front6 (two 768-thread workgroups per CU, one frame per iteration) vs k_front3:
# config-3 parity suite with MKID_FRONT_V6=1, same-process A/B, bench lines both ways
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04h_parity6|600|MKID_FRONT_V6=1 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k 'chain_parity or fused or speculative'" \
  "r04h_kbench|600|python -u tools/kbench.py --log2-samples 30 --rounds 12 $V/f6a.so $V/f6a.so#MKID_FRONT_V6=1 $V/f6a.so $V/f6a.so#MKID_FRONT_V6=1 > gpurun_out/r04h_kbench.json" \
  "r04h_bench6|300|MKID_FRONT_V6=1 python -u bench.py --no-cpu-baseline --cpu-samples-log2 26" \
  "r04h_bench3|300|python -u bench.py --no-cpu-baseline"
