#!/bin/bash
# round 4, call f: k_front3 with 4 transform waves (sub-FFT w of both frames, interleaved) against 8
# (one sub-FFT each): config-3 parity suite on the in-tree FW = 4 library, same-process A/B, stamps
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04f_parity|600|python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k 'chain_parity or fused or speculative'" \
  "r04f_kbench|600|python -u tools/kbench.py --log2-samples 30 --rounds 12 $V/f3_fw8.so $V/f3_fw4.so $V/f3_fw8.so $V/f3_fw4.so > gpurun_out/r04f_kbench.json" \
  "r04f_stamps_fw4|120|python -u tools/stamps4.py $V/st_fw4.so 1024 v3f4"
