#!/bin/bash
# round 4, call y: k_front3 ring refill moved onto the older transform wave of each SIMD (the
# younger one is the iteration's critical chain, r04_e stamps): parity at config 3 + same-box A/B
cd "$GRAFT_REPO_ROOT"
V=build/variants
cp mkids_sdr_amd/libmkidgpu.so /tmp/adopted.so
bash tools/gpu_steps.sh \
  "r04y_kbench_c3|600|python -u tools/kbench.py --log2-samples 30 --rounds 12 $V/r04_trig3.so $V/f3_refold.so $V/r04_trig3.so $V/f3_refold.so > gpurun_out/r04y_kbench_c3.json" \
  "r04y_parity_refold|600|cp $V/f3_refold.so mkids_sdr_amd/libmkidgpu.so && python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'fused or witness or 2048 or chain'" \
  "r04y_restore|60|cp /tmp/adopted.so mkids_sdr_amd/libmkidgpu.so"
