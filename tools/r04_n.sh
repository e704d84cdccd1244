#!/bin/bash
# round 4, call n: branch-free emitting trigger loop (deferred packet re-step from LDS-held
# filtered samples), buffer loads with SGPR row offsets, med3 clamp, zero-accumulator first dot2;
# full GPU suite on it, then same-process A/B against the round-4 base, the dot2-only step, the
# L2-hit what-if and the kSegL variants
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04n_gputest|900|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
  "r04n_kbench_c3|600|python -u tools/kbench.py --log2-samples 30 --rounds 8 $V/base.so $V/trignb.so $V/dot2f.so $V/wi_trig_l2.so $V/segl1024.so $V/trignb.so > gpurun_out/r04n_kbench_c3.json" \
  "r04n_kbench_c2|600|python -u tools/kbench.py --channels 256 --log2-samples 28 --rounds 10 $V/base.so $V/trignb.so $V/segl1024.so $V/segl512.so $V/trignb.so > gpurun_out/r04n_kbench_c2.json"
