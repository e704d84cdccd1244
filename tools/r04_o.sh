#!/bin/bash
# round 4, call o: the trigger's three loop changes one at a time on top of the zero-accumulator
# dot2 (t_d, kSegL 1024): m = med3 clamp, b = buffer loads with SGPR row offsets, d = branch-free
# emitting loop with deferred packet re-step; base = round-4 library (kSegL 2048)
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04o_kbench_c3|600|python -u tools/kbench.py --log2-samples 30 --rounds 6 $V/base.so $V/t_d.so $V/t_dm.so $V/t_db.so $V/t_dd.so $V/t_dmb.so $V/t_all.so > gpurun_out/r04o_kbench_c3.json" \
  "r04o_kbench_c2|600|python -u tools/kbench.py --channels 256 --log2-samples 28 --rounds 10 $V/base.so $V/t_d.so $V/t_dm.so $V/t_db.so $V/t_dd.so $V/t_dmb.so $V/t_all.so > gpurun_out/r04o_kbench_c2.json"
