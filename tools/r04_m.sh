#!/bin/bash
# round 4, call m: minimum trigger segment length (kSegL 2048 / 1024 / 512) at config 2 (C = 256,
# where the 2048 floor leaves one wave per SIMD) and config 3
cd "$GRAFT_REPO_ROOT"
V=build/variants
bash tools/gpu_steps.sh \
  "r04m_kbench_c2|600|python -u tools/kbench.py --channels 256 --log2-samples 28 --rounds 10 $V/base.so $V/segl1024.so $V/segl512.so $V/base.so > gpurun_out/r04m_kbench_c2.json" \
  "r04m_kbench_c3|600|python -u tools/kbench.py --log2-samples 30 --rounds 8 $V/base.so $V/segl1024.so $V/segl512.so > gpurun_out/r04m_kbench_c3.json"
