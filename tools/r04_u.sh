#!/bin/bash
# round 4, call u: bench.py's SVF trigger regression of call r (11.9 -> 15.8 ms) was a waterfall
# loop around every SVF warm-up load (the compiler kept the group counter in a VGPR, so the buffer
# load's SGPR row offset looked divergent); fixed with readfirstlane. SVF bench same box: fixed
# library vs round-4 base; kbench config 3 EMA: base / call-r library / fixed library
cd "$GRAFT_REPO_ROOT"
V=build/variants
cp mkids_sdr_amd/libmkidgpu.so /tmp/adopted.so
bash tools/gpu_steps.sh \
  "r04u_svf_fixed|300|python -u bench.py --baseline svf" \
  "r04u_svf_base|300|cp $V/base.so mkids_sdr_amd/libmkidgpu.so && python -u bench.py --baseline svf" \
  "r04u_restore|60|cp /tmp/adopted.so mkids_sdr_amd/libmkidgpu.so" \
  "r04u_kbench_c3|600|python -u tools/kbench.py --log2-samples 30 --rounds 8 $V/base.so $V/r04_trig.so $V/r04_trig2.so > gpurun_out/r04u_kbench_c3.json"
