#!/bin/bash
# round 4, call t: bench.py --baseline svf, same box, adopted library vs round-4 base vs adopted
# (the call-r SVF line was 33 % slower in the trigger than call j's, on another box)
cd "$GRAFT_REPO_ROOT"
cp mkids_sdr_amd/libmkidgpu.so /tmp/adopted.so
bash tools/gpu_steps.sh \
  "r04t_svf_adopted1|300|python -u bench.py --baseline svf" \
  "r04t_svf_base|300|cp build/variants/base.so mkids_sdr_amd/libmkidgpu.so && python -u bench.py --baseline svf" \
  "r04t_svf_adopted2|300|cp /tmp/adopted.so mkids_sdr_amd/libmkidgpu.so && python -u bench.py --baseline svf"
