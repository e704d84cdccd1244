#!/bin/bash
# round 4, call ae: SVF warm-up with 2 / 4 whole groups of rows in flight (run_groups_deep; the
# walk runs at half a wave per SIMD, so the prefetch registers cost no occupancy): SVF parity and
# SVF bench, same box, against the final library
cd "$GRAFT_REPO_ROOT"
V=build/variants
cp mkids_sdr_amd/libmkidgpu.so /tmp/adopted.so
bash tools/gpu_steps.sh \
  "r04ae_svf_base|300|python -u bench.py --baseline svf --no-cpu-baseline" \
  "r04ae_svf_d2|300|cp $V/svf_d2.so mkids_sdr_amd/libmkidgpu.so && python -u bench.py --baseline svf --no-cpu-baseline" \
  "r04ae_svf_d4|300|cp $V/svf_d4.so mkids_sdr_amd/libmkidgpu.so && python -u bench.py --baseline svf --no-cpu-baseline" \
  "r04ae_svf_d4_parity|600|python -u -m pytest tests/test_gpu_svf.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r04ae_restore|60|cp /tmp/adopted.so mkids_sdr_amd/libmkidgpu.so" \
  "r04ae_svf_base2|300|python -u bench.py --baseline svf --no-cpu-baseline"
