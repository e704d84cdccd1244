#!/bin/bash
# round 4, call ab: SVF matched-filter pre-pass (k_mf_rows writes f as int16 rows; the SVF walk
# reads f instead of filtering: 40 -> 25 VALU per warm-up sample): SVF + baseline-mode parity,
# same-box SVF bench A/B against the previous library, EMA bench unchanged
cd "$GRAFT_REPO_ROOT"
V=build/variants
cp mkids_sdr_amd/libmkidgpu.so /tmp/adopted.so
bash tools/gpu_steps.sh \
  "r04ab_gputest_svf|600|python -u -m pytest tests/test_gpu_svf.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k 'svf or baseline or speculative or fused_deleted'" \
  "r04ab_svf_new|300|python -u bench.py --baseline svf" \
  "r04ab_svf_old|300|cp $V/r04_tmask.so mkids_sdr_amd/libmkidgpu.so && python -u bench.py --baseline svf" \
  "r04ab_restore|60|cp /tmp/adopted.so mkids_sdr_amd/libmkidgpu.so" \
  "r04ab_svf_new2|300|python -u bench.py --baseline svf" \
  "r04ab_svf_new_l64k|300|MKID_SVF_LANES=65536 python -u bench.py --baseline svf --no-cpu-baseline" \
  "r04ab_svf_new_l16k|300|MKID_SVF_LANES=16384 python -u bench.py --baseline svf --no-cpu-baseline" \
  "r04ab_bench_c3|300|python -u bench.py"
