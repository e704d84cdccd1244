#!/bin/bash
# round 4, call ad: the round's final library (full GPU suite, smoke, bench lines for configs 3,
# 2, 5, SVF), then the experimental exact-fp64 SVF base-only warm-up (-DMKID_SVF_F64): SVF parity
# and SVF bench on the same box
cd "$GRAFT_REPO_ROOT"
V=build/variants
cp mkids_sdr_amd/libmkidgpu.so /tmp/adopted.so
bash tools/gpu_steps.sh \
  "r04ac_gputest|900|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=10" \
  "r04ac_smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "r04ac_bench_c3|300|python -u bench.py" \
  "r04ac_bench_c2|300|python -u bench.py --config 2" \
  "r04ac_bench_c5|300|python -u bench.py --config 5" \
  "r04ac_bench_svf|300|python -u bench.py --baseline svf" \
  "r04ad_svf_f64_bench|300|cp $V/svf_f64.so mkids_sdr_amd/libmkidgpu.so && python -u bench.py --baseline svf --no-cpu-baseline" \
  "r04ad_svf_f64_parity|600|python -u -m pytest tests/test_gpu_svf.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r04ad_restore|60|cp /tmp/adopted.so mkids_sdr_amd/libmkidgpu.so"
