set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_contexts.py tests/test_gpu_feedlines.py tests/test_gpu_roach.py > gpurun_out/slot_parity.log 2>&1
