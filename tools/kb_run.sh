set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/ > gpurun_out/r03_j_gpu.log 2>&1
