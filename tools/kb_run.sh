set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/ > gpurun_out/r03_i_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_i_smoke.log 2>&1
