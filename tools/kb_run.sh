set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/kbench.py --channels 1024 --log2-samples 30 --rounds 15 build/variants/f3_head.so build/variants/f3_tw.so build/variants/f3_tw_pr.so > gpurun_out/kb_twpr.json 2> gpurun_out/kb_twpr.err
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k "test_chain_parity and 1024" > gpurun_out/twpr_parity.log 2>&1
