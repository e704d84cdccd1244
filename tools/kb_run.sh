set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/kbench.py --channels 1024 --log2-samples 30 --rounds 15 build/variants/f3_head.so build/variants/f3_sr.so > gpurun_out/kb_f3sr.json 2> gpurun_out/kb_f3sr.err
timeout -k 10 200 python -u tools/stamps4.py build/variants/f3_sr_stamps.so 1024 v3 > gpurun_out/stamps_f3sr.txt 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k "test_chain_parity and 1024" > gpurun_out/f3sr_parity.log 2>&1
