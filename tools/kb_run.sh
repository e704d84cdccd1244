set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/kbench.py --channels 2048 --log2-samples 30 --rounds 5 build/variants/t1_off.so build/variants/t1_on.so > gpurun_out/kb_t1_c5.json 2> gpurun_out/kb_t1_c5.err
timeout -k 10 300 python -u tools/kbench.py --channels 256 --log2-samples 28 --rounds 6 build/variants/t1_off.so build/variants/t1_on.so > gpurun_out/kb_t1_c2.json 2> gpurun_out/kb_t1_c2.err
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k "test_chain_parity or front2_at_2048" > gpurun_out/t1b_parity.log 2>&1
