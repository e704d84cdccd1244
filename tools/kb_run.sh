set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k "test_chain_parity and 1024" > gpurun_out/f3s_parity.log 2>&1
timeout -k 10 500 python -u tools/kbench.py --channels 1024 --log2-samples 30 --rounds 12 build/variants/f3s.so#MKID_F3_SLOTS=0 build/variants/f3s.so build/variants/f3n.so#n build/variants/f3n.so#a build/variants/f3n.so#b > gpurun_out/kb_slots.json 2> gpurun_out/kb_slots.err
