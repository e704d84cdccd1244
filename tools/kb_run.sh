set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/kbench.py --channels 256 --log2-samples 28 --rounds 12 build/variants/f2n.so build/variants/f2p.so > gpurun_out/kb_f2p_256.json 2> gpurun_out/kb_f2p_256.err
timeout -k 10 300 python -u tools/kbench.py --channels 512 --log2-samples 29 --rounds 10 build/variants/f2n.so build/variants/f2p.so > gpurun_out/kb_f2p_512.json 2> gpurun_out/kb_f2p_512.err
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/f2p_parity.log 2>&1
