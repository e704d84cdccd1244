set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/stamps4.py build/variants/f3_stamps.so 1024 v3 > gpurun_out/stamps_f3.txt 2>&1
timeout -k 10 300 python -u tools/kbench.py --channels 1024 --log2-samples 30 --rounds 5 build/variants/f3.so build/variants/f3_px.so build/variants/f3_ps.so > gpurun_out/kb_f3p.json 2> gpurun_out/kb_f3p.err
