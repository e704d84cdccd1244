set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/kbench.py --channels 1024 --log2-samples 30 --rounds 10 build/variants/mf1.so build/variants/mf2.so build/variants/mf3.so > gpurun_out/kb_mf.json 2> gpurun_out/kb_mf.err
