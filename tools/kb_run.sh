set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/kbench.py --channels 1024 --log2-samples 30 --rounds 15 build/variants/f3_t1vec.so build/variants/f3nm.so build/variants/f3m.so > gpurun_out/kb_f3m2.json 2> gpurun_out/kb_f3m2.err
