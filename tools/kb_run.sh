set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/kbench.py --channels 2048 --log2-samples 30 --rounds 4 build/variants/f4_noperm.so build/variants/f4_noperm_plain.so build/variants/f4_perm_plain.so > gpurun_out/kb_f4perm2.json 2> gpurun_out/kb_f4perm2.err
