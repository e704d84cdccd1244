set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/stamps4.py build/variants/f4_stamps.so 2048 > gpurun_out/stamps_f4.txt 2>&1
timeout -k 10 200 python -u tools/stamps4.py build/variants/f2_stamps.so 1024 > gpurun_out/stamps_f2.txt 2>&1
