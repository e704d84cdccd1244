#!/bin/bash
# Round-3 rocprofv3 passes: config 3, config 5, config 3 with the SVF baseline (tools/profile.sh).
set -e
timeout -k 10 600 bash tools/profile.sh r03_f_c3
timeout -k 10 600 bash tools/profile.sh r03_f_c5 --config 5
timeout -k 10 600 bash tools/profile.sh r03_f_svf --baseline svf
