#!/bin/bash
# Round-3 rocprofv3 passes: config 3, config 5, config 3 with the SVF baseline (tools/profile.sh).
set -e
TAG=${1:-r03_f}
timeout -k 10 600 bash tools/profile.sh ${TAG}_c3
timeout -k 10 600 bash tools/profile.sh ${TAG}_c5 --config 5
timeout -k 10 600 bash tools/profile.sh ${TAG}_svf --baseline svf
