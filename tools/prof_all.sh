#!/bin/bash
# rocprofv3 passes of the bench configs: config 3, config 5, config 3 with the SVF baseline
# (tools/profile.sh), e.g. bash tools/prof_all.sh r05_x
set -e
TAG=${1:-r05}
timeout -k 10 600 bash tools/profile.sh ${TAG}_c3
timeout -k 10 600 bash tools/profile.sh ${TAG}_c5 --config 5
timeout -k 10 600 bash tools/profile.sh ${TAG}_svf --baseline svf
