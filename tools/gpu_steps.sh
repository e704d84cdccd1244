#!/bin/bash
# Run GPU steps in sequence on the gpurun box, each under its own time limit; ordinary failures
# (pytest failures, rc < 124) continue, a time limit / abort / fault (rc >= 124) ends the script.
#   bash tools/gpu_steps.sh 'name|seconds|command' ...
mkdir -p gpurun_out
for spec in "$@"; do
    name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
    start=$(date +%s)
    timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "$name rc=$rc $(( $(date +%s) - start ))s"
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
done
