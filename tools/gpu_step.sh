#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that ends in a
# time limit, abort, segfault or GPU fault (exit 124/134/137/139 or > 128). Plain test failures
# (exit 1) do not stop the chain. Usage: tools/gpu_step.sh SECS LOG CMD [SECS LOG CMD ...]
mkdir -p gpurun_out
while [ $# -ge 3 ]; do
    secs=$1; log=$2; cmd=$3; shift 3
    echo "[gpu_step] $cmd" > "gpurun_out/$log"
    timeout -k 10 "$secs" bash -c "$cmd" >> "gpurun_out/$log" 2>&1
    rc=$?
    echo "[gpu_step] rc=$rc" >> "gpurun_out/$log"
    echo "$log rc=$rc"
    if [ $rc -ge 2 ]; then echo "stopping after $log"; exit $rc; fi
done
