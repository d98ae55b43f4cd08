#!/bin/bash
# Round 3 measurement set, call 1: the new GPU tests, the default bench line, a same-lease
# rocprofv3 trace of the primary workload, and the config-3 (pruned) profile with PMC passes.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_api.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_new.log 2>&1
rc=$?; echo "new_tests_rc=$rc"; tail -3 gpurun_out/t_new.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_measure.sh r3a "3" || exit $?
