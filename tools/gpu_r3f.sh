#!/bin/bash
# Round 3 final measurement set, call 1: full GPU suite + smoke, the default bench line with a
# same-lease rocprofv3 trace, profiles (trace + PMC) of configs 2 and 3.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 5
echo smoke_ok
bash tools/gpu_measure.sh r3f "2 3" || exit $?
