#!/bin/bash
# GPU session: the given test files first (fast feedback), then the full -m gpu suite + smoke.
#   bash tools/gpu_tests.sh [tests/test_x.py ...]
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_new.log 2>&1
  rc=$?; echo "new_rc=$rc"; tail -5 gpurun_out/t_new.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 5
echo smoke_ok
