#!/bin/bash
# Sparse-program tile layout A/B on config 2 (processing order vs vocabulary order), parity first.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_slowpath.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_qlayout.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/t_qlayout.log; [ $rc -eq 0 ] || exit $rc
for v in slot vocab slot vocab slot; do
  DICE_PROG_QLAYOUT=$v timeout -k 10 300 python bench.py --steps 50 --warmup 5 --extra-configs= --no-cpu-baseline > gpurun_out/ql_$v.json 2> gpurun_out/ql_$v.err || exit 10
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['roofline']['launch_ms']*1e3,2), 'us', round(d['roofline']['frac'],4))" gpurun_out/ql_$v.json
done
