#!/bin/bash
# Round 3 final verification (after the matrix store diagnostics): full GPU suite + smoke, the default bench line

set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 5
echo smoke_ok; tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r3p_bench.json 2> gpurun_out/r3p_bench.err || exit 6
python -c "import json;d=json.load(open('gpurun_out/r3p_bench.json'));r=d['roofline'];print('cfg2', d['value'], r['launch_ms'], r['frac'], d['parity']['mismatches']);[print(k, v['launch_ms'], v['roofline_frac'], v['parity']['mismatches']) for k,v in d['extras']['configs'].items()]"
