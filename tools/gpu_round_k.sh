#!/bin/bash
# Full GPU suite + default bench x3 (bursts of 5).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_k.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -1 gpurun_out/t_k.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_k$r.json 2> gpurun_out/bench_k$r.err || exit 6
python -c "import json;d=json.load(open('gpurun_out/bench_k$r.json'));print('c2', d['value'], round(d['roofline']['launch_ms']*1000,1), d['roofline']['frac'])"
done
