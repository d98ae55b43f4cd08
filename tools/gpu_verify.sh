#!/bin/bash
# GPU session: full gpu test suite, smoke, default bench (config 2) and config 3/5 bench lines.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/t_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 5
echo smoke_ok
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 6
cat gpurun_out/bench_default.json
for c in 3 4 5; do
timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || exit 7
python -c "import json;d=json.load(open('gpurun_out/bench_c$c.json'));print('config $c', d['value'], d['roofline']['frac'])"
done
