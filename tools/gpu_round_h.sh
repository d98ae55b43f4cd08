#!/bin/bash
# Full GPU suite + smoke + default bench, then the config-3 profile of the default LDS variant.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_h.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -2 gpurun_out/t_h.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_h.log 2>&1 || exit 5
echo smoke_ok
timeout -k 10 400 python bench.py > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err || exit 6
python -c "import json;d=json.load(open('gpurun_out/bench_h.json'));print('c2', d['value'], d['roofline']['frac'], d['parity'])"
bash tools/profile_round.sh r1c_config3 --config 3 || exit 7
timeout -k 10 300 python bench.py --config 3 --steps 10 --warmup 2 > gpurun_out/bench_h3.json 2> gpurun_out/bench_h3.err || exit 8
python -c "import json;d=json.load(open('gpurun_out/bench_h3.json'));print('c3', d['value'], d['roofline']['launch_ms'], d['parity'], d['cpu_baseline']['value'])"
