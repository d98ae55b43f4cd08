#!/bin/bash
# Final-state verification: full GPU suite, smoke, default bench, profiles for configs 2-5.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_l.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -1 gpurun_out/t_l.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_l.log 2>&1 || exit 5
echo smoke_ok
timeout -k 10 400 python bench.py > gpurun_out/bench_l.json 2> gpurun_out/bench_l.err || exit 6
cat gpurun_out/bench_l.json
bash tools/profile_round.sh r1g_config2 || exit 7
bash tools/profile_round.sh r1g_config4 --config 4 || exit 8
bash tools/profile_round.sh r1g_config5 --config 5 || exit 9
bash tools/profile_round.sh r1g_config3 --config 3 || exit 11
for c in 3 4 5; do
timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 2 > gpurun_out/bench_l$c.json 2> gpurun_out/bench_l$c.err || exit 10
python -c "import json;d=json.load(open('gpurun_out/bench_l$c.json'));print('c$c', d['value'], round(d['roofline']['launch_ms']*1000,1), d['roofline']['frac'], d['parity'])"
done
