#!/bin/bash
# Full GPU suite, bench x3 (config 2), config-2 and config-5 profiles.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_i.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -2 gpurun_out/t_i.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_i$r.json 2> gpurun_out/bench_i$r.err || exit 6
python -c "import json;d=json.load(open('gpurun_out/bench_i$r.json'));print('c2', d['value'], round(d['roofline']['launch_ms']*1000,1), d['roofline']['frac'], d['config']['program_entries'])"
done
bash tools/profile_round.sh r1d_config2 || exit 7
bash tools/profile_round.sh r1d_config5 --config 5 || exit 8
timeout -k 10 400 python bench.py > gpurun_out/bench_i.json 2> gpurun_out/bench_i.err || exit 9
cat gpurun_out/bench_i.json
