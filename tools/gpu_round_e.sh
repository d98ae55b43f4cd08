#!/bin/bash
# GPU session: full GPU parity suite, config-2 bench (grouped asm blocks), config-3 LDS variants.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t_e.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -4 gpurun_out/t_e.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline > gpurun_out/c2_e$i.json 2> gpurun_out/c2_e$i.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/c2_e$i.json'));print('c2', d['value'], d['roofline']['launch_ms'], d['roofline']['frac'])"
done
for v in 0 1 2 3; do
DICE_LDS_VARIANT=$v timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c3_v$v.json 2> gpurun_out/c3_v$v.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/c3_v$v.json'));print('c3 variant $v', d['value'], d['roofline']['launch_ms'], d['config']['kernel'])"
done
