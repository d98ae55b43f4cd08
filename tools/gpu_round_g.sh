#!/bin/bash
# GPU session: LDS kernel parity + config-3 variants after moving record loads behind the wait.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_golden.py -x -q -m gpu -k "lds or 600 or large" > gpurun_out/t_g.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/t_g.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1 2; do
DICE_LDS_VARIANT=$v timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c3g_v$v.json 2> gpurun_out/c3g_v$v.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/c3g_v$v.json'));print('c3 variant $v', d['value'], d['roofline']['launch_ms'])"
done
