#!/bin/bash
# GPU session: LDS-tiled kernel parity (corpus sizes, T=600) then config-3 bench A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_golden.py -x -q -m gpu > gpurun_out/t_c.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -15 gpurun_out/t_c.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c3_lds.json 2> gpurun_out/c3_lds.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/c3_lds.json'));print('lds', d['value'], d['roofline']['launch_ms'], d['config']['kernel'])"
DICE_FORCE_DENSE=1 timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c3_dense.json 2> gpurun_out/c3_dense.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/c3_dense.json'));print('dense', d['value'], d['roofline']['launch_ms'], d['config']['kernel'])"
