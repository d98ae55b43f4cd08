#!/bin/bash
# Parity subset + interleaved A/B: non-temporal output stores (default) vs plain stores
# (DICE_PROG_NTSTORE=0), configs 2 and 5.
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -1 gpurun_out/ab/tests.log; [ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag failed"; tail -3 gpurun_out/ab/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag', round(d['roofline']['launch_ms']*1000,1), 'us')"
}
for rep in 1 2 3; do
run c2nt_$rep 2 DICE_X=0
run c2plain_$rep 2 DICE_PROG_NTSTORE=0
run c5nt_$rep 5 DICE_X=0
run c5plain_$rep 5 DICE_PROG_NTSTORE=0
done
