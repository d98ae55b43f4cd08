#!/bin/bash
# Parity subset + A/B: epilogues inside the stream vs after it (config 2, interleaved).
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -1 gpurun_out/ab/tests.log; [ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag failed"; tail -3 gpurun_out/ab/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag', round(d['roofline']['launch_ms']*1000,1), 'us')"
}
for rep in 1 2 3; do
run stream_$rep DICE_X=0
run tail_$rep DICE_PROG_EPI=tail
run stream4_$rep DICE_PROG_BURST=4
done
