#!/bin/bash
# LDS kernel (config 3): parity of the snake slab order, then interleaved A/B against the
# forward-only order (DICE_LDS_SNAKE=0).
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for sn in 1 0; do
DICE_LDS_SNAKE=$sn timeout -k 10 400 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_corpus_sizes.py -x -q -m gpu -k "600 or lds" --timeout 300 --timeout-method thread > gpurun_out/ab/snake$sn.log 2>&1
rc=$?; echo "snake=$sn pytest_rc=$rc"; tail -1 gpurun_out/ab/snake$sn.log; [ $rc -eq 0 ] || exit $rc
done
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/ab/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag', round(d['value']/1e6,2), 'Mfiles/s', round(d['roofline']['launch_ms'],3), 'ms')"
}
for rep in 1 2 3; do
for sn in 1 0; do run c3snake${sn}_$rep DICE_LDS_SNAKE=$sn; done
done
