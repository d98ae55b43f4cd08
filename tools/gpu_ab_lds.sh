#!/bin/bash
# LDS kernel (config 3): parity at each templates-per-wave setting (DICE_LDS_G) + interleaved A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for g in 12 24; do
DICE_LDS_G=$g timeout -k 10 400 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_corpus_sizes.py -x -q -m gpu -k "600 or lds" --timeout 300 --timeout-method thread > gpurun_out/ab/lds_g$g.log 2>&1
rc=$?; echo "G=$g pytest_rc=$rc"; tail -1 gpurun_out/ab/lds_g$g.log; [ $rc -eq 0 ] || exit $rc
done
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/ab/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag', round(d['value']/1e6,1), 'Mfiles/s', round(d['roofline']['launch_ms'],3), 'ms')"
}
for rep in 1 2; do
for g in 16 24 12; do run c3g${g}_$rep DICE_LDS_G=$g; done
done
