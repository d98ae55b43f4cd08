#!/bin/bash
# Config-3 (LDS kernel) knob A/B: parity of both settings, then 3 interleaved bench reps.
# usage: bash tools/gpu_ab_env.sh "VAR=a [VAR2=b]" "VAR=c"   (quoted env assignments per arm)
export TMPDIR=/tmp
A=$1; B=$2
mkdir -p gpurun_out/ab
i=0
for arm in "$A" "$B"; do
i=$((i+1))
env $arm timeout -k 10 400 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_corpus_sizes.py -x -q -m gpu -k "600 or lds" --timeout 300 --timeout-method thread > gpurun_out/ab/arm$i.log 2>&1
rc=$?; echo "[$arm] pytest_rc=$rc"; tail -1 gpurun_out/ab/arm$i.log; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2 3; do
i=0
for arm in "$A" "$B"; do
  i=$((i+1)); tag=c3_arm${i}_$rep
  env $arm timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/ab/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('[$arm] $rep', round(d['value']/1e6,2), 'Mfiles/s', round(d['roofline']['launch_ms'],3), 'ms')"
done
done
