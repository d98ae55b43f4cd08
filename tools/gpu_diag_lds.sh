#!/bin/bash
# Config-3 LDS kernel: product build vs a diagnostic build (licensee_amd/lib/diag/, built with
# -DDICE_LDS_DIAG_NORING: one record-ring read per template run, results intentionally wrong),
# 3 interleaved reps. Bounds what cheaper record reads could gain.
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
L=licensee_amd/lib
cp $L/liblicensee_dice.so /tmp/prod.so
for rep in 1 2 3; do
for v in prod diag; do
  if [ $v = diag ]; then cp $L/diag/liblicensee_dice.so $L/liblicensee_dice.so; else cp /tmp/prod.so $L/liblicensee_dice.so; fi
  tag=c3_${v}_$rep
  timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/ab/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$v $rep', round(d['value']/1e6,2), 'Mfiles/s', round(d['roofline']['launch_ms'],3), 'ms')"
done
done
cp /tmp/prod.so $L/liblicensee_dice.so
