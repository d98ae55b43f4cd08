export TMPDIR=/tmp
mkdir -p gpurun_out/surv
for e in base 16 4; do
  if [ $e = base ]; then ENV=""; else ENV="DICE_PRUNE_SURVIVORS=$e"; fi
  env $ENV timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/surv/$e -o run --output-format csv -- python bench.py --config 3 --steps 10 --warmup 2 --match-mode top1 --no-cpu-baseline --no-extras --extra-configs= > gpurun_out/surv/$e.json 2> gpurun_out/surv/$e.err || exit 3
done
python - <<'PY'
import csv, glob
for e in ('base', '16', '4'):
    f = glob.glob(f'gpurun_out/surv/{e}/**/run_kernel_stats.csv', recursive=True)
    print(e)
    for r in csv.DictReader(open(f[0])):
        print('  ', r['Name'][:60], r['Calls'], r['AverageNs'])
PY
