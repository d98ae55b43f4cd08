set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "--config 2 --steps 100 --warmup 10" "--config 4 --steps 100 --warmup 10" "--config 2 --steps 20 --warmup 2" "--config 4 --steps 20 --warmup 2" "--config 2 --steps 100 --warmup 10"; do
  timeout -k 10 300 python bench.py $a --extra-configs= --no-cpu-baseline > gpurun_out/c24.json 2> gpurun_out/c24.err || exit 10
  python -c "import json,sys; d=json.loads(open('gpurun_out/c24.json').read().strip().splitlines()[-1]); print(sys.argv[1], round(d['roofline']['launch_ms']*1e3,2), 'us', round(d['ms_per_step']*1e3,2))" "$a"
done
