#!/bin/bash
# Full GPU suite; A/B around the new defaults; profiles for configs 2, 4, 5; default bench; config-4 bench.
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_j.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -1 gpurun_out/t_j.log; [ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag', round(d['roofline']['launch_ms']*1000,1), 'us')"
}
for rep in 1 2 3; do
run b4a4_$rep DICE_X=0
run b5a4_$rep DICE_PROG_BURST=5
run b4a2_$rep DICE_PROG_ACC_BLOCK=2
run b6a4_$rep DICE_PROG_BURST=6
done
bash tools/profile_round.sh r1e_config2 || exit 7
bash tools/profile_round.sh r1e_config4 --config 4 || exit 8
bash tools/profile_round.sh r1e_config5 --config 5 || exit 9
timeout -k 10 400 python bench.py > gpurun_out/bench_j.json 2> gpurun_out/bench_j.err || exit 10
cat gpurun_out/bench_j.json
timeout -k 10 400 python bench.py --config 4 --steps 50 > gpurun_out/bench_j4.json 2> gpurun_out/bench_j4.err || exit 11
python -c "import json;d=json.load(open('gpurun_out/bench_j4.json'));print('c4', d['value'], d['roofline']['frac'], d['parity'], d['extras'].get('host_prep_native_files_per_s'))"
