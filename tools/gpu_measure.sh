#!/bin/bash
# One GPU session = one self-consistent measurement set (tag e.g. r2a):
#   1. the driver's default bench line (config 2 + extras.configs 3/4/5, CPU baseline, parity);
#   2. rocprofv3 --kernel-trace --stats of the SAME primary workload and step count
#      (bench.py --extra-configs= --no-cpu-baseline), so profiles/<tag>_config2 kernel averages
#      and the bench line's launch_ms come from one lease;
#   3. tools/profile_round.sh (trace + PMC passes) for the configs given (default "2 3 4 5";
#      split them over calls to stay inside one call's time limit).
# Then `python tools/summarize_session.py <tag>` here turns gpurun_out/ into profiles/.
set -u
TAG=$1
CONFIGS=${2:-2 3 4 5}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 11
cat gpurun_out/${TAG}_bench.json
OUT=gpurun_out/prof_${TAG}_same
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --extra-configs= --no-cpu-baseline --no-extras > $OUT/bench.json 2> $OUT/bench.err || exit 12
echo same_session_trace_done
for c in $CONFIGS; do
  bash tools/profile_round.sh ${TAG}_config$c --config $c || exit $((20 + c))
done
echo measure_done
