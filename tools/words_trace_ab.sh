#!/bin/bash
# Kernel-trace A/B of the device wordset scan: this build and a variant (tools/build_variant.sh),
# alternating, rocprofv3 --kernel-trace --stats over tools/words_bench.py each time.
#   bash tools/words_trace_ab.sh <variant> [reps]
VAR=$1; R=${2:-2}
export TMPDIR=/tmp
for i in $(seq 1 $R); do
  for b in main $VAR; do
    if [ $b = main ]; then unset LICENSEE_DICE_LIB; else export LICENSEE_DICE_LIB=licensee_amd/lib/var/$VAR.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/wtab_${b}_$i -o run --output-format csv -- python tools/words_bench.py 64000 5 > /dev/null 2>&1 || exit 1
    python -c "import csv,glob,sys; [print(sys.argv[1], sys.argv[2], round(float(r[3]) / 1e6, 3), 'ms') for r in csv.reader(open(glob.glob(sys.argv[3])[0])) if 'dice_words_kernel' in r[0]]" $b $i "gpurun_out/wtab_${b}_$i/*kernel_stats.csv"
  done
done
