#!/bin/bash
# The words parity tests, then the device wordset scan's upload wall time (tools/words_bench.py) of
# this build against a variant build (tools/build_variant.sh <variant> ...), twice each.
#   bash tools/words_ab.sh [variant]     (default: blocks = -DWORDS_BLOCKS_ONLY=1)
VAR=${1:-blocks}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_words.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_words.log 2>&1; rc=$?; echo words_rc=$rc; tail -3 gpurun_out/t_words.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python tools/words_bench.py 64000 5 > gpurun_out/wb_main_$i.json 2>&1 || exit 3
LICENSEE_DICE_LIB=licensee_amd/lib/var/$VAR.so timeout -k 10 200 python tools/words_bench.py 64000 5 > gpurun_out/wb_${VAR}_$i.json 2>&1 || exit 4
done
echo ab_done
