#!/bin/bash
# Profile the device wordset scan (tools/words_bench.py) on the GPU box: kernel trace + stats, then
# separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ issue counters), as tools/profile_round.sh does.
#   bash tools/profile_words.sh <tag> [n_texts]
set -u
TAG=$1; N=${2:-64000}
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}_words
mkdir -p $OUT
B="python tools/words_bench.py $N 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.json 2>$OUT/trace.err || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.json 2>$OUT/fetch.err || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.json 2>$OUT/write.err || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d $OUT/sq -o run --output-format csv -- $B > $OUT/sq.json 2>$OUT/sq.err || exit 4
echo words_profile_done
