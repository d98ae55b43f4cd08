#!/bin/bash
# Profile the bench workload on the GPU box (run under gpurun from the repo root).
#   tools/profile_round.sh <tag> [bench args...]
# Separate rocprofv3 passes: kernel trace + stats, FETCH_SIZE, WRITE_SIZE, SQ issue counters.
set -u
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --extra-configs= $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.json 2>$OUT/trace.err || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.json 2>$OUT/fetch.err || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.json 2>$OUT/write.err || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d $OUT/sq -o run --output-format csv -- $B > $OUT/sq.json 2>$OUT/sq.err || exit 4
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $OUT/clk -o run --output-format csv -- $B > $OUT/clk.json 2>$OUT/clk.err || exit 5
echo profile_done
