#!/bin/bash
# PMC passes over the config-3 LDS kernel (diagnostic; each pass its own rocprofv3 run).
export TMPDIR=/tmp
OUT=gpurun_out/prof_lds
mkdir -p $OUT
B="python bench.py --config 3 --steps 3 --warmup 1 --files-per-gpu 250000 --no-cpu-baseline"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.json 2>$OUT/trace.err || exit 1
echo trace_ok
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d $OUT/a -o run --output-format csv -- $B > $OUT/a.json 2>$OUT/a.err || exit 2
echo a_ok
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES -d $OUT/b -o run --output-format csv -- $B > $OUT/b.json 2>$OUT/b.err || exit 3
echo b_ok
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/c -o run --output-format csv -- $B > $OUT/c.json 2>$OUT/c.err || exit 4
echo c_ok
