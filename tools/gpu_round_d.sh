#!/bin/bash
# GPU session: counter inventory + config-3 profiles of the LDS kernel.
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_c3
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
B="python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3/trace -o run --output-format csv -- $B > gpurun_out/prof_c3/trace.json 2> gpurun_out/prof_c3/trace.err || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/prof_c3/sq -o run --output-format csv -- $B > gpurun_out/prof_c3/sq.json 2> gpurun_out/prof_c3/sq.err || exit 2
timeout -k 10 300 rocprofv3 --pmc SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/prof_c3/sqc -o run --output-format csv -- $B > gpurun_out/prof_c3/sqc.json 2> gpurun_out/prof_c3/sqc.err || echo sqc_failed
echo done
