#!/bin/bash
# GPU session: config-2 A/B over asm block sizes; config-3 LDS kernel SQ/LDS counters.
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_c3f
for rep in 1 2; do
for b in 1 4 8 16; do
DICE_PROG_ACC_BLOCK=$b timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline > gpurun_out/c2_b$b.json 2> gpurun_out/c2_b$b.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/c2_b$b.json'));print('c2 block $b', d['value'], d['roofline']['launch_ms'], round(d['roofline']['frac'],4))"
done
done
B="python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/prof_c3f/sq -o run --output-format csv -- $B > gpurun_out/prof_c3f/sq.json 2> gpurun_out/prof_c3f/sq.err || exit 2
timeout -k 10 300 rocprofv3 --pmc SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/prof_c3f/sqc -o run --output-format csv -- $B > gpurun_out/prof_c3f/sqc.json 2> gpurun_out/prof_c3f/sqc.err || echo sqc_failed
timeout -k 10 300 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH -d gpurun_out/prof_c3f/lds -o run --output-format csv -- $B > gpurun_out/prof_c3f/lds.json 2> gpurun_out/prof_c3f/lds.err || echo lds_failed
echo done
