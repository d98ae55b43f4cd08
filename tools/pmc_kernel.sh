#!/bin/bash
# PMC passes (one rocprofv3 run per pass) over a short bench run of one config.
#   tools/pmc_kernel.sh <tag> [bench args...]   -> gpurun_out/pmc_<tag>/p{A,B,C}
set -u
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
B="python bench.py --steps 5 --warmup 1 --no-cpu-baseline --extra-configs= $*"
P[0]="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P[1]="SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
P[2]="SQC_ICACHE_MISSES SQC_ICACHE_HITS GRBM_GUI_ACTIVE"
for i in 0 1 2; do
  timeout -s KILL 120 rocprofv3 --pmc ${P[$i]} -d $OUT/p$i -o run --output-format csv -- $B > /dev/null 2> $OUT/p$i.err || exit $((30 + i))
done
echo pmc_done
