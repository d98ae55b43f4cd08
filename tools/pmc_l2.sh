#!/bin/bash
# L2 / L1 request counters for one config (two passes): tools/pmc_l2.sh <tag> <config>
set -u
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${1:-c3l2}
mkdir -p $OUT
B="python bench.py --config ${2:-3} --steps 3 --warmup 1 --no-cpu-baseline --extra-configs="
timeout -s KILL 180 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum -d $OUT/a -o run --output-format csv -- $B > /dev/null 2> $OUT/a.err || exit 31
timeout -s KILL 180 rocprofv3 --pmc TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCC_EA0_RDREQ_sum TCC_REQ_sum -d $OUT/b -o run --output-format csv -- $B > /dev/null 2> $OUT/b.err || exit 32
echo pmc_done
