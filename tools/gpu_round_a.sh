#!/bin/bash
# GPU session: new parity tests, single-rank distributed bench, non-temporal A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_golden.py -x -q -m gpu > gpurun_out/t1.log 2>&1
echo "pytest_rc=$?"; tail -5 gpurun_out/t1.log
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 timeout -k 10 200 python -X faulthandler bench.py --no-cpu-baseline --steps 5 > gpurun_out/bm.json 2> gpurun_out/bm.err
rc=$?; echo "manual_dist_rc=$rc"; tail -5 gpurun_out/bm.err; cut -c1-200 gpurun_out/bm.json
case $rc in 124|134|137|139) exit $rc;; esac
for nt in 0 1 0 1; do
  DICE_PROG_NT=$nt timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 > gpurun_out/nt$nt.json 2> gpurun_out/nt$nt.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/nt$nt.json'));print('nt=$nt', d['value'], d['roofline']['launch_ms'], d['roofline']['frac'])"
done
