#!/bin/bash
# Round 3: top-k rescan spread over the lanes (matrix mode) -- matrix/top-k parity tests, then
# the config 5-T600 A/B against the previous build (licensee_amd/lib/var/base0.so).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py \
  tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_corpus_sizes.py > gpurun_out/r3o_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3o_tests.log; [ $rc -eq 0 ] || exit 2
bash tools/gpu_matrix_ab.sh 2 base0 base
