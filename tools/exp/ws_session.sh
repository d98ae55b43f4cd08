#!/bin/bash
# Round 6: walk/store wave split of the matrix kernel -- parity on the matrix tests, then an
# interleaved A/B of 5-T600 over the splits (DICE_POST_WS=0 is the uniform kernel).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_slowpath.py -m gpu -x -q \
  -k "post" --timeout 200 --timeout-method thread > gpurun_out/ws_t1.log 2>&1
rc=$?; echo "t1_rc=$rc"; tail -3 gpurun_out/ws_t1.log; [ $rc -eq 0 ] || exit $rc
for v in 8x8 6x6 4x4; do
  DICE_POST_WS=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_corpus_sizes.py -m gpu -x -q \
    -k "post and (600 or 700 or 130)" --timeout 200 --timeout-method thread > gpurun_out/ws_t_$v.log 2>&1
  rc=$?; echo "t_${v}_rc=$rc"; tail -1 gpurun_out/ws_t_$v.log; [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" DICE_POST_WS=0 DICE_POST_WS=8x4 DICE_POST_WS=8x8 DICE_POST_WS=6x6 DICE_POST_WS=4x4 \
  lib:noscore,DICE_POST_WS=0 lib:noscore,DICE_POST_WS=8x8 lib:noscore,DICE_POST_WS=8x4
