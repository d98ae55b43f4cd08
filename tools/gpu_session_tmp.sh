export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_confidence.py tests/test_gpu_api.py tests/test_gpu_sharded.py -x -q --timeout 300 -m gpu > gpurun_out/t_route.log 2>&1 || { echo tests failed; tail -30 gpurun_out/t_route.log; exit 3; }
tail -2 gpurun_out/t_route.log
timeout -k 10 400 python tools/exp/prune_long_files.py 250000 > gpurun_out/long_route.txt 2>&1 || { echo failed; tail -5 gpurun_out/long_route.txt; exit 3; }
grep profile gpurun_out/long_route.txt
bash tools/gpu_ab.sh 3 "--config 3 --match-mode top1 --steps 20" base DICE_PRUNE_LONG_ROUTE=0
