export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_slowpath.py tests/test_gpu_prune.py tests/test_gpu_parity.py tests/test_gpu_golden.py "tests/test_gpu_configs.py::test_config3_shard" -x -q --timeout 300 -m gpu > gpurun_out/t_shuf2.log 2>&1 || { echo tests failed; tail -20 gpurun_out/t_shuf2.log; exit 3; }
tail -1 gpurun_out/t_shuf2.log
bash tools/gpu_ab.sh 2 "--config 3 --match-mode top1 --steps 20" base DICE_POST_ROW_SHUFFLE=0
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" base DICE_POST_ROW_SHUFFLE=0
