export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_corpus_sizes.py -k "variants" -x -q --timeout 300 -m gpu > gpurun_out/t_var.log 2>&1; echo variants=$?; tail -3 gpurun_out/t_var.log
DICE_PROG_QUEUE=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 -m gpu > gpurun_out/t_q8.log 2>&1; echo q8_parity=$?; tail -2 gpurun_out/t_q8.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_confidence.py::test_scored_pairs_counted_on_device tests/test_bench_launch.py -x -v --timeout 300 -m gpu > gpurun_out/t_new2.log 2>&1; echo new2=$?; tail -5 gpurun_out/t_new2.log
bash tools/gpu_ab.sh 2 "--config 3 --steps 10" DICE_POST_PRUNE=0 DICE_POST_PRUNE=0,DICE_POST_MFMA=4 DICE_POST_PRUNE=0,DICE_POST_MFMA=4,DICE_POST_MFMA_MT=2
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" base DICE_POST_MFMA=4
bash tools/gpu_ab.sh 3 "--config 2 --steps 50" base DICE_PROG_QUEUE=8 DICE_PROG_QUEUE=1
