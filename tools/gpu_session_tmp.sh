export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh > gpurun_out/final_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/final_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh 2 "--config 3 --match-mode top1 --steps 20" base DICE_PRUNE_MAX_EVALS=4 DICE_PRUNE_MAX_EVALS=6 DICE_PRUNE_MAX_EVALS=12 DICE_PRUNE_ROUTE=10 DICE_PRUNE_ROUTE=24
