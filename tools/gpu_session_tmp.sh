export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_slowpath.py tests/test_gpu_prune.py tests/test_gpu_parity.py tests/test_gpu_confidence.py "tests/test_gpu_configs.py::test_config3_shard" -x -q --timeout 300 -m gpu > gpurun_out/t_u8.log 2>&1 || { echo tests failed; tail -30 gpurun_out/t_u8.log; exit 3; }
tail -2 gpurun_out/t_u8.log
for v in base u16; do
  unset DICE_POST_U8
  [ $v = u16 ] && export DICE_POST_U8=0
  for cfg in 5-T600 3; do
    extra=""; [ $cfg = 3 ] && extra="DICE_POST_PRUNE=0"
    rm -rf gpurun_out/u8_${v}_$cfg
    env $extra timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/u8_${v}_$cfg -o run -- python bench.py --config $cfg --steps 10 --warmup 2 --extra-configs= --no-cpu-baseline --no-extras > gpurun_out/u8_${v}_$cfg.json 2> gpurun_out/u8_${v}_$cfg.err || { echo "$v $cfg failed"; exit 3; }
    echo "== $v $cfg"; python tools/rocpd_summary.py gpurun_out/u8_${v}_$cfg/run_results.db --match dice_post
  done
done
unset DICE_POST_U8
bash tools/gpu_ab.sh 3 "--config 5-T600 --steps 10" base DICE_POST_U8=0
bash tools/gpu_ab.sh 3 "--config 3 --steps 10" DICE_POST_PRUNE=0 DICE_POST_PRUNE=0,DICE_POST_U8=0 lib:head,DICE_POST_PRUNE=0
