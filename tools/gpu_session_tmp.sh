export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_confidence.py tests/test_gpu_parity.py tests/test_gpu_corpus_sizes.py "tests/test_gpu_configs.py::test_config3_shard" -x -q --timeout 300 -m gpu > gpurun_out/t_bal.log 2>&1 || { echo tests failed; tail -30 gpurun_out/t_bal.log; exit 3; }
tail -2 gpurun_out/t_bal.log
for v in base nobal; do
  unset LICENSEE_DICE_LIB
  [ $v != base ] && export LICENSEE_DICE_LIB=licensee_amd/lib/var/$v.so
  rm -rf gpurun_out/split_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/split_$v -o run -- python bench.py --config 3 --match-mode top1 --steps 10 --warmup 2 --extra-configs= --no-cpu-baseline --no-extras > gpurun_out/split_$v.json 2> gpurun_out/split_$v.err || { echo "$v failed"; exit 3; }
  echo "== $v"; python tools/rocpd_summary.py gpurun_out/split_$v/run_results.db --match dice_
done
unset LICENSEE_DICE_LIB
bash tools/gpu_ab.sh 3 "--config 3 --match-mode top1 --steps 20" base lib:nobal
