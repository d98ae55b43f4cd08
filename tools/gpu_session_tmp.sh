export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base nodiv noscorestore; do
  unset LICENSEE_DICE_LIB
  [ $v != base ] && export LICENSEE_DICE_LIB=licensee_amd/lib/var/$v.so
  for cfg in 5-T600; do
    rm -rf gpurun_out/diag_${v}_$cfg
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/diag_${v}_$cfg -o run -- python bench.py --config $cfg --steps 10 --warmup 2 --extra-configs= --no-cpu-baseline --no-extras > gpurun_out/diag_${v}_$cfg.json 2> gpurun_out/diag_${v}_$cfg.err || { echo "$v $cfg failed"; exit 3; }
    echo "== $v $cfg"; python tools/rocpd_summary.py gpurun_out/diag_${v}_$cfg/run_results.db --match narrow
  done
done
