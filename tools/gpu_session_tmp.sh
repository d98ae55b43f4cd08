export TMPDIR=/tmp
mkdir -p gpurun_out
for e in "DICE_PRUNE_ROUTE_AT=1,DICE_PRUNE_ROUTE=48" "DICE_PRUNE_ROUTE_AT=1,DICE_PRUNE_ROUTE=128" "DICE_PRUNE_ROUTE_AT=1,DICE_PRUNE_ROUTE=300" "DICE_PRUNE_ROUTE=48"; do
  echo "== $e"
  env $(echo $e | tr ',' ' ') timeout -k 10 400 python tools/exp/prune_long_files.py 250000 > gpurun_out/long_$e.txt 2>&1 || { echo failed; tail -5 gpurun_out/long_$e.txt; exit 3; }
  grep "kernel pruned:" gpurun_out/long_$e.txt
done
