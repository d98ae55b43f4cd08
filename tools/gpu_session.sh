# round-6 session 2: the pruned kernel's phase clocks through both config-3 entry points (one lease),
# then a small A/B of the deferral knobs on dice_match (3-top1)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r6_phases
for mode in top1 confidence; do
  LICENSEE_DICE_LIB=licensee_amd/lib/var/pdiag.so timeout -k 10 300 python bench.py --config 3 --match-mode $mode \
    --steps 10 --warmup 2 --extra-configs= --no-cpu-baseline --no-extras > gpurun_out/r6_phases/$mode.json \
    2> gpurun_out/r6_phases/$mode.err || { echo "phase run $mode failed"; exit 3; }
  grep "prune4 phases" gpurun_out/r6_phases/$mode.err | tail -2
done
bash tools/gpu_ab.sh 2 "--config 3 --match-mode top1 --steps 20" base DICE_PRUNE_MAX_EVALS=5 DICE_PRUNE_MAX_EVALS=12 \
  DICE_PRUNE_ROUTE=8 DICE_PRUNE_ROUTE=24
