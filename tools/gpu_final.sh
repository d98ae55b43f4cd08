#!/bin/bash
# A round's final measurement set, over two leases (each call stays inside gpurun's 20-minute limit):
#   bash tools/gpu_final.sh <tag> a   -- the GPU suite + smoke (gpu_tests.sh), the default bench line,
#                                        the same-lease trace of config 2, profiles of configs 2 and 3
#                                        (config 3 through dice_batch_match_confidence)  [gpu_measure.sh]
#   bash tools/gpu_final.sh <tag> b   -- profiles of configs 4, 5, 3-top1 (dice_batch_match), 3 on the
#                                        postings kernels (all pairs) and 5-T600, and one matrix-core
#                                        counter pass on 5-T600 (dice_post_dense_mfma)
# Then: python tools/summarize_session.py <tag>; tools/summarize_profile.py per prof_<tag>_* directory.
set -u
TAG=$1
PART=${2:-a}
export TMPDIR=/tmp
if [ "$PART" = a ]; then
  bash tools/gpu_tests.sh && bash tools/gpu_measure.sh $TAG "2 3"
  exit $?
fi
bash tools/profile_round.sh ${TAG}_config4 --config 4 && bash tools/profile_round.sh ${TAG}_config5 --config 5 \
  && bash tools/profile_round.sh ${TAG}_config3_top1 --config 3 --match-mode top1 \
  && DICE_POST_PRUNE=0 bash tools/profile_round.sh ${TAG}_config3_post --config 3 \
  && bash tools/profile_round.sh ${TAG}_config5_T600 --config 5-T600 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
  SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE -d gpurun_out/prof_${TAG}_mfma -o run --output-format csv -- python bench.py \
  --config 5-T600 --steps 5 --warmup 1 --no-cpu-baseline --no-extras --extra-configs= > gpurun_out/${TAG}_mfma.json \
  2> gpurun_out/${TAG}_mfma.err
echo "final_rc=$?"
