#!/bin/bash
# A round's final measurement set in one lease (round 4: tag r4r):
#   1. gpu_measure.sh <tag>: the default bench line, the same-lease trace of config 2, and
#      profile_round.sh for configs 2-5 (config 3 through dice_batch_match_confidence);
#   2. profiles of config 3 on the postings kernels (all pairs) and of 5-T600;
#   3. one matrix-core utilisation counter pass on 5-T600 (dice_post_dense_mfma).
# Then: python tools/summarize_session.py <tag>; tools/summarize_profile.py per prof_<tag>_* directory.
set -u
TAG=$1
export TMPDIR=/tmp
bash tools/gpu_measure.sh $TAG && DICE_POST_PRUNE=0 bash tools/profile_round.sh ${TAG}_config3_post --config 3 \
  && bash tools/profile_round.sh ${TAG}_config5_T600 --config 5-T600 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
  SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE -d gpurun_out/prof_${TAG}_mfma -o run --output-format csv -- python bench.py \
  --config 5-T600 --steps 5 --warmup 1 --no-cpu-baseline --no-extras --extra-configs= > gpurun_out/${TAG}_mfma.json \
  2> gpurun_out/${TAG}_mfma.err
echo "final_rc=$?"
