# round-4 session r: the final measurement set -- default bench line + same-lease trace of
# config 2 (gpu_measure.sh with no per-config profiles), profiles of config 3 on the postings
# kernels (all pairs) and of 5-T600, and one MFMA-utilisation counter pass on 5-T600
export TMPDIR=/tmp
bash tools/gpu_measure.sh r4r "" && DICE_POST_PRUNE=0 bash tools/profile_round.sh r4r_config3_post --config 3 && bash tools/profile_round.sh r4r_config5_T600 --config 5-T600 && timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE -d gpurun_out/prof_r4r_mfma -o run --output-format csv -- python bench.py --config 5-T600 --steps 5 --warmup 1 --no-cpu-baseline --no-extras --extra-configs= > gpurun_out/r4r_mfma.json 2> gpurun_out/r4r_mfma.err
echo "rc=$?"
