# round-6 session 3: the walk's second-half adds -- skipped (no2nd, results wrong) and compacted (compact)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
DICE_POST_PRUNE=0 bash tools/gpu_ab.sh 2 "--config 3 --steps 20" base lib:no2nd lib:compact || exit $?
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" base lib:no2nd lib:compact || exit $?
# parity of the compacted walk: its bench lines with the oracle sample, then the postings tests
LICENSEE_DICE_LIB=licensee_amd/lib/var/compact.so DICE_POST_PRUNE=0 timeout -k 10 300 python bench.py --config 3 \
  --steps 5 --warmup 1 --extra-configs= --no-extras > gpurun_out/compact_c3.json 2> gpurun_out/compact_c3.err || exit 4
LICENSEE_DICE_LIB=licensee_amd/lib/var/compact.so timeout -k 10 300 python bench.py --config 5-T600 \
  --steps 5 --warmup 1 --extra-configs= --no-extras > gpurun_out/compact_t600.json 2> gpurun_out/compact_t600.err || exit 5
python -c "
import json
for f in ('gpurun_out/compact_c3.json','gpurun_out/compact_t600.json'):
    d=json.load(open(f)); print(f, d['parity'])"
LICENSEE_DICE_LIB=licensee_amd/lib/var/compact.so timeout -k 10 600 python -u -m pytest tests/test_gpu_corpus_sizes.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -k "post" > gpurun_out/compact_tests.log 2>&1; echo "tests_rc=$?"; tail -3 gpurun_out/compact_tests.log
