#!/bin/bash
# After an encoder change: the whole GPU suite, the encoder alone (L = 300 and 296), LDS counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-enc_check}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 120 python -u tools/enc_time.py --reps 7 > $OUT/enc300_$i.txt 2>&1 || { echo "enc_time failed"; tail $OUT/enc300_$i.txt; exit 1; }
  grep us/launch $OUT/enc300_$i.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc -o pmc -- python3 $R/tools/enc_time.py --iters 3 --reps 1 > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/pmc.log; exit 1; }
python3 $R/tools/pmc_summary.py $(find $OUT/pmc -name '*counter_collection.csv') | grep -A6 encode_tile
