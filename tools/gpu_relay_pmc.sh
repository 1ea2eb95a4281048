#!/bin/bash
# Type-2 relay / destination kernels: SQ and LDS counters (two passes) over tools/swdf_bench.py.
#   bash tools/gpu_relay_pmc.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-relay_pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o pmc -- python3 $R/tools/swdf_bench.py 2 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $(find $OUT -name '*counter_collection.csv') > $OUT/summary.txt
grep -A20 "fast_relay" $OUT/summary.txt | head -40
