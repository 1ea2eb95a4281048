#!/bin/bash
# Config 4 device work under rocprofv3: kernel-trace summary, then HBM traffic and SQ counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-vr}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/vr_prof.py 10 > $OUT/vr_prof.log 2>&1 || { echo "vr_prof failed"; tail -20 $OUT/vr_prof.log; exit 1; }
cat $OUT/vr_prof.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o vr -- python3 $R/tools/vr_prof.py 20 > $OUT/vr_prof_rp.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/vr_prof_rp.log; exit 1; }
KS=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 $R/tools/kstats.py "$KS" | head -20
PMC_SCRIPT=vr_prof.py bash $R/tools/pmc_diag.sh $TAG "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT" -- > /dev/null || { echo "pmc failed"; exit 1; }
grep -A20 "fec_vr" $OUT/pmc/summary.txt | head -80
