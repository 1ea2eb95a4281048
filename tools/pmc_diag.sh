#!/bin/bash
# Diagnostic PMC passes (one rocprofv3 run per counter group) over tools/profile_step.py.
#   bash tools/pmc_diag.sh TAG "GROUP1" "GROUP2" ... -- profile_step args
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
GROUPS_=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do GROUPS_+=("$1"); shift; done
[ "$1" == "--" ] && shift
OUT=$R/gpurun_out/$TAG/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for C in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o pmc -- python3 $R/tools/${PMC_SCRIPT:-profile_step.py} --iters 3 "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $(find $OUT -name '*counter_collection.csv') > $OUT/summary.txt
cat $OUT/summary.txt
