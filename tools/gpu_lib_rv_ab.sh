#!/bin/bash
# The adaptive relay's wall time per run (tools/relay_vr_prof.py, type 2) of two library builds on one
# box, in alternating processes (FEC_AMD_LIB selects the library).   bash tools/gpu_lib_rv_ab.sh TAG LIB_A LIB_B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-librv}
mkdir -p $OUT
cd $R
for i in 1 2 3; do
  for L in $2 $3; do
    FEC_AMD_LIB=$R/$L timeout -k 10 200 python3 -u tools/relay_vr_prof.py 10 2 > $OUT/run.txt 2>&1 || { tail -20 $OUT/run.txt; exit 1; }
    echo "$L $(grep 'type 2' $OUT/run.txt)" | tee -a $OUT/ab.txt
  done
done
