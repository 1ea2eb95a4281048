#!/bin/bash
# Config 3: recovery placement A/B (12 rounds) and a kernel trace of the default; headline step:
# episode grid A/B.   bash tools/gpu_r06w_check.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06w}
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u tools/config3_ab.py FEC_RECOVER_BESIDE=0 FEC_RECOVER_BESIDE=1 12 > $OUT/config3_ab.txt 2>&1 || { tail -20 $OUT/config3_ab.txt; exit 1; }
cat $OUT/config3_ab.txt
timeout -k 10 300 python3 -u tools/step_ab.py env=FEC_EPISODE_GRID:245 env=FEC_EPISODE_GRID:384 > $OUT/step_ab.txt 2>&1 || { tail -20 $OUT/step_ab.txt; exit 1; }
timeout -k 10 300 python3 -u tools/step_ab.py env=FEC_EPISODE_GRID:384 env=FEC_EPISODE_GRID:245 >> $OUT/step_ab.txt 2>&1 || { tail -20 $OUT/step_ab.txt; exit 1; }
cat $OUT/step_ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3 -o run -- python3 $R/tools/config3_prof.py 20 > $OUT/config3_prof.log 2>&1 || { tail -20 $OUT/config3_prof.log; exit 1; }
python3 $R/tools/kstats.py $(find $OUT/c3 -name '*kernel_stats.csv') > $OUT/config3_stats.txt 2>&1
tail -1 $OUT/config3_prof.log >> $OUT/config3_stats.txt
python3 $R/tools/trace_run.py $(find $OUT/c3 -name '*kernel_trace.csv') fec_copy_pair > $OUT/config3_timeline.txt
cat $OUT/config3_timeline.txt; tail -1 $OUT/config3_stats.txt
