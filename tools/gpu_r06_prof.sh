#!/bin/bash
# Round-6 profiles: the adaptive relay (fec_relay_vr) per run and its kernel trace, config 3's decode
# launch chain.   bash tools/gpu_r06_prof.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06_prof}
mkdir -p $OUT
cd $R && timeout -k 10 200 python3 -u tools/relay_vr_prof.py 5 > $OUT/relay_vr_wall.txt 2>&1 || { tail -20 $OUT/relay_vr_wall.txt; exit 1; }
cat $OUT/relay_vr_wall.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/relay_vr -o run -- python3 $R/tools/relay_vr_prof.py 3 2 > $OUT/relay_vr_prof.log 2>&1 || { tail -20 $OUT/relay_vr_prof.log; exit 1; }
python3 $R/tools/kstats.py $(find $OUT/relay_vr -name '*kernel_stats.csv') > $OUT/relay_vr_stats.txt 2>&1
head -14 $OUT/relay_vr_stats.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/config3 -o run -- python3 $R/tools/config3_prof.py 20 > $OUT/config3_prof.log 2>&1 || { tail -20 $OUT/config3_prof.log; exit 1; }
grep "config 3" $OUT/config3_prof.log
python3 $R/tools/kstats.py $(find $OUT/config3 -name '*kernel_stats.csv') > $OUT/config3_stats.txt 2>&1
head -14 $OUT/config3_stats.txt
