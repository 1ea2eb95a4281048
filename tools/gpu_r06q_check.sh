#!/bin/bash
# Decode-planner parity (test_gpu_parity: every decode, loss-count, continuing-decode and stream-group
# case) and the relay suites, then config 3's kernel trace and the adaptive relay's wall time and trace.
#   bash tools/gpu_r06q_check.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06q}
mkdir -p $OUT
cd $R && timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu > $OUT/pytest_parity.log 2>&1 || { tail -30 $OUT/pytest_parity.log; exit 1; }
tail -2 $OUT/pytest_parity.log
cd $R && timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_swdf.py tests/test_sdswdf.py -m gpu > $OUT/pytest_relay.log 2>&1 || { tail -30 $OUT/pytest_relay.log; exit 1; }
tail -2 $OUT/pytest_relay.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3 -o run -- python3 $R/tools/config3_prof.py 20 > $OUT/config3_prof.log 2>&1 || { tail -20 $OUT/config3_prof.log; exit 1; }
python3 $R/tools/kstats.py $(find $OUT/c3 -name '*kernel_stats.csv') > $OUT/config3_stats.txt 2>&1
tail -1 $OUT/config3_prof.log >> $OUT/config3_stats.txt
head -8 $OUT/config3_stats.txt; tail -1 $OUT/config3_stats.txt
timeout -k 10 200 python3 -u $R/tools/relay_vr_prof.py 5 > $OUT/relay_vr_wall.txt 2>&1 || { tail -20 $OUT/relay_vr_wall.txt; exit 1; }
cat $OUT/relay_vr_wall.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rv -o run -- python3 $R/tools/relay_vr_prof.py 3 2 > $OUT/relay_vr_prof.log 2>&1 || { tail -20 $OUT/relay_vr_prof.log; exit 1; }
python3 $R/tools/kstats.py $(find $OUT/rv -name '*kernel_stats.csv') > $OUT/relay_vr_stats.txt 2>&1
head -12 $OUT/relay_vr_stats.txt
cd $R && timeout -k 10 200 python3 -u tools/config3_ab.py FEC_PLAN_GRID=1024 FEC_PLAN_GRID=2048 FEC_PLAN_GRID=4096 FEC_PLAN_GRID=8192 5 > $OUT/config3_ab.txt 2>&1 || { tail -20 $OUT/config3_ab.txt; exit 1; }
cat $OUT/config3_ab.txt
