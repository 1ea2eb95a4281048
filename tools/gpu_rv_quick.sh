#!/bin/bash
# The adaptive relay's parity (types 2, 3 on the golden schedule) and wall time, with a kernel trace
#   bash tools/gpu_rv_quick.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-rvq}
mkdir -p $OUT
cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sdswdf.py -m gpu -k "full_schedule or vr" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python3 -u tools/relay_vr_prof.py 10 2 > $OUT/wall.txt 2>&1 || { tail -20 $OUT/wall.txt; exit 1; }
cat $OUT/wall.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rv -o run -- python3 $R/tools/relay_vr_prof.py 3 2 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 $R/tools/kstats.py $(find $OUT/rv -name '*kernel_stats.csv') > $OUT/stats.txt 2>&1
head -6 $OUT/stats.txt
