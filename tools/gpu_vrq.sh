#!/bin/bash
# Quick: config 4 GPU tests, config 4 device timing (tile path and the generic kernel), VR kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-vrq}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_vr.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python -u tools/vr_prof.py 10 2>&1 | tee $OUT/vr_prof.log
FEC_VR_NO_TILE=1 timeout -k 10 120 python -u tools/vr_prof.py 10 2>&1 | tee $OUT/vr_prof_notile.log
timeout -k 10 200 python -u tools/step_env_ab.py "" "FEC_COPY_THREADS=1" 2>&1 | tee $OUT/copy_threads_ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o vr -- python3 $R/tools/vr_prof.py 20 > $OUT/vr_prof_rp.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/vr_prof_rp.log; exit 1; }
python3 $R/tools/kstats.py $(find $OUT/prof -name "*kernel_stats.csv" | head -1) | head -14
