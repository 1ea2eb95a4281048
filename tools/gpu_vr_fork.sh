#!/bin/bash
# Config 4 device work: VR GPU tests, timing and a kernel trace (side-stream launches).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-vrf}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_vr.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python -u tools/vr_prof.py 10 2>&1 | tee $OUT/vr_prof.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/vr_prof.py 20 > $OUT/rocprof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/rocprof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp "$f" $OUT/kernel_stats.csv
cut -d, -f1-4 $OUT/kernel_stats.csv | head -14
