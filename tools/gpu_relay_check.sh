#!/bin/bash
# One GPU call: relay parity tests, relay timings, rocprofv3 kernel stats of the relay chains.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-relay}
TESTS=${2:-tests/test_swdf.py}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u tools/relay_prof.py 3 > $OUT/relay_prof.txt 2>&1 || { echo relay_prof failed; tail -20 $OUT/relay_prof.txt; exit 1; }
cat $OUT/relay_prof.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o relay -- python3 $R/tools/relay_prof.py 3 > $OUT/relay_prof_rocprof.txt 2>&1 || { echo rocprof failed; tail -20 $OUT/relay_prof_rocprof.txt; exit 1; }
KS=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$KS" | cut -c1-160 | head -12
