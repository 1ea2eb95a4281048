#!/bin/bash
# One GPU call: parity tests, bench line, rocprofv3 kernel-trace summary of the same bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $R/bench.py --no-cpu-baseline --no-host-inclusive --no-extra-configs > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof failed"; tail -30 $OUT/bench_prof.err; exit 1; }
find $OUT/prof -name "*stats*"
KS=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 $R/tools/kernel_time.py $OUT/kernel_time.json $TAG "$KS" > /dev/null || { echo "kernel_time failed"; exit 1; }
# HBM traffic of the step's kernels (FETCH_SIZE / WRITE_SIZE passes) -> profiles-ready JSON
bash $R/tools/pmc_traffic.sh $TAG > /dev/null 2>&1 || { echo "pmc passes failed"; exit 1; }
python3 $R/tools/pmc_traffic.py $OUT/traffic.json $TAG $OUT/pmc/p1 $OUT/pmc/p2
