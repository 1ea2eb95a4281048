#!/bin/bash
# Quick GPU iteration: selected parity tests, one bench line, rocprofv3 kernel stats of the step.
#   bash tools/gpu_quick.sh TAG "pytest -k expression" [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
K=$2
shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $R/bench.py --no-cpu-baseline --no-host-inclusive --no-extra-configs "$@" > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof failed"; tail -30 $OUT/bench_prof.err; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fec" in r["Name"]:
            print(r["Name"][:58].ljust(58), r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
