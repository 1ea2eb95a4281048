#!/bin/bash
# Bench step kernel trace (rocprofv3 --kernel-trace --stats) without the extra configs, summarised
# per kernel and per step.   gpurun -- bash tools/gpu_quick_prof.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-qp}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $R/bench.py --no-cpu-baseline --no-host-inclusive --no-extra-configs > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof failed"; tail -30 $OUT/bench_prof.err; exit 1; }
KS=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 $R/tools/kernel_time.py $OUT/kernel_time.json $TAG "$KS" > /dev/null || { echo "kernel_time failed"; exit 1; }
python3 - "$KS" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>6}  {r['Name'][:100]}")
PY
