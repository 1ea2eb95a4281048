#!/bin/bash
# One GPU call: kernel-trace of the bench step and its per-step timeline (gaps between kernels).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-tl}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o bench -- python3 $R/bench.py --no-cpu-baseline --no-host-inclusive --no-extra-configs --warm-seconds 0.3 > $OUT/bench.json 2> $OUT/bench.err || { echo "rocprof failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
KT=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_timeline.py "$KT" | tee $OUT/timeline.txt
