#!/bin/bash
# Bench step with and without --pipeline (batch i's recovery beside batch i+1's encode), alternating
# processes on one box.   gpurun -- bash tools/pipeline_ab.sh [tag]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pipeline_ab}
mkdir -p $OUT
cd $R
i=0
for a in "" "--pipeline" "" "--pipeline" "" "--pipeline"; do
    i=$((i + 1))
    timeout -k 10 200 python -u bench.py --no-extra-configs --no-cpu-baseline --no-host-inclusive $a > $OUT/run$i.json 2> $OUT/run$i.err || { echo "bench failed: $a"; tail -20 $OUT/run$i.err; exit 1; }
    python3 - "$OUT/run$i.json" "$a" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"[{sys.argv[2]:>10}] {d['value']:8.1f} GiB/s  {d['ms_per_step']:.4f} ms  verified {d['verified']}  {d['kernels_ms_per_launch']}")
PY
done
