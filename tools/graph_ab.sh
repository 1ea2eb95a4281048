#!/bin/bash
# Bench step: hipGraph replay vs eager launches, 20 and 100 steps, separate processes (one GPU call).
#   gpurun -- bash tools/graph_ab.sh [tag] [extra bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-graph_ab}
shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
B="--no-cpu-baseline --no-host-inclusive --no-extra-configs $*"
i=0
for a in "--graph" "" "--graph" "" "--graph --steps 100" "--steps 100"; do
    i=$((i + 1))
    timeout -k 10 120 python -u $R/bench.py $B $a > $OUT/run$i.json 2> $OUT/run$i.err || { echo "bench failed: $a"; tail -20 $OUT/run$i.err; exit 1; }
    python3 - "$OUT/run$i.json" "$a" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"[{sys.argv[2]:>22}] {d['value']:8.1f} GiB/s  {d['ms_per_step']:.4f} ms  kernels {d['kernels_ms_per_launch']}")
EOF
done
