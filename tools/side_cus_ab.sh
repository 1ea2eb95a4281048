#!/bin/bash
# Bench step with the planner's side stream on a CU subset (FEC_SIDE_CUS) vs all CUs, alternating
# processes on one box.   bash tools/side_cus_ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-side_ab}
mkdir -p $OUT
B="--no-cpu-baseline --no-host-inclusive --no-extra-configs --steps 50"
i=0
for e in "" "FEC_SIDE_CUS=32" "FEC_SIDE_CUS=64" "" "FEC_SIDE_CUS=32" "FEC_SIDE_CUS=64"; do
    i=$((i + 1))
    env $e timeout -k 10 120 python -u $R/bench.py $B > $OUT/run$i.json 2> $OUT/run$i.err || { echo "bench failed: $e"; tail -20 $OUT/run$i.err; exit 1; }
    python3 - "$OUT/run$i.json" "$e" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"[{sys.argv[2]:>18}] {d['value']:8.1f} GiB/s  {d['ms_per_step']:.4f} ms  kernels {d['kernels_ms_per_launch']}")
PY
done
