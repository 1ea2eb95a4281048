#!/bin/bash
# Default bench.py run (all legs) plus the config-4 VR tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-bf}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 - <<PY
import json
d = json.loads(open("$OUT/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d.get("kernels_ms_per_launch"))
print("host_inclusive", json.dumps(d.get("host_inclusive")))
ex = d.get("extra_configs", {})
print("config4", json.dumps(ex.get("config4_adaptive")))
print("cpu_baseline", json.dumps(d.get("cpu_baseline")))
PY
