#!/bin/bash
# Bench line vs the untimed device warm-up (--warm-seconds), separate processes (one GPU call).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-warm_ab}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
B="--no-cpu-baseline --no-host-inclusive --no-extra-configs"
i=0
for a in "--warm-seconds 0" "--warm-seconds 0.3" "--warm-seconds 1" "--warm-seconds 3" "--warm-seconds 1 --steps 100" "--warm-seconds 0"; do
    i=$((i + 1))
    timeout -k 10 120 python -u $R/bench.py $B $a > $OUT/run$i.json 2> $OUT/run$i.err || { echo "bench failed: $a"; tail -20 $OUT/run$i.err; exit 1; }
    python3 - "$OUT/run$i.json" "$a" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"[{sys.argv[2]:>26}] {d['value']:8.1f} GiB/s  {d['ms_per_step']:.4f} ms  warm {d['device_warmup']['untimed_steps']}  kernels {d['kernels_ms_per_launch']}")
PY
done
