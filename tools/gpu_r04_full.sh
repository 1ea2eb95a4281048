#!/bin/bash
# Round-4 check: the whole -m gpu suite, smoke(), the per-packet latency probe, config 4's unit sweep
# + kernel trace, one bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
g++ -O2 -std=c++17 -I include tools/stream_latency.cpp -L fec_erasure_code_unit_test_relay_amd -lfec_amd -Wl,-rpath,$R/fec_erasure_code_unit_test_relay_amd -o /tmp/stream_latency || exit 1
timeout -k 10 120 /tmp/stream_latency 20000 > $OUT/stream_latency.txt 2>&1 || { cat $OUT/stream_latency.txt; exit 1; }
tail -12 $OUT/stream_latency.txt
bash tools/gpu_vr_unit.sh $TAG/vr || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("bench", d["value"], "GiB/s", d["ms_per_step"], "ms", d["kernels_ms_per_launch"])
for k, v in d.get("configs", {}).items():
    print(k, {kk: v[kk] for kk in v if kk in ("value", "ms_per_step", "device_only_ms", "verified", "host_plan_ms")})
PY
