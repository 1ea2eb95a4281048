#!/bin/bash
# Streaming (per-packet) API: its GPU tests, the per-call latency, then a quick bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-stream}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "stream or dropin or transmit or mid" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python -u tools/stream_latency.py 3000 > $OUT/latency.txt 2>&1 || { echo "latency failed"; tail -20 $OUT/latency.txt; exit 1; }
cat $OUT/latency.txt
timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-host-inclusive --no-extra-configs > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline'],d['kernels_ms_back_to_back'])"
