#!/bin/bash
# GPU tests of the encode paths, then bench + kernel trace for the stream and wave encoders.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ab}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "encode" > $OUT/pytest_enc.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $OUT/pytest_enc.log | head -30; tail -5 $OUT/pytest_enc.log; exit 1; }
tail -2 $OUT/pytest_enc.log
for p in stream wave; do
  timeout -k 10 200 python -u bench.py --encode-path $p --no-cpu-baseline --no-host-inclusive > $OUT/bench_$p.json 2> $OUT/bench_$p.err || { echo "bench $p failed"; tail -20 $OUT/bench_$p.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$p.json')); print('$p', d['value'], d['kernels_ms_per_launch'])"
done
