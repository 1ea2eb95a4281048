#!/bin/bash
# Per-packet servers: the per-packet API tests, then the C latency probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-srv}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "streaming_api or dropin" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
g++ -O2 -std=c++17 -I include tools/stream_latency.cpp -L fec_erasure_code_unit_test_relay_amd -lfec_amd -Wl,-rpath,$R/fec_erasure_code_unit_test_relay_amd -o /tmp/stream_latency || exit 1
timeout -k 10 120 /tmp/stream_latency 20000 2>&1 | tee $OUT/stream_latency.txt
timeout -k 10 120 /tmp/stream_latency 20000 2>&1 | tee -a $OUT/stream_latency.txt
