#!/bin/bash
# Streaming API after the completion-word change: GPU tests, C ABI latency (spin vs stream sync), Python latency.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-stream2}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "stream or dropin or transmit or mid" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 60 ./tools/stream_latency 5000 > $OUT/cabi_spin.txt 2>&1 || { echo "latency failed"; cat $OUT/cabi_spin.txt; exit 1; }
FEC_STREAM_SPIN=0 timeout -k 10 60 ./tools/stream_latency 5000 > $OUT/cabi_sync.txt 2>&1 || { echo "latency failed"; cat $OUT/cabi_sync.txt; exit 1; }
timeout -k 10 60 ./tools/stream_latency 5000 >> $OUT/cabi_spin.txt 2>&1 || { echo "latency failed"; exit 1; }
echo "spin: $(cat $OUT/cabi_spin.txt)"; echo "sync: $(cat $OUT/cabi_sync.txt)"
timeout -k 10 120 python -u tools/stream_latency.py 3000 > $OUT/latency_py.txt 2>&1 || { echo "py latency failed"; tail $OUT/latency_py.txt; exit 1; }
cat $OUT/latency_py.txt
