#!/bin/bash
# One GPU call: relay parity tests + stamps, and the queue-priority ubench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05x}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 120 ./tools/ubench/queue_prio > $OUT/queue_prio.txt 2>&1 || { echo "queue_prio failed"; tail -20 $OUT/queue_prio.txt; exit 1; }
cat $OUT/queue_prio.txt
bash tools/swdf_stamps.sh $TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "config5" > $OUT/pytest_config5.log 2>&1 || { echo "config5 test failed"; tail -30 $OUT/pytest_config5.log; exit 1; }
tail -3 $OUT/pytest_config5.log
