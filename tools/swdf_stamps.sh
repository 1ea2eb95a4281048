#!/bin/bash
# Phase breakdown of the tiled type-2 relay / destination kernels (FEC_SWDF_STAMPS diagnostics).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-stamps}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_swdf.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python -u tools/relay_prof.py 3 > $OUT/relay_prof.txt 2>&1 || { echo relay_prof failed; tail -20 $OUT/relay_prof.txt; exit 1; }
head -3 $OUT/relay_prof.txt
FEC_SWDF_STAMPS=1 timeout -k 10 200 python -u tools/relay_prof.py 1 > $OUT/stamps.txt 2>&1 || { echo stamps failed; tail -20 $OUT/stamps.txt; exit 1; }
grep -E "STAMPS|type 2" $OUT/stamps.txt
