#!/bin/bash
# A GPU call for kernel work: selected parity tests, then A/B commands, each under its own time
# limit; stops at the first failure.  Usage: gpu_ab.sh TAG "pytest -k expr" "cmd1" "cmd2" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
K="$1"; shift
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
  tail -3 $OUT/pytest.log
fi
i=0
for C in "$@"; do
  i=$((i+1))
  echo "== $C" | tee -a $OUT/ab.log
  timeout -k 10 600 bash -c "$C" >> $OUT/ab.log 2>&1 || { echo "step $i failed: $C"; tail -40 $OUT/ab.log; exit 1; }
done
cat $OUT/ab.log
