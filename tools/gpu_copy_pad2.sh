#!/bin/bash
# Copy row padding: decode parity tests, then the copy kernel under rocprof with and without padding.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-cpad}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "decode or copy or stream" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp
for pad in 0 def 0 def; do
  if [ $pad = def ]; then unset FEC_COPY_ROW_PAD; else export FEC_COPY_ROW_PAD=$pad; fi
  rm -rf $OUT/prof_$pad
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$pad -o s -- python3 $R/tools/profile_step.py --iters 20 > $OUT/prof_$pad.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_$pad.log; exit 1; }
  echo "pad $pad: $(grep -h copy_fast $(find $OUT/prof_$pad -name '*kernel_stats.csv') | cut -d, -f1-4)"
done | tee $OUT/ab.txt
