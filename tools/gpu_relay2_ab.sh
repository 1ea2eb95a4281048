#!/bin/bash
# Type-2 relay kernel A/B: the row-scatter kernel (default) against round 5's three-tile kernel
# (FEC_SWDF_RELAY=3).  Parity tests (fixed-rate relay, the adaptive relay's 360 000-seq schedule,
# the session), kernel times of each variant, the row scatter's phase stamps, then its FETCH_SIZE /
# WRITE_SIZE.   bash tools/gpu_relay2_ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-relay2}
mkdir -p $OUT/pmc
cd $R && timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_swdf.py tests/test_sdswdf.py tests/test_gpu_session.py -m gpu -k "swdf_bit_exact or swdf_large or full_schedule or session" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
for V in 2 3; do
  FEC_SWDF_RELAY=$V timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/v$V -o run -- python3 $R/tools/swdf_bench.py 20 > $OUT/v$V.log 2>&1 || { tail -20 $OUT/v$V.log; exit 1; }
  python3 $R/tools/kstats.py $(find $OUT/v$V -name '*kernel_stats.csv') > $OUT/v${V}_stats.txt 2>&1
  grep -E "kernel|fast" $OUT/v${V}_stats.txt
done
FEC_SWDF_STAMPS=1 timeout -k 10 120 python3 $R/tools/swdf_bench.py 1 > $OUT/stamps.txt 2>&1 || { tail -20 $OUT/stamps.txt; exit 1; }
grep STAMPS $OUT/stamps.txt
i=0
for C in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc/p$i -o pmc -- python3 $R/tools/swdf_bench.py 2 > $OUT/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/pmc/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $(find $OUT/pmc -name '*counter_collection.csv') > $OUT/pmc_summary.txt
grep -E "fast_relay|fast_dest" $OUT/pmc_summary.txt
