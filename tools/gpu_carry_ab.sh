#!/bin/bash
# Type-2 relay: parity tests, then kernel times with the front rows carried (default) and reloaded
# (FEC_SWDF_CARRY=0), then FETCH_SIZE / WRITE_SIZE of the carried run.   bash tools/gpu_carry_ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-carry}
mkdir -p $OUT/pmc
cd $R && timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_swdf.py tests/test_sdswdf.py -m gpu -k "not vr_schedule and not full_schedule" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
grep '^{"class"' $OUT/pytest.log > $OUT/per_call_relay.txt
cd /tmp && export TMPDIR=/tmp
for C in 1 0; do
  FEC_SWDF_CARRY=$C timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/c$C -o run -- python3 $R/tools/swdf_bench.py 20 > $OUT/c$C.log 2>&1 || { tail -20 $OUT/c$C.log; exit 1; }
  python3 $R/tools/kstats.py $(find $OUT/c$C -name '*kernel_stats.csv') > $OUT/c${C}_stats.txt 2>&1 || cp $(find $OUT/c$C -name '*kernel_stats.csv' | head -1) $OUT/c${C}_stats.txt
done
i=0
for C in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc/p$i -o pmc -- python3 $R/tools/swdf_bench.py 2 > $OUT/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/pmc/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $(find $OUT/pmc -name '*counter_collection.csv') > $OUT/pmc_summary.txt
cat $OUT/c1_stats.txt $OUT/c0_stats.txt $OUT/pmc_summary.txt $OUT/per_call_relay.txt
