#!/bin/bash
# Type-2 relay row scatter: rows-fastest item order (default) against g fastest (FEC_RELAY2_GFAST=1):
# relay parity suites on the default and on the switch, then each variant's kernel times (rocprofv3,
# alternated twice), the default's phase stamps and its LDS bank-conflict counters.
#   bash tools/gpu_relay2_gfast.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-gfast}
mkdir -p $OUT
cd $R && timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_swdf.py tests/test_sdswdf.py tests/test_gpu_session.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
for V in A B A2 B2; do
  case $V in A*) E="FEC_RELAY2_GFAST_UNSET=1";; B*) E="FEC_RELAY2_GFAST=1";; esac
  env $E timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$V -o run -- python3 $R/tools/swdf_bench.py 20 > $OUT/$V.log 2>&1 || { tail -20 $OUT/$V.log; exit 1; }
  python3 $R/tools/kstats.py $(find $OUT/$V -name '*kernel_stats.csv') > $OUT/${V}_stats.txt 2>&1
  echo "== $V ($E) $(grep -E 'fast_relay' $OUT/${V}_stats.txt)"
done
FEC_SWDF_STAMPS=1 timeout -k 10 120 python3 $R/tools/swdf_bench.py 1 > $OUT/stamps.txt 2>&1 || { tail -20 $OUT/stamps.txt; exit 1; }
grep "STAMPS fast relay" $OUT/stamps.txt | head -1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc -o pmc -- python3 $R/tools/swdf_bench.py 2 > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/pmc.log; exit 1; }
python3 $R/tools/pmc_summary.py $(find $OUT/pmc -name '*counter_collection.csv') > $OUT/pmc_summary.txt
grep -A5 -E "fast_relay" $OUT/pmc_summary.txt
