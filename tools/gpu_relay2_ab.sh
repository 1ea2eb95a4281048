#!/bin/bash
# Type-2 relay kernel A/B: the row-scatter kernel at its tile sizes (FEC_SWDF_TR = 64 / 48 with 512
# threads, 32 with 256 threads) against round 5's three-tile kernel (FEC_SWDF_RELAY=3).  Parity
# tests (fixed-rate relay, the adaptive relay's 360 000-seq schedule, the session) on the default,
# the fixed-rate parity tests on the other tile sizes, kernel times of each variant, the default's
# phase stamps, then its FETCH_SIZE / WRITE_SIZE.   bash tools/gpu_relay2_ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-relay2}
mkdir -p $OUT/pmc
cd $R && timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_swdf.py tests/test_sdswdf.py tests/test_gpu_session.py -m gpu -k "swdf_bit_exact or swdf_large or full_schedule or session" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for TR in 48 32; do
  FEC_SWDF_TR=$TR timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_swdf.py -m gpu -k "swdf_bit_exact or swdf_large" > $OUT/pytest_tr$TR.log 2>&1 || { tail -30 $OUT/pytest_tr$TR.log; exit 1; }
  echo "TR=$TR: $(tail -1 $OUT/pytest_tr$TR.log)"
done
cd /tmp && export TMPDIR=/tmp
for V in "FEC_SWDF_TR=64" "FEC_SWDF_TR=48" "FEC_SWDF_TR=32" "FEC_SWDF_RELAY=3"; do
  env $V timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$V -o run -- python3 $R/tools/swdf_bench.py 20 > $OUT/$V.log 2>&1 || { tail -20 $OUT/$V.log; exit 1; }
  python3 $R/tools/kstats.py $(find $OUT/$V -name '*kernel_stats.csv') > $OUT/${V}_stats.txt 2>&1
  echo "== $V"; grep -E "fast_relay" $OUT/${V}_stats.txt
done
for TR in 64 32; do
  FEC_SWDF_TR=$TR FEC_SWDF_STAMPS=1 timeout -k 10 120 python3 $R/tools/swdf_bench.py 1 > $OUT/stamps_tr$TR.txt 2>&1 || { tail -20 $OUT/stamps_tr$TR.txt; exit 1; }
  grep "STAMPS fast relay" $OUT/stamps_tr$TR.txt | head -1
done
i=0
for C in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc/p$i -o pmc -- python3 $R/tools/swdf_bench.py 2 > $OUT/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/pmc/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $(find $OUT/pmc -name '*counter_collection.csv') > $OUT/pmc_summary.txt
grep -A6 -E "fast_relay" $OUT/pmc_summary.txt | grep -E "fast_relay|traffic"
