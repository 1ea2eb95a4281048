#!/bin/bash
# Type-2 relay frame stores from five LDS dwords per chunk (FEC_SWDF_STORE5=1, default) vs dword by
# dword (0): relay GPU tests, then kernel times of tools/swdf_bench.py per setting.   bash tools/gpu_store5_ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-store5}
mkdir -p $OUT
cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_swdf.py tests/test_sdswdf.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
for C in 1 0 1 0; do
  FEC_SWDF_STORE5=$C timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/s$C -o run -- python3 $R/tools/swdf_bench.py 20 > $OUT/s$C.log 2>&1 || { tail -20 $OUT/s$C.log; exit 1; }
  echo "FEC_SWDF_STORE5=$C"; python3 $R/tools/kstats.py $(ls -t $(find $OUT/s$C -name '*.db') | head -1) | grep sw_fast
done
