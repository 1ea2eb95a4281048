#!/bin/bash
# Type-2 / type-3 relay GPU tests, then the type-2 kernels' times (tools/swdf_bench.py under a
# kernel trace).   bash tools/gpu_relay_quick.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-relayq}
mkdir -p $OUT
cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_swdf.py tests/test_sdswdf.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/k -o run -- python3 $R/tools/swdf_bench.py 20 > $OUT/k.log 2>&1 || { tail -20 $OUT/k.log; exit 1; }
python3 $R/tools/kstats.py $(find $OUT/k -name '*.db' | head -1) | tee $OUT/kernel_times.txt | grep sw_fast
