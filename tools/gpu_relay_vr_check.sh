#!/bin/bash
# Relay parity (fixed-rate type 2/3, the adaptive relay's 360 000-seq schedule, the session), then the
# adaptive relay's wall time per run and its kernel trace.   bash tools/gpu_relay_vr_check.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-relay_vr}
mkdir -p $OUT
cd $R && timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_swdf.py tests/test_sdswdf.py tests/test_gpu_session.py -m gpu -k "swdf_bit_exact or swdf_large or full_schedule or session" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python3 -u tools/relay_vr_prof.py 5 > $OUT/relay_vr_wall.txt 2>&1 || { tail -20 $OUT/relay_vr_wall.txt; exit 1; }
cat $OUT/relay_vr_wall.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/relay_vr_prof.py 3 2 > $OUT/relay_vr_prof.log 2>&1 || { tail -20 $OUT/relay_vr_prof.log; exit 1; }
python3 $R/tools/kstats.py $(find $OUT/trace -name '*kernel_stats.csv') > $OUT/relay_vr_stats.txt 2>&1
head -16 $OUT/relay_vr_stats.txt
