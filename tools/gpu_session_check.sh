#!/bin/bash
# The relay session and the adaptive relay: parity (session per seq + 360k digests, relay fixed-rate
# and adaptive), the session's time per run with the rotating-row lineage kernel and with the map
# kernel (FEC_SES_LIN_MAP=1), its kernel trace, the adaptive relay's wall time.
#   bash tools/gpu_session_check.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-session}
mkdir -p $OUT
cd $R && timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_session.py tests/test_swdf.py tests/test_sdswdf.py tests/test_vr.py -m gpu -k "session or swdf_bit_exact or full_schedule or adaptive" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python3 -u tools/session_prof.py 3 > $OUT/session_wall.txt 2>&1 || { tail -20 $OUT/session_wall.txt; exit 1; }
cat $OUT/session_wall.txt
FEC_SES_LIN_MAP=1 timeout -k 10 200 python3 -u tools/session_prof.py 3 > $OUT/session_wall_map.txt 2>&1 || { tail -20 $OUT/session_wall_map.txt; exit 1; }
echo "map kernel:"; cat $OUT/session_wall_map.txt
timeout -k 10 200 python3 -u tools/relay_vr_prof.py 5 > $OUT/relay_vr_wall.txt 2>&1 || { tail -20 $OUT/relay_vr_wall.txt; exit 1; }
cat $OUT/relay_vr_wall.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o session -- python3 $R/tools/session_prof.py 2 > $OUT/session_prof.log 2>&1 || { tail -20 $OUT/session_prof.log; exit 1; }
python3 $R/tools/kstats.py $(find $OUT/trace -name '*kernel_stats.csv') > $OUT/session_stats.txt 2>&1
head -14 $OUT/session_stats.txt
