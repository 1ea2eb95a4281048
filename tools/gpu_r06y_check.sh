#!/bin/bash
# Encoder trimmed-size scan: parity of every encoder user (parity suite, relays, VR, session), the
# encoder probe at the adaptive relay's shapes, the adaptive relay's wall time.   bash tools/gpu_r06y_check.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06y}
mkdir -p $OUT
cd $R && timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_swdf.py tests/test_sdswdf.py tests/test_vr.py tests/test_gpu_session.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 -u tools/enc_rl_probe.py > $OUT/enc_rl_probe.txt 2>&1 || { tail -20 $OUT/enc_rl_probe.txt; exit 1; }
grep -v amdgpu.ids $OUT/enc_rl_probe.txt
timeout -k 10 200 python3 -u tools/relay_vr_prof.py 10 > $OUT/wall.txt 2>&1 || { tail -20 $OUT/wall.txt; exit 1; }
grep -v amdgpu.ids $OUT/wall.txt
