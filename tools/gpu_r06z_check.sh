#!/bin/bash
# After restricting the encoder scan: headline kernel times and step, the encoder probe, parity of the
# encoder users.   bash tools/gpu_r06z_check.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06z}
mkdir -p $OUT
bash $R/tools/gpu_enc_time.sh ${1:-r06z}_t || exit 1
cd $R && timeout -k 10 300 python3 -u tools/enc_rl_probe.py > $OUT/enc_rl_probe.txt 2>&1 || { tail -20 $OUT/enc_rl_probe.txt; exit 1; }
grep -v amdgpu.ids $OUT/enc_rl_probe.txt
cd $R && timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_swdf.py tests/test_sdswdf.py tests/test_vr.py tests/test_gpu_session.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
