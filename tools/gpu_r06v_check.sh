#!/bin/bash
# Decode parity (every decode case), config 3 and headline-step A/B of the recovery placement and
# the episode grid.   bash tools/gpu_r06v_check.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06v}
mkdir -p $OUT
cd $R && timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_block.py -m gpu > $OUT/pytest_parity.log 2>&1 || { tail -30 $OUT/pytest_parity.log; exit 1; }
tail -1 $OUT/pytest_parity.log
timeout -k 10 300 python3 -u tools/config3_ab.py FEC_RECOVER_BESIDE=0,FEC_EPISODE_GRID=256 FEC_RECOVER_BESIDE=1,FEC_EPISODE_GRID=256 FEC_RECOVER_BESIDE=1,FEC_EPISODE_GRID=352 FEC_RECOVER_BESIDE=0,FEC_EPISODE_GRID=352 6 > $OUT/config3_ab.txt 2>&1 || { tail -20 $OUT/config3_ab.txt; exit 1; }
cat $OUT/config3_ab.txt
timeout -k 10 300 python3 -u tools/step_ab.py env=FEC_RECOVER_BESIDE:0 env=FEC_RECOVER_BESIDE:1 > $OUT/step_ab.txt 2>&1 || { tail -20 $OUT/step_ab.txt; exit 1; }
timeout -k 10 300 python3 -u tools/step_ab.py env=FEC_RECOVER_BESIDE:1 env=FEC_RECOVER_BESIDE:0 >> $OUT/step_ab.txt 2>&1 || { tail -20 $OUT/step_ab.txt; exit 1; }
cat $OUT/step_ab.txt
