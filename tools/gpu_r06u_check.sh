#!/bin/bash
# Episode-grid A/B (headline step, config 3), then the bench without its rocprof child.
#   bash tools/gpu_r06u_check.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06u}
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u tools/step_ab.py env=FEC_EPISODE_GRID:245 env=FEC_EPISODE_GRID:32768 > $OUT/step_ab.txt 2>&1 || { tail -20 $OUT/step_ab.txt; exit 1; }
timeout -k 10 300 python3 -u tools/step_ab.py env=FEC_EPISODE_GRID:32768 env=FEC_EPISODE_GRID:245 >> $OUT/step_ab.txt 2>&1 || { tail -20 $OUT/step_ab.txt; exit 1; }
cat $OUT/step_ab.txt
timeout -k 10 200 python3 -u tools/config3_ab.py FEC_EPISODE_GRID=88 FEC_EPISODE_GRID=32768 6 > $OUT/config3_ab.txt 2>&1 || { tail -20 $OUT/config3_ab.txt; exit 1; }
cat $OUT/config3_ab.txt
timeout -k 10 900 python -u bench.py --no-rocprof > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); c=d['configs']
print(d['value'], d['ms_per_step'])
for k in ('config3_decode_10_5_2','config4_adaptive'): print(k, json.dumps(c[k])[:420])
print('relay_adaptive', json.dumps(c['relay_adaptive'])[:200])"
