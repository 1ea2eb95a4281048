#!/bin/bash
# VR / session GPU tests, then the whole bench (its configs: config 4's host plan, the relays).
#   bash tools/gpu_r06t_check.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06t}
mkdir -p $OUT
cd $R && timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vr.py tests/test_gpu_session.py tests/test_session.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 900 python -u bench.py --no-rocprof > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); c=d['configs']
print(d['value'], d['ms_per_step'])
for k in ('config3_decode_10_5_2','config4_adaptive'): print(k, json.dumps(c[k])[:420])
print('relay_adaptive', json.dumps(c['relay_adaptive'])[:200])
print('relay_session', json.dumps(c['relay_session'])[:200])"
