#!/bin/bash
# Quick: decode parity tests touching the copy, then two short bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-q3}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "row_padding or startup or bit_exact" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-host-inclusive --no-extra-configs > $OUT/bench$i.json 2> $OUT/bench$i.err || { echo "bench failed"; tail -20 $OUT/bench$i.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernels_ms_per_launch'], d['kernels_ms_back_to_back'])"; done
