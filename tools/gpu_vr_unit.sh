#!/bin/bash
# Config 4 device work: VR GPU tests, then encode/decode timing per tile-segment unit
# (FEC_VR_TILE_UNIT) and a kernel trace of the default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-vru}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_vr.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for u in ${FEC_UNITS:-4 8 16 4 8 16}; do
    echo "unit $u"; FEC_VR_TILE_UNIT=$u timeout -k 10 120 python -u tools/vr_prof.py 20 2>&1 | grep -E "encode|decode" | tee -a $OUT/vr_unit.log || exit 1
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/vr_prof.py 20 > $OUT/rocprof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/rocprof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp "$f" $OUT/kernel_stats.csv
python3 - $OUT/kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{float(r['AverageNs'])/1e3:9.1f} us  x{r['Calls']:>3}  {r['Name'][:90]}")
PY
