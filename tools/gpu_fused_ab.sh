#!/bin/bash
# Config 4 decode as one launch (copy + recovery, FEC_VR_FUSED=1 default) vs the fork (0): VR GPU
# tests, encode/decode timing A/B, the host-vs-GPU probe, a kernel trace.   bash tools/gpu_fused_ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-fused}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_vr.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in 0 1 0 1 0 1; do
    echo "FEC_VR_FUSED=$v" | tee -a $OUT/ab.log; FEC_VR_FUSED=$v timeout -k 10 120 python -u tools/vr_prof.py 20 2>&1 | grep -E "^encode:|^decode:" | tee -a $OUT/ab.log || exit 1
done
for v in 0 1; do
    echo "FEC_VR_FUSED=$v" | tee -a $OUT/probe.log; FEC_VR_FUSED=$v timeout -k 10 120 python -u tools/vr_host_probe.py 50 2>&1 | grep -v amdgpu.ids | tee -a $OUT/probe.log || exit 1
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/vr_prof.py 20 > $OUT/rocprof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/rocprof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp "$f" $OUT/kernel_stats.csv
python3 - $OUT/kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{float(r['AverageNs'])/1e3:9.1f} us  x{r['Calls']:>3}  {r['Name'][:90]}")
PY
