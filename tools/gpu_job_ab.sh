#!/bin/bash
# Config 4's multi-tuple encoder with segment runs per workgroup: VR GPU tests, encode/decode
# timing over FEC_VR_JOB_TILES values, a kernel trace of the default, then the headline step A/B
# against a baseline library build (libfec_amd_b.so).   bash tools/gpu_job_ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-jobab}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_vr.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in 0 8 16 24 32 0 16; do
    echo "FEC_VR_JOB_TILES=$v" | tee -a $OUT/ab.log; FEC_VR_JOB_TILES=$v timeout -k 10 120 python -u tools/vr_prof.py 20 2>&1 | grep -E "^encode:|^decode:" | tee -a $OUT/ab.log || exit 1
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/vr_prof.py 20 > $OUT/rocprof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/rocprof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp "$f" $OUT/kernel_stats.csv
python3 - $OUT/kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{float(r['AverageNs'])/1e3:9.1f} us  x{r['Calls']:>3}  {r['Name'][:90]}")
PY
timeout -k 10 300 python -u tools/step_lib_ab.py fec_erasure_code_unit_test_relay_amd/libfec_amd.so fec_erasure_code_unit_test_relay_amd/libfec_amd_b.so > $OUT/step_lib_ab.log 2>&1 || { tail -20 $OUT/step_lib_ab.log; exit 1; }
tail -8 $OUT/step_lib_ab.log
