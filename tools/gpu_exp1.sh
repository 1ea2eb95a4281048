#!/bin/bash
# Store-policy A/B of the step kernels, eager vs graph timelines, VR GPU tests, bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-exp1}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_vr.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u tools/step_env_ab.py "" "FEC_TILE_NT=4" "FEC_COPY_NT=3" "FEC_TILE_NT=4,FEC_COPY_NT=3" > $OUT/store_ab.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/store_ab.txt; exit 1; }
cat $OUT/store_ab.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_eager -o bench -- python3 $R/bench.py --no-cpu-baseline --no-host-inclusive --no-extra-configs --warm-seconds 0.3 --no-graph > $OUT/bench_eager.json 2> $OUT/bench_eager.err || { echo "rocprof failed"; tail -30 $OUT/bench_eager.err; exit 1; }
KT=$(find $OUT/prof_eager -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_timeline.py "$KT" | tee $OUT/timeline_eager.txt
cd $R
C=fec_erasure_code_unit_test_relay_amd/csrc
python3 -c "
import sys; sys.path.insert(0,'.')
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern
load_pattern('bin_erasure').tofile('/tmp/bin_erasure.bin')"
g++ -O2 -std=c++17 -pthread -I$C -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/vr_plan_bench.cpp -o /tmp/vr_plan_bench -Lfec_erasure_code_unit_test_relay_amd -lfec_amd -Wl,-rpath,$R/fec_erasure_code_unit_test_relay_amd -L/opt/rocm/lib -lamdhip64
for t in 1 2 4 8 12; do echo "threads $t: $(FEC_VR_THREADS=$t timeout 60 /tmp/vr_plan_bench /tmp/bin_erasure.bin 30)"; done | tee $OUT/vr_plan_threads.txt
nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))"
