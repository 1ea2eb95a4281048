#!/bin/bash
# Control-loop diagnostics on the box: the loop's time (FEC_VR_DEBUG) with the feedback jobs on the
# producer thread vs run to the end first on the control thread (FEC_VR_FB_SYNC), and with 1 / 8 workers.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-vrdiag}
mkdir -p $OUT
cd $R
C=fec_erasure_code_unit_test_relay_amd/csrc
python3 -c "
import sys; sys.path.insert(0,'.')
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern
load_pattern('bin_erasure').tofile('/tmp/bin_erasure.bin')" || exit 1
g++ -O2 -std=c++17 -pthread -I$C -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/vr_plan_bench.cpp $C/fec_vr.cpp $C/fec_host.cpp -o /tmp/vr_plan_bench -Lfec_erasure_code_unit_test_relay_amd -lfec_amd -Wl,-rpath,$R/fec_erasure_code_unit_test_relay_amd -L/opt/rocm/lib -lamdhip64 || exit 1
for v in "" "FEC_VR_FB_SYNC=1" "FEC_VR_THREADS=1" "FEC_VR_THREADS=2" "FEC_VR_THREADS=3" "FEC_VR_THREADS=4" "FEC_VR_THREADS=8" "" "FEC_VR_THREADS=2" "FEC_VR_THREADS=4"; do
  echo "[$v] $(env $v FEC_VR_DEBUG=1 timeout 60 /tmp/vr_plan_bench /tmp/bin_erasure.bin 30 2>&1 | grep -E 'loop [0-9]' | sort -t' ' -k7 -n | head -1 | cut -c1-60) | $(env $v timeout 60 /tmp/vr_plan_bench /tmp/bin_erasure.bin 30 2>&1 | cut -c1-60)"
done | tee $OUT/diag.txt
nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())"
