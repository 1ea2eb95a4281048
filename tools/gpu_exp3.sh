#!/bin/bash
# Config 4 kernels under rocprofv3 (kernel trace + PMC), PCIe duplex ceiling, per-packet latency.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-exp3}
mkdir -p $OUT
cd $R
timeout -k 10 120 python -u tools/pcie_duplex.py 2>&1 | tee $OUT/pcie_duplex.txt
g++ -O2 -std=c++17 -I include tools/stream_latency.cpp -L fec_erasure_code_unit_test_relay_amd -lfec_amd -Wl,-rpath,$R/fec_erasure_code_unit_test_relay_amd -o /tmp/stream_latency
timeout -k 10 120 /tmp/stream_latency 20000 2>&1 | tee $OUT/stream_latency.txt
bash tools/gpu_vr_prof.sh ${1:-exp3}_vr 2>&1 | tail -60 | tee $OUT/vr_prof.txt
cd $R
python3 -c "
import sys; sys.path.insert(0,'.')
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern
load_pattern('bin_erasure').tofile('/tmp/bin_erasure.bin')"
C=fec_erasure_code_unit_test_relay_amd/csrc
g++ -O2 -std=c++17 -pthread -I$C -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/vr_plan_bench.cpp -o /tmp/vr_plan_bench -Lfec_erasure_code_unit_test_relay_amd -lfec_amd -Wl,-rpath,$R/fec_erasure_code_unit_test_relay_amd -L/opt/rocm/lib -lamdhip64
for t in 1 2 4 8; do echo "threads $t: $(FEC_VR_DEBUG=1 FEC_VR_THREADS=$t timeout 60 /tmp/vr_plan_bench /tmp/bin_erasure.bin 20 2>&1 | tail -3 | tr '\n' ' ')"; done | tee $OUT/vr_plan_threads.txt
FEC_VR_DEBUG=1 timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
grep "vr control" $OUT/bench.err | tail -3
