#!/bin/bash
# Host-inclusive zero-copy and per-packet latency with the process on either socket.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-numa}
mkdir -p $OUT
cd $R
for f in /sys/class/drm/card*/device/numa_node; do echo "$f: $(cat $f)"; done 2>/dev/null | head -4
g++ -O2 -std=c++17 -I include tools/stream_latency.cpp -L fec_erasure_code_unit_test_relay_amd -lfec_amd -Wl,-rpath,$R/fec_erasure_code_unit_test_relay_amd -o /tmp/stream_latency || exit 1
for cpus in 0-15 64-79; do
  echo "== cpus $cpus"
  timeout -k 10 120 taskset -c $cpus python3 -u tools/host_zero_copy_exp.py --reps 3 --no-pipe 2>&1 | grep -v amdgpu.ids | head -1
  timeout -k 10 120 taskset -c $cpus /tmp/stream_latency 20000 2>&1 | tail -1
done | tee $OUT/numa.txt
