# Config 4 host plan vs the decoder workers' queue polling (FEC_VR_SPIN) and count, alternating, on the
# box host; records the CPU topology the plan's threads land on.
set -e
out=gpurun_out/${1:-plan_spin}
mkdir -p $out
python -c "from fec_erasure_code_unit_test_relay_amd.streams import load_pattern; load_pattern(\"bin_erasure\").tofile(\"$out/pat.bin\")"
{ nproc; taskset -pc $$; cat /sys/devices/system/cpu/cpu0/topology/thread_siblings_list; cat /sys/devices/system/cpu/cpu1/topology/thread_siblings_list; } > $out/topology.txt 2>&1 || true
for rep in 1 2 3; do
for cfg in "FEC_VR_SPIN=4096" "FEC_VR_SPIN=0" "FEC_VR_SPIN=256" "FEC_VR_SPIN=0 FEC_VR_THREADS=4"; do
  echo "[$cfg]"; env $cfg timeout -k 10 60 ./tools/ubench/vr_plan_bench $out/pat.bin 30
done; done > $out/plan_spin_ab.txt 2>&1
rm -f $out/pat.bin
