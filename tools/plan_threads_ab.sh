set -e
mkdir -p gpurun_out/r04zj
python -c "from fec_erasure_code_unit_test_relay_amd.streams import load_pattern; load_pattern(\"bin_erasure\").tofile(\"gpurun_out/r04zj/pat.bin\")"
for rep in 1 2; do
for cfg in "" "FEC_VR_THREADS=4" "FEC_VR_THREADS=6" "FEC_VR_THREADS=12" "FEC_VR_PIN=1" "FEC_VR_PIN=0"; do
  echo "[$cfg]"
  env $cfg timeout -k 10 60 ./tools/ubench/vr_plan_bench gpurun_out/r04zj/pat.bin 30
done
done > gpurun_out/r04zj/plan_threads_ab.txt 2>&1
rm -f gpurun_out/r04zj/pat.bin
