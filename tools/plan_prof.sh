# Config 4 host plan on the box host: plan timing (tools/ubench/vr_plan_bench) and the control loop's
# cycle split (vr_plan_bench_prof, linked against a -DFEC_VR_PROFILE build of the library).
set -e
out=gpurun_out/${1:-plan_prof}
mkdir -p $out
python -c "from fec_erasure_code_unit_test_relay_amd.streams import load_pattern; load_pattern(\"bin_erasure\").tofile(\"$out/pat.bin\")"
for i in 1 2 3; do timeout -k 10 60 ./tools/ubench/vr_plan_bench $out/pat.bin 30; done > $out/plan.txt 2>&1
if [ -x tools/ubench/vr_plan_bench_prof ]; then
  FEC_VR_DEBUG=1 timeout -k 10 60 ./tools/ubench/vr_plan_bench_prof $out/pat.bin 6 > $out/plan_prof.txt 2>&1
fi
rm -f $out/pat.bin
