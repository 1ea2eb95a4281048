set -o pipefail
O=gpurun_out/ep5; mkdir -p $O
timeout -k 10 100 python -u tools/stamps_plan.py > $O/st.txt 2>&1 || exit 1
for g in 256 512 1024 2048 4096; do FEC_REC_GRID=$g timeout -k 10 100 python -u tools/step_parts.py --reps 10 2>&1 | grep P= | sed "s/^/rgrid=$g /" >> $O/a.txt || exit 1; done
grep -v amdgpu.ids $O/st.txt; cat $O/a.txt
