set -o pipefail
O=gpurun_out/ep4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; tail -3 $O/pytest.log
timeout -k 10 200 python -u tools/step_parts.py > $O/a.txt 2>&1 || exit 1
timeout -k 10 100 python -u tools/step_parts.py --packets 360000 --tbn 10,5,2 >> $O/a.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/a.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o sp -- python3 $GRAFT_REPO_ROOT/tools/step_parts.py --reps 5 > /dev/null 2>&1
