set -o pipefail
O=gpurun_out/ep2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; tail -3 $O/pytest.log
timeout -k 10 200 python -u tools/step_parts.py --grids 8192,2048,1024,512,256 > $O/a.txt 2>&1 || exit 1
FEC_SIDE_CUS=16 timeout -k 10 100 python -u tools/step_parts.py >> $O/a.txt 2>&1 || exit 1
FEC_SIDE_CUS=32 timeout -k 10 100 python -u tools/step_parts.py >> $O/a.txt 2>&1 || exit 1
FEC_SIDE_PRIO=low timeout -k 10 100 python -u tools/step_parts.py >> $O/a.txt 2>&1 || exit 1
FEC_SIDE_PRIO=high timeout -k 10 100 python -u tools/step_parts.py >> $O/a.txt 2>&1 || exit 1
timeout -k 10 100 python -u tools/step_parts.py --packets 360000 --tbn 10,5,2 >> $O/a.txt 2>&1
grep -v amdgpu.ids $O/a.txt
