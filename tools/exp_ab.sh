set -o pipefail
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; tail -3 $O/pytest.log
timeout -k 10 200 python -u tools/graph_parts.py 2>&1 | grep -v amdgpu.ids | sed 's/^/new /'
(cd tmp_base && timeout -k 10 200 python -u tools/graph_parts.py 2>&1 | grep -v amdgpu.ids | sed 's/^/base /')
timeout -k 10 200 python -u tools/graph_parts.py --packets 360000 --tbn 10,5,2 2>&1 | grep -v amdgpu.ids | sed 's/^/new /'
(cd tmp_base && timeout -k 10 200 python -u tools/graph_parts.py --packets 360000 --tbn 10,5,2 2>&1 | grep -v amdgpu.ids | sed 's/^/base /')
