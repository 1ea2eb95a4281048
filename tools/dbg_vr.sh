set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/debug_vr_tile.py 8 2>&1 | tee gpurun_out/dbg_vr1.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_vr.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -5
