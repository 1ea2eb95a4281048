#!/bin/bash
# Round-6 GPU check: the session's GPU tests, then the bench with its rocprofv3 child.
# usage (on the box): bash tools/gpu_r06_check.sh TAG
set -o pipefail
TAG=${1:-r06}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_session.py -x -v --timeout 300 --timeout-method thread -m gpu \
    > gpurun_out/${TAG}_pytest_session.log 2>&1 || { echo "session tests failed"; tail -30 gpurun_out/${TAG}_pytest_session.log; exit 1; }
tail -8 gpurun_out/${TAG}_pytest_session.log
timeout -k 10 500 python -u bench.py --rocprof-keep gpurun_out/${TAG}_rocprof > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?
tail -3 gpurun_out/${TAG}_bench.err
exit $rc
