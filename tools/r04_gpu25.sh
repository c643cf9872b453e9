#!/bin/bash
# Round-4: the sharded file (capacity check now in a fresh process), then the whole suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sharded.py > gpurun_out/t25.log 2>&1 || { tail -30 gpurun_out/t25.log; exit 1; }
tail -1 gpurun_out/t25.log
PYTEST_STOP=--maxfail=10 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
echo smoke ok
