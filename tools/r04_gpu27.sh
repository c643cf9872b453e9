#!/bin/bash
# Round-4 last check on the rebuilt library: smoke, kernel / deferred tests, the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_deferred.py tests/test_gpu_kernels.py > gpurun_out/t27.log 2>&1 || { tail -30 gpurun_out/t27.log; exit 1; }
tail -1 gpurun_out/t27.log
timeout -k 10 600 python bench.py > gpurun_out/b27.log 2>&1 || { tail -5 gpurun_out/b27.log; exit 1; }
tail -1 gpurun_out/b27.log | grep -o '"value": [0-9.]*' | head -1
