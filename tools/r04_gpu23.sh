#!/bin/bash
# Round-4: the sharded / deferred GPU tests after the capacity-read test's longer sleep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sharded.py tests/test_gpu_deferred.py -rA > gpurun_out/t23.log 2>&1 || { tail -30 gpurun_out/t23.log; exit 1; }
grep -E "capacity_read|passed|failed" gpurun_out/t23.log | tail -4
