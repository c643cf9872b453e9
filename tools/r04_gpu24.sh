#!/bin/bash
# Round-4: the capacity-read test alone, then after the rest of its file (diagnosis).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sharded.py -k capacity_read > gpurun_out/t24a.log 2>&1; echo "alone rc=$?"; grep -E "passed|failed|AssertionError" gpurun_out/t24a.log | tail -3
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sharded.py -k "world1 or capacity_read" > gpurun_out/t24b.log 2>&1; echo "after world1 rc=$?"; grep -E "passed|failed|AssertionError" gpurun_out/t24b.log | tail -3
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sharded.py -k "host or capacity_read" > gpurun_out/t24c.log 2>&1; echo "after host rc=$?"; grep -E "passed|failed|AssertionError" gpurun_out/t24c.log | tail -3
