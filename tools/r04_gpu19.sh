#!/bin/bash
# Round-4: the row catch-up with two rows per lane group (deferred tests, rows_bench, C3
# bench), then the dW0 split A/B (tools/r04_gpu18.sh). Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_deferred.py tests/test_gpu_models.py tests/test_gpu_streaming.py > gpurun_out/t19.log 2>&1 || { tail -30 gpurun_out/t19.log; exit 1; }
tail -1 gpurun_out/t19.log
for C in c3 c2; do
  timeout -k 10 300 python tools/rows_bench.py --config $C > gpurun_out/rows19_$C.txt 2>&1 || { cat gpurun_out/rows19_$C.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/rows19_$C.txt
done
bash tools/r04_gpu18.sh || exit 1
