#!/bin/bash
# Round-4: the FM step tail with its scalars prefetched: FM / deferred / driver tests, C2
# bench lines, C2 kernel stats. Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_deferred.py tests/test_gpu_models.py tests/test_gpu_driver_loop.py tests/test_gpu_streaming.py tests/test_gpu_kernels.py > gpurun_out/t26.log 2>&1 || { tail -30 gpurun_out/t26.log; exit 1; }
tail -1 gpurun_out/t26.log
for i in 1 2 3; do
  timeout -k 10 600 python bench.py --config c2 --steps 20 --warmup 5 --no-driver-loop --no-cpu-baseline > gpurun_out/b26_$i.log 2>&1 || { tail -5 gpurun_out/b26_$i.log; exit 1; }
  echo "c2 $(tail -1 gpurun_out/b26_$i.log | grep -o '"value": [0-9.]*' | head -1)"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof26_c2 -o run -- \
  python3 bench.py --config c2 --steps 50 --warmup 3 --no-cpu-baseline --no-driver-loop > gpurun_out/prof26_c2.log 2>&1 || { tail -5 gpurun_out/prof26_c2.log; exit 1; }
grep -E "fm_step_tail|deferred_rows|fm_forward" gpurun_out/prof26_c2/run_kernel_stats.csv | cut -d, -f1-4
