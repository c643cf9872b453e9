#!/bin/bash
# Round-4: the IPNN / plan kernel tests on the new defaults, the IPNN backward timing, bench
# lines for ipnn / c2 / c3, a kernel trace of c2 and ipnn. Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_models.py -k "ipnn or IPNN or plan" > gpurun_out/t13.log 2>&1 || { tail -30 gpurun_out/t13.log; exit 1; }
tail -2 gpurun_out/t13.log
timeout -k 10 300 python tools/ipnn_bwd_bench.py > gpurun_out/r04_ipnn_bwd2.txt 2>&1 || { cat gpurun_out/r04_ipnn_bwd2.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_ipnn_bwd2.txt
for C in ipnn c2 c3 c2; do
  timeout -k 10 600 python bench.py --config $C --steps 20 --warmup 5 --no-driver-loop > gpurun_out/b13_$C.log 2>&1 || { tail -5 gpurun_out/b13_$C.log; exit 1; }
  echo "$C $(tail -1 gpurun_out/b13_$C.log | grep -o '"value": [0-9.]*')"
done
for C in c2 ipnn; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof13_$C -o run -- \
    python3 bench.py --config $C --steps 50 --warmup 3 --no-cpu-baseline --no-driver-loop > gpurun_out/prof13_$C.log 2>&1 || { tail -5 gpurun_out/prof13_$C.log; exit 1; }
done
find gpurun_out/prof13_* -name "*kernel_stats.csv"
