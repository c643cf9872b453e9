#!/bin/bash
# Round-4: the 8-bit-capped equal-width column sort (plan tests, phase trace, build time),
# the C3 / C2 kernel stats after the staging / head changes, bench lines. Stops at the first
# failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "plan" > gpurun_out/t15.log 2>&1 || { tail -30 gpurun_out/t15.log; exit 1; }
tail -1 gpurun_out/t15.log
CTR_HIP_LIB=rl_ctr_prediction_amd/variants/lib_cptrace.so timeout -k 10 120 python tools/colplan_trace.py > gpurun_out/r04_colplan_trace3.txt 2>&1 || { cat gpurun_out/r04_colplan_trace3.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_colplan_trace3.txt | cut -c1-120
timeout -k 10 300 python tools/plan_bench.py --configs c2,c3 > gpurun_out/r04_plan_bench_v4.txt 2>&1 || { cat gpurun_out/r04_plan_bench_v4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_plan_bench_v4.txt | grep columns
for C in c3 c2; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof15_$C -o run -- \
    python3 bench.py --config $C --steps 50 --warmup 3 --no-cpu-baseline --no-driver-loop > gpurun_out/prof15_$C.log 2>&1 || { tail -5 gpurun_out/prof15_$C.log; exit 1; }
done
for C in c3 c2 c3 c2; do
  timeout -k 10 600 python bench.py --config $C --steps 20 --warmup 5 --no-driver-loop --no-cpu-baseline > gpurun_out/b15_$C.log 2>&1 || { tail -5 gpurun_out/b15_$C.log; exit 1; }
  echo "$C $(tail -1 gpurun_out/b15_$C.log | grep -o '"value": [0-9.]*' | head -1)"
done
