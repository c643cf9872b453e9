#!/bin/bash
# Round-4: the staged-row fast path (IPNN forward, Feature_Embedding, IPNN LDS backward) and
# the variable-width column sort: their tests, kernel timings, bench lines. Stops at the
# first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_torch_ops.py tests/test_gpu_deferred.py > gpurun_out/t14.log 2>&1 || { tail -30 gpurun_out/t14.log; exit 1; }
tail -2 gpurun_out/t14.log
timeout -k 10 300 python tools/ipnn_bwd_bench.py --kernels default,sreg > gpurun_out/r04_ipnn_bwd3.txt 2>&1 || { cat gpurun_out/r04_ipnn_bwd3.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_ipnn_bwd3.txt
timeout -k 10 300 python tools/plan_bench.py --configs c2,c3 > gpurun_out/r04_plan_bench_v3.txt 2>&1 || { cat gpurun_out/r04_plan_bench_v3.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_plan_bench_v3.txt
CTR_HIP_LIB=rl_ctr_prediction_amd/variants/lib_cptrace.so timeout -k 10 120 python tools/colplan_trace.py > gpurun_out/r04_colplan_trace2.txt 2>&1 || { cat gpurun_out/r04_colplan_trace2.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_colplan_trace2.txt
for C in ipnn c3 c2 ipnn c3 c2; do
  timeout -k 10 600 python bench.py --config $C --steps 20 --warmup 5 --no-driver-loop --no-cpu-baseline > gpurun_out/b14_$C.log 2>&1 || { tail -5 gpurun_out/b14_$C.log; exit 1; }
  echo "$C $(tail -1 gpurun_out/b14_$C.log | grep -o '"value": [0-9.]*' | head -1)"
done
