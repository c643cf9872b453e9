#!/bin/bash
# Round-4: the row catch-up's LDS step-table window (A/B against the global-table build),
# deferred / kernel tests, C3 bench lines. Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_deferred.py tests/test_gpu_kernels.py tests/test_gpu_gemm_planes.py > gpurun_out/t17.log 2>&1 || { tail -30 gpurun_out/t17.log; exit 1; }
tail -1 gpurun_out/t17.log
for i in 1 2; do
  for L in "" rl_ctr_prediction_amd/variants/lib_rowsglobal.so; do
    CTR_HIP_LIB=${L:-rl_ctr_prediction_amd/libctr_hip.so} timeout -k 10 300 python tools/rows_bench.py --config c3 > gpurun_out/rows17_$i.txt 2>&1 || { cat gpurun_out/rows17_$i.txt; exit 1; }
    echo "lib=${L:-default}"; grep -v amdgpu.ids gpurun_out/rows17_$i.txt
  done
done
for C in c3 c3; do
  timeout -k 10 600 python bench.py --config $C --steps 20 --warmup 5 --no-driver-loop --no-cpu-baseline > gpurun_out/b17_$C.log 2>&1 || { tail -5 gpurun_out/b17_$C.log; exit 1; }
  echo "$C $(tail -1 gpurun_out/b17_$C.log | grep -o '"value": [0-9.]*' | head -1)"
done
