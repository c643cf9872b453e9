#!/bin/bash
# Round-4 GPU session 1: parity tests of this round's changes, flush A/B, C3/C2 bench lines,
# dX tiling in-step A/B, scatter counters. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_STOP="--maxfail=15" bash tools/gpu_tests.sh tests/test_gpu_kernels.py tests/test_gpu_deferred.py tests/test_gpu_driver_loop.py tests/test_gpu_sharded.py tests/test_ops_abi.py "tests/test_gpu_gemm_planes.py::test_gemm_planes_every_tiling"
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests.log | head -20
[ $rc -le 1 ] || exit $rc  # a crash, abort or time limit: nothing more on the GPU in this call
bash tools/r04_flush_ab.sh > gpurun_out/flush_ab.log 2>&1 || { tail -5 gpurun_out/flush_ab.log; exit 1; }
echo "flush ab ok"; cat gpurun_out/r04_flush_ab.txt | head -20
for C in c3 c2; do
  timeout -k 10 300 python bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04_bench_$C.log 2>&1 || { tail -5 gpurun_out/r04_bench_$C.log; exit 1; }
  echo "bench $C $(tail -1 gpurun_out/r04_bench_$C.log | grep -o '"value": [0-9.]*')"
done
ENV_A="CTR_SEG_DIRECT=1" ENV_B="CTR_SEG_DIRECT=0" CFGS="c3 c2" RUNS=1 bash tools/env_ab.sh || exit 1
ENV_A="CTR_PLAN_V2=1" ENV_B="CTR_PLAN_V2=0" CFGS="c2 c3" RUNS=1 bash tools/env_ab.sh || exit 1
