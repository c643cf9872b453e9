#!/bin/bash
# Round-4 GPU session: IPNN backward kernels — bitwise tests, standalone timing, IPNN bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_STOP=--maxfail=3 bash tools/gpu_tests.sh tests/test_gpu_kernels.py -k "ipnn" || exit 1
timeout -k 10 300 python tools/ipnn_bwd_bench.py > gpurun_out/r04_ipnn_bwd.txt 2>&1 || { cat gpurun_out/r04_ipnn_bwd.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_ipnn_bwd.txt
ENV_A="CTR_IPNN_BWD=" ENV_B="CTR_IPNN_BWD=reg" CFGS="ipnn" RUNS=2 BENCH_ARGS="--no-driver-loop" bash tools/env_ab.sh || exit 1
