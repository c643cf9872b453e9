#!/bin/bash
# Round-4: labels staged with the lookahead (next_y): tests, then alternating C2 / C3 bench
# runs with and without. Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_deferred.py tests/test_gpu_driver_loop.py tests/test_gpu_streaming.py > gpurun_out/t21.log 2>&1 || { tail -30 gpurun_out/t21.log; exit 1; }
tail -1 gpurun_out/t21.log
ENV_A="CTR_AB=stage" ENV_B="CTR_AB=nostage" ARGS_B="--no-stage-labels" CFGS="c2 c3" RUNS=3 BENCH_ARGS="--no-driver-loop" bash tools/env_ab.sh || exit 1
