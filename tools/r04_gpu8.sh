#!/bin/bash
# Round-4 GPU session 8: C3 weight gradients on the side stream (default) vs serial on the
# main stream, three alternating runs; the IPNN line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ENV_A="CTR_WGRAD_SIDE=1" ENV_B="CTR_WGRAD_SIDE=0" CFGS="c3" RUNS=3 BENCH_ARGS="--no-driver-loop" bash tools/env_ab.sh || exit 1
timeout -k 10 400 python bench.py --config ipnn --steps 20 --warmup 5 --no-driver-loop > gpurun_out/r04_bench_ipnn.log 2>&1 || exit 1
tail -1 gpurun_out/r04_bench_ipnn.log | cut -c1-400
