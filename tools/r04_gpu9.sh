#!/bin/bash
# Round-4 GPU session 10: the next batch's catch-up in the step's tail — its bitwise test,
# the deferred / driver-loop suites, C3 / IPNN bench A/B (CTR_CATCHUP_AHEAD=1 default vs 0)
# and a C3 kernel trace. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PYTEST_STOP=--maxfail=3 bash tools/gpu_tests.sh tests/test_gpu_catchup_ahead.py tests/test_gpu_deferred.py tests/test_gpu_streaming.py tests/test_gpu_driver_loop.py || exit 1
ENV_A="CTR_CATCHUP_AHEAD=1" ENV_B="CTR_CATCHUP_AHEAD=0" CFGS="c3 ipnn" RUNS=2 BENCH_ARGS="--no-driver-loop" bash tools/env_ab.sh || exit 1
OUT=gpurun_out/r04_ahead_c3; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-driver-loop > $OUT/bench.log 2>&1 || exit 1
python3 tools/kstats.py $(find $OUT -name "*kernel_stats.csv" | head -1) 14
