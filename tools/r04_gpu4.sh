#!/bin/bash
# Round-4 GPU session 4: column plan — plan tests, plan build times, C2 / C3 bench A/B
# (CTR_PLAN_COLS=1 default vs 0 the LSD plan) and a C2 kernel trace. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_STOP=--maxfail=5 bash tools/gpu_tests.sh tests/test_gpu_kernels.py -k "sparse_plan or segment" || exit 1
timeout -k 10 300 python tools/plan_bench.py > gpurun_out/r04_plan_bench_cols.txt 2>&1 || exit 1; cat gpurun_out/r04_plan_bench_cols.txt | grep config
ENV_A="CTR_PLAN_COLS=1" ENV_B="CTR_PLAN_COLS=0" CFGS="c2 c3" RUNS=2 BENCH_ARGS="--no-driver-loop" bash tools/env_ab.sh || exit 1
OUT=gpurun_out/r04_cols_c2; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-driver-loop > $OUT/bench.log 2>&1 || exit 1
python3 tools/kstats.py $(find $OUT -name "*kernel_stats.csv" | head -1) 16
