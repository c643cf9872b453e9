#!/bin/bash
# Round-4 GPU session 6: C2 bimodality (4 alternating runs each: default hardware queues vs
# GPU_MAX_HW_QUEUES=8), the row-sharded step's host cost + its launch count, scatter
# counters, dX tiling in-step A/B. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ENV_A="GPU_MAX_HW_QUEUES=4" ENV_B="GPU_MAX_HW_QUEUES=8" CFGS="c2" RUNS=4 BENCH_ARGS="--no-driver-loop" bash tools/env_ab.sh || exit 1
timeout -k 10 300 python tools/sharded_host_cost.py --config c3 > gpurun_out/r04_sharded_host.txt 2>&1 || exit 1; tail -1 gpurun_out/r04_sharded_host.txt
OUT=gpurun_out/r04_sharded_trace; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- \
  python3 tools/sharded_host_cost.py --config c3 --modes eager --steps 10 > $OUT/run.log 2>&1 || exit 1
python3 tools/timeline.py $(find $OUT -name "*kernel_trace.csv" | head -1) --marker step_end_kernel > gpurun_out/r04_sharded_timeline.txt 2>&1; tail -3 gpurun_out/r04_sharded_timeline.txt
bash tools/scatter_pmc.sh > gpurun_out/r04_scatter_pmc.log 2>&1 || { tail -5 gpurun_out/r04_scatter_pmc.log; exit 1; }
tail -30 gpurun_out/r04_scatter_pmc.log
VARIANTS="base|
t29|8192,1664,320,0,1=29,1,1
t30|8192,1664,320,0,1=30,1,1
t31|8192,1664,320,0,1=31,1,1" bash tools/gemm_instep.sh || exit 1
python3 tools/gemm_instep.py gpurun_out/instep_base gpurun_out/instep_t29 gpurun_out/instep_t30 gpurun_out/instep_t31 > gpurun_out/r04_dx_instep.txt 2>&1; head -30 gpurun_out/r04_dx_instep.txt
