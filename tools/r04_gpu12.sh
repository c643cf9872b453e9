#!/bin/bash
# Round-4 late session: the GPU suite (stop after 10 failures), smoke, the IPNN backward
# timing (incl. the matrix-core kernel), the plan build timing + its per-kernel stats, the
# IPNN bench line on the current code. Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_STOP=--maxfail=10 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python tools/ipnn_bwd_bench.py > gpurun_out/r04_ipnn_bwd.txt 2>&1 || { cat gpurun_out/r04_ipnn_bwd.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_ipnn_bwd.txt
timeout -k 10 300 python tools/plan_bench.py --configs c2,c3 > gpurun_out/r04_plan_bench_v2.txt 2>&1 || { cat gpurun_out/r04_plan_bench_v2.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_plan_bench_v2.txt
CTR_HIP_LIB=rl_ctr_prediction_amd/variants/lib_cptrace.so timeout -k 10 120 python tools/colplan_trace.py > gpurun_out/r04_colplan_trace.txt 2>&1 || { cat gpurun_out/r04_colplan_trace.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_colplan_trace.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_plan -o plan -- python tools/plan_bench.py --configs c2,c3 > gpurun_out/prof_plan.log 2>&1 || { tail -5 gpurun_out/prof_plan.log; exit 1; }
find gpurun_out/prof_plan -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | head -12
timeout -k 10 600 python bench.py --config ipnn --steps 20 --warmup 5 > gpurun_out/r04_bench_ipnn_final.log 2>&1 || { tail -5 gpurun_out/r04_bench_ipnn_final.log; exit 1; }
tail -1 gpurun_out/r04_bench_ipnn_final.log | cut -c1-300
