#!/bin/bash
# Round-4 GPU session 2: plan build times (v2 vs two-launch passes), dX tiling in-step A/B,
# scatter counters, sharded host cost, the host profile of the C2 step. Stops at the first
# failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 0; do CTR_PLAN_V2=$v timeout -k 10 300 python tools/plan_bench.py > gpurun_out/r04_plan_bench_v$v.txt 2>&1 || exit 1; echo "plan v2=$v"; tail -3 gpurun_out/r04_plan_bench_v$v.txt; done
timeout -k 10 300 python tools/host_profile.py --config c2 > gpurun_out/r04_host_profile_c2.txt 2>&1 || exit 1; head -3 gpurun_out/r04_host_profile_c2.txt
timeout -k 10 300 python tools/sharded_host_cost.py --config c3 > gpurun_out/r04_sharded_host.txt 2>&1 || exit 1; tail -1 gpurun_out/r04_sharded_host.txt
bash tools/scatter_pmc.sh > gpurun_out/r04_scatter_pmc.log 2>&1 || { tail -5 gpurun_out/r04_scatter_pmc.log; exit 1; }
tail -30 gpurun_out/r04_scatter_pmc.log
VARIANTS="base|
t29|8192,1664,320,0,1=29,1,1
t30|8192,1664,320,0,1=30,1,1
t31|8192,1664,320,0,1=31,1,1" bash tools/gemm_instep.sh || exit 1
python3 tools/gemm_instep.py gpurun_out/instep_base gpurun_out/instep_t29 gpurun_out/instep_t30 gpurun_out/instep_t31 > gpurun_out/r04_dx_instep.txt 2>&1; head -30 gpurun_out/r04_dx_instep.txt
