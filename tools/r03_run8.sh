#!/bin/bash
# round 3, GPU run 8: GEMM counters per C3 shape; C3 kernel trace + FETCH/WRITE passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gemm_planes_pmc.sh > gpurun_out/gemm_pmc.log 2>&1 || { echo "gemm pmc failed"; tail -20 gpurun_out/gemm_pmc.log; exit 1; }
tail -30 gpurun_out/gemm_pmc.log
CFG=c3 TAG=r03 bash tools/gpu_profile.sh > gpurun_out/profile_c3.log 2>&1 || { echo "profile failed"; tail -5 gpurun_out/profile_c3.log; exit 1; }
echo profile ok
