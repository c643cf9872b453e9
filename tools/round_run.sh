#!/bin/bash
# Round evidence in one GPU call: parity tests + smoke + benches (tools/gpu_check.sh),
# then the rocprofv3 kernel trace + PMC passes of the C3 bench (tools/gpu_profile.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export BENCH_LIST="${BENCH_LIST:---steps 30 --warmup 5}"
bash tools/gpu_check.sh || exit $?
for CFG in ${PROFILE_CFGS:-c3}; do
  CFG=$CFG TAG=${TAG:-r01} bash tools/gpu_profile.sh > gpurun_out/profile_$CFG.log 2>&1 || exit $?
done
echo done
