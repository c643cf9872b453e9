#!/bin/bash
# C3 A/B: plan lookahead for DeepFM (with the catch-up over the plan's rows) vs in-step plans.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 0 1; do
    CTR_PLAN_LOOKAHEAD=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c3la.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/c3la.log; exit 1; }
    echo "lookahead $v: $(tail -1 gpurun_out/c3la.log | cut -c100-150)"
  done
done
