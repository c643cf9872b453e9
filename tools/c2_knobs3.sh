#!/bin/bash
# C2 A/B confirmation: one vs two lookahead plan streams (alternating, 3 runs each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for ps in 1 2; do
    CTR_PLAN_STREAMS=$ps timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c2k3.log 2>&1 || { echo "$ps failed"; tail -3 gpurun_out/c2k3.log; exit 1; }
    echo "plan_streams $ps: $(tail -1 gpurun_out/c2k3.log | cut -c100-150)"
  done
done
