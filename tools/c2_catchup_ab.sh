#!/bin/bash
# C2 A/B: catch-up over the lookahead plan's rows vs the id-driven mark + catch-up pair.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in 1 0; do
    CTR_CATCHUP_BY_PLAN=$v timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c2c.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/c2c.log; exit 1; }
    echo "by_plan $v: $(tail -1 gpurun_out/c2c.log | cut -c100-150)"
  done
done
