#!/bin/bash
# C2 A/B with the host off the critical path: plan streams and lookahead depth.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "base" "CTR_PLAN_STREAMS=2" "LA3"; do
    envs=""; args=""
    [ "$cfg" = "CTR_PLAN_STREAMS=2" ] && envs="CTR_PLAN_STREAMS=2"
    [ "$cfg" = "LA3" ] && args="--lookahead 3"
    env $envs timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline $args > gpurun_out/c2k2.log 2>&1 || { echo "$cfg failed"; tail -3 gpurun_out/c2k2.log; exit 1; }
    echo "$cfg: $(tail -1 gpurun_out/c2k2.log | cut -c100-150)"
  done
done
