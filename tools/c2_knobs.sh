#!/bin/bash
# C2 A/B of step-structure knobs, alternating, 20-step regions (the driver's).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "base" "CTR_FUSE_APPLY_MIN_K=16" "CTR_PLAN_FUSED_HIST=1" "CTR_FM_TAIL=0" "CTR_PLAN_FIRST=0"; do
    envs=""; [ "$cfg" != "base" ] && envs="$cfg"
    env $envs timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c2k.log 2>&1 || { echo "$cfg failed"; tail -3 gpurun_out/c2k.log; exit 1; }
    echo "$cfg: $(tail -1 gpurun_out/c2k.log | cut -c100-150)"
  done
done
