#!/bin/bash
# In-step GEMM tiling A/B: rocprofv3 kernel traces of the C3 bench under per-shape overrides
# (CTR_GEMM_PLANES_SHAPE_CFG), one trace per variant in $VARIANTS ("name|override" lines);
# tools/gemm_instep.py then prints each GEMM launch's median duration per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
while IFS='|' read -r name cfg; do
  [ -z "$name" ] && continue
  OUT=gpurun_out/instep_$name
  mkdir -p $OUT
  CTR_GEMM_PLANES_SHAPE_CFG="$cfg" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- \
    python3 bench.py --config c3 --steps 30 --warmup 3 --no-cpu-baseline --no-driver-loop > $OUT/bench.log 2>&1 || exit $?
  echo "$name $(tail -1 $OUT/bench.log | grep -o '"value": [0-9.]*')"
done <<< "$VARIANTS"
