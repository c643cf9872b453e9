#!/bin/bash
# C2 A/B: lookahead depth 2 vs 3 (two plan streams), alternating, 3 runs each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for la in 2 3; do
    timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline --lookahead $la > gpurun_out/c2la.log 2>&1 || { echo "$la failed"; tail -3 gpurun_out/c2la.log; exit 1; }
    echo "lookahead $la: $(tail -1 gpurun_out/c2la.log | cut -c100-150)"
  done
done
