#!/bin/bash
# Round-4: dW0 split count in the C3 step (fewer splits: fewer CUs taken from the scatter
# chain beside it), alternating bench runs. Per-shape override: M,N,Kp,a_rc,b_rc=tile,splits,xg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for S in 9 6 4; do
    CTR_GEMM_PLANES_SHAPE_CFG="300,1665,8192,1,1=25,$S,1" timeout -k 10 600 python bench.py --config c3 --steps 20 --warmup 5 --no-driver-loop --no-cpu-baseline > gpurun_out/b18_$S.log 2>&1 || { tail -5 gpurun_out/b18_$S.log; exit 1; }
    echo "splits=$S $(tail -1 gpurun_out/b18_$S.log | grep -o '"value": [0-9.]*' | head -1)"
  done
done
