#!/bin/bash
# Round-4: fwd1 (M 8192, N 200, K 300 -> Kp 320) tiling in the C3 step, per-shape override,
# alternating bench runs; the chooser's tile (17) first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for T in default 12 3 11; do
    if [ $T = default ]; then E=""; else E="CTR_GEMM_PLANES_SHAPE_CFG=8192,200,320,0,0=$T,1,1"; fi
    env $E timeout -k 10 600 python bench.py --config c3 --steps 20 --warmup 5 --no-driver-loop --no-cpu-baseline > gpurun_out/b29_$T.log 2>&1 || { tail -5 gpurun_out/b29_$T.log; exit 1; }
    echo "fwd1 tile=$T $(tail -1 gpurun_out/b29_$T.log | grep -o '"value": [0-9.]*' | head -1)"
  done
done
