#!/bin/bash
# Round-4: dH1 (M 8192, N 300, K 200 -> Kp 224, B k-strided) tiling in the C3 step, per-shape
# override, alternating bench runs; the chooser's tile first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "
from rl_ctr_prediction_amd import hip_ops as H
print('dH1 cfg', H.gemm_planes_config(False, True, 8192, 300, 200))
print('fwd1 cfg', H.gemm_planes_config(False, False, 8192, 200, 300))
" 2>&1 | grep cfg
for i in 1 2; do
  for T in default 11 2 17; do
    if [ $T = default ]; then E=""; else E="CTR_GEMM_PLANES_SHAPE_CFG=8192,300,224,0,1=$T,1,1"; fi
    env $E timeout -k 10 600 python bench.py --config c3 --steps 20 --warmup 5 --no-driver-loop --no-cpu-baseline > gpurun_out/b28_$T.log 2>&1 || { tail -5 gpurun_out/b28_$T.log; exit 1; }
    echo "dH1 tile=$T $(tail -1 gpurun_out/b28_$T.log | grep -o '"value": [0-9.]*' | head -1)"
  done
done
