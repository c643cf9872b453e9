#!/bin/bash
# C3 A/B of the weight-gradient GEMMs' split-K block target (CTR_GEMM_PLANES_WG_BLOCKS),
# alternating, 20-step regions (the driver's).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for wb in 512 256 384 768 1024; do
    CTR_GEMM_PLANES_WG_BLOCKS=$wb timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c3wb.log 2>&1 || { echo "$wb failed"; tail -3 gpurun_out/c3wb.log; exit 1; }
    echo "wg_blocks $wb: $(tail -1 gpurun_out/c3wb.log | cut -c100-150) $(tail -1 gpurun_out/c3wb.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
