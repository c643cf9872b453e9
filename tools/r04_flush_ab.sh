#!/bin/bash
# Flush kernels A/B (tools/flush_bench.py): the tile kernel vs the LDS-DMA kernel at the C3
# and C5 table shapes, 1 and 20 replayed steps. Output gpurun_out/r04_flush_ab.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/r04_flush_ab.txt
timeout -k 10 300 python tools/flush_bench.py --V 10000000 --K 64 --variants tile,dma,tile,dma --steps-list 1,20 --reps 3 >> gpurun_out/r04_flush_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/flush_bench.py --V 40000000 --K 128 --variants tile,dma --steps-list 1,20 --reps 2 >> gpurun_out/r04_flush_ab.txt 2>&1 || exit 1
cat gpurun_out/r04_flush_ab.txt
