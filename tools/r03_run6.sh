#!/bin/bash
# round 3, GPU run 6: padded-vs-varsplit diagnostic; sharded N=1 bench with the grow-only capacity
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/diag_padded.py > gpurun_out/diag_padded.log 2>&1
echo "diag rc=$?"
grep -v Gloo gpurun_out/diag_padded.log | grep -v socket | tail -40
timeout -k 10 300 python -u bench.py --steps 40 --warmup 10 --sharding rows --no-cpu-baseline \
  > gpurun_out/c3_rows.json 2> gpurun_out/c3_rows.err && tail -c 400 gpurun_out/c3_rows.json
