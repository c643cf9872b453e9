#!/bin/bash
# round 3, GPU run 7: padded/varsplit diagnostic after the plan-stream allocation fix; eager
# (host-paced) step cost at C3 for the fused and the row-sharded trainer
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/diag_padded.py > gpurun_out/diag_padded2.log 2>&1
echo "diag rc=$?"
grep "^FM\|^DeepFM" gpurun_out/diag_padded2.log | cut -c1-200
for a in "" "--sharding rows" "--no-graphs" "--sharding rows --no-graphs"; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline $a \
    > gpurun_out/b7.json 2> gpurun_out/b7.err || { tail -5 gpurun_out/b7.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b7.json'));print('$a', round(d['value']/1e6,3), round(d['ms_per_step'],4))"
done
