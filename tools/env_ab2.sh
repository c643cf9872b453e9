#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for V in 0 1; do for C in c2 c3; do
  CTR_PLAN_FIRST=$V timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/envab.log 2>&1 || { tail -3 gpurun_out/envab.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/envab.log') if l.startswith('{')][-1]); print('plan_first=$V', '$C', round(d['value']/1e6,3), 'M ex/s', round(d['ms_per_step'],4), 'ms')"
done; done
