#!/bin/bash
# C2 bench under plan / scatter variants (env knobs of the library and the trainer)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for V in "A=1" "CTR_PLAN_IPT=4" "CTR_FUSE_APPLY=0" "CTR_PLAN_IPT=4 CTR_FUSE_APPLY=0"; do
  env $V timeout -k 10 300 python3 bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/planab.log 2>&1 || { tail -3 gpurun_out/planab.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/planab.log') if l.startswith('{')][-1]); print('$V', round(d['value']/1e6,3), 'M ex/s', round(d['ms_per_step'],4))"
done
