#!/bin/bash
# A/B of HIP runtime graph settings on the bench (C2 and C3 lines, no CPU baseline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # $1 = label, rest = env assignments
  local label=$1; shift
  for C in c2 c3; do
    env "$@" timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/envab.log 2>&1 || { tail -3 gpurun_out/envab.log; return 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/envab.log') if l.startswith('{')][-1]); print('$label', '$C', round(d['value']/1e6,3), 'M ex/s', round(d['ms_per_step'],4), 'ms')"
  done
}
run base A=1 && run pktcap DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 && run batch8 DEBUG_HIP_GRAPH_BATCH_SIZE=8 && run batch64 DEBUG_HIP_GRAPH_BATCH_SIZE=64 && run pktcap_false DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
