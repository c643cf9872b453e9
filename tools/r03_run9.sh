#!/bin/bash
# round 3, GPU run 9: C3 A/B (plan lookahead, whole-M weight-gradient tiles), C2 trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab9.txt
for r in 1 2; do
  for e in "CTR_X=0" "CTR_PLAN_LOOKAHEAD=1" "CTR_GEMM_PLANES_WIDE=1" "CTR_PLAN_LOOKAHEAD=1 CTR_GEMM_PLANES_WIDE=1"; do
    env $e timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline \
      > gpurun_out/b9.json 2> gpurun_out/b9.err || { tail -5 gpurun_out/b9.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/b9.json'));print('$e', round(d['value']/1e6,3), round(d['ms_per_step'],4))" | tee -a gpurun_out/ab9.txt
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03_c2 -o run -- \
  python3 bench.py --config c2 --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/c2_trace.log 2>&1 || exit 1
tail -c 300 gpurun_out/c2_trace.log
