#!/bin/bash
# round 3, GPU run 11: host enqueue time (C2/C3, native vs python), wide-tile scope A/B (C3),
# C4 on the new chooser, C3 kernel trace on the new defaults
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab11.txt
run() {  # label, env, args
  env $2 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline $3 \
    > gpurun_out/b11.json 2> gpurun_out/b11.err || { tail -5 gpurun_out/b11.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b11.json'));print('$1', round(d['value']/1e6,3), round(d['ms_per_step'],4), 'host', round(d.get('host_ms_per_step',0),4))" | tee -a gpurun_out/ab11.txt
}
for r in 1 2; do
  run "c2 native" "CTR_X=0" "--config c2"
  run "c2 python" "CTR_NATIVE_LAUNCH=0" "--config c2"
  run "c3 wide1" "CTR_X=0" "--config c3"
  run "c3 wide2" "CTR_GEMM_PLANES_WIDE=2" "--config c3"
done
run "c4 default" "CTR_X=0" "--config c4"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03_c3b -o run -- \
  python3 bench.py --config c3 --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/c3b_trace.log 2>&1 || exit 1
echo traced
