#!/bin/bash
# round 3, GPU run 12: stages issued before the step graph (native) — C2 / C3 native vs python
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_streaming.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest12.log 2>&1 || { tail -20 gpurun_out/pytest12.log; exit 1; }
tail -2 gpurun_out/pytest12.log
: > gpurun_out/ab12.txt
run() {  # label, env, args
  env $2 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline $3 \
    > gpurun_out/b12.json 2> gpurun_out/b12.err || { tail -5 gpurun_out/b12.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b12.json'));print('$1', round(d['value']/1e6,3), round(d['ms_per_step'],4), 'host', round(d.get('host_ms_per_step',0),4))" | tee -a gpurun_out/ab12.txt
}
for r in 1 2; do
  run "c2 native" "CTR_X=0" "--config c2"
  run "c2 python" "CTR_NATIVE_LAUNCH=0" "--config c2"
  run "c3 native" "CTR_X=0" "--config c3"
  run "c3 python" "CTR_NATIVE_LAUNCH=0" "--config c3"
done
