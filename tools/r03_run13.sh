#!/bin/bash
# round 3, GPU run 13: C3 dW0 fork point / db0 placement A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab13.txt
run() {  # label, env, args
  env $2 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline $3 \
    > gpurun_out/b13.json 2> gpurun_out/b13.err || { tail -5 gpurun_out/b13.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b13.json'));print('$1', round(d['value']/1e6,3), round(d['ms_per_step'],4))" | tee -a gpurun_out/ab13.txt
}
for r in 1 2; do
  run "c3 default" "CTR_X=0" "--config c3"
  run "c3 dw0@dh1" "CTR_DW0_FORK=dh1" "--config c3"
  run "c3 db0last" "CTR_DB0_LAST=1" "--config c3"
  run "c3 both" "CTR_DW0_FORK=dh1 CTR_DB0_LAST=1" "--config c3"
  run "c3 dw0@dh1 wide0" "CTR_DW0_FORK=dh1 CTR_GEMM_PLANES_WIDE=0" "--config c3"
done
