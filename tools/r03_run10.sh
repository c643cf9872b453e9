#!/bin/bash
# round 3, GPU run 10: full GPU suite; native step launch A/B (C2, C3); IPNN / C4 under the
# new defaults (plan lookahead everywhere, whole-M weight-gradient tiles)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_deferred.py tests/test_gpu_streaming.py tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest10.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest10.log | tail -8
[ $rc -eq 0 ] || exit 1
: > gpurun_out/ab10.txt
run() {  # label, env, args
  env $2 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline $3 \
    > gpurun_out/b10.json 2> gpurun_out/b10.err || { tail -5 gpurun_out/b10.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b10.json'));print('$1', round(d['value']/1e6,3), round(d['ms_per_step'],4))" | tee -a gpurun_out/ab10.txt
}
for r in 1 2; do
  run "c2 native" "CTR_X=0" "--config c2"
  run "c2 python" "CTR_NATIVE_LAUNCH=0" "--config c2"
  run "c3 native" "CTR_X=0" "--config c3"
  run "c3 python" "CTR_NATIVE_LAUNCH=0" "--config c3"
done
run "ipnn default" "CTR_X=0" "--config ipnn"
run "ipnn wide0" "CTR_GEMM_PLANES_WIDE=0" "--config ipnn"
run "ipnn la0" "CTR_PLAN_LOOKAHEAD=0" "--config ipnn"
run "c4 default" "CTR_X=0" "--config c4"
run "c4 wide0" "CTR_GEMM_PLANES_WIDE=0" "--config c4"
run "c5 default" "CTR_X=0" "--config c5"
