#!/bin/bash
# Round-3 check 3: sharded (fixed-capacity exchange) / deferred (tiled sweep) / streaming
# tests, then C3 A/B of the background sweep against the periodic flush.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_deferred.py tests/test_gpu_streaming.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest3.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest3.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > gpurun_out/sweep_ab.jsonl
run() {
  timeout -k 10 300 env "$@" python bench.py --steps 60 --warmup 5 --no-cpu-baseline $BARGS > gpurun_out/bench_one.log 2>&1 || return 1
  echo "$* $(tail -1 gpurun_out/bench_one.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), round(d["ms_per_step"],4))')"
  tail -1 gpurun_out/bench_one.log >> gpurun_out/sweep_ab.jsonl
}
BARGS="" run CTR_SWEEP_BLOCKS=256 || exit 1
for S in 16 32 64; do
  for BL in 128 256 512; do
    BARGS="--sweep-slices $S" run CTR_SWEEP_BLOCKS=$BL || exit 1
  done
done
BARGS="" run CTR_SWEEP_BLOCKS=256 || exit 1
BARGS="--sharding rows" run CTR_SWEEP_BLOCKS=256 || exit 1
