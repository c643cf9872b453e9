#!/bin/bash
# Round-3 check 5 (= 3 + 4): GEMM (asm transpose reads), sharded (fixed-capacity exchange),
# deferred (tiled sweep) and streaming tests; GEMM bench per library variant; C3 per variant;
# C3 background-sweep A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_gemm_planes.py tests/test_gpu_sharded.py tests/test_gpu_deferred.py tests/test_gpu_streaming.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest5.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest5.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for L in main trbuiltin spread; do
  if [ $L = main ]; then unset CTR_HIP_LIB; else export CTR_HIP_LIB=$PWD/rl_ctr_prediction_amd/variants/lib_$L.so; fi
  timeout -k 10 300 python tools/gemm_planes_bench.py > gpurun_out/gemm_$L.jsonl 2>&1 || exit $?
  echo "$L $(python -c "
import json
r=[json.loads(l) for l in open('gpurun_out/gemm_$L.jsonl') if l.startswith('{')]
print(' '.join(f\"{x['shape'][:5]}={x['us']}\" for x in r if 'us' in x and 'cfg' in x), r[-1])")"
  timeout -k 10 300 python tools/gemm_planes_bench.py --pg > gpurun_out/gemm_pg_$L.jsonl 2>&1 || exit $?
  echo "$L pg $(tail -1 gpurun_out/gemm_pg_$L.jsonl)"
done
: > gpurun_out/c3_ab.jsonl
run() {
  timeout -k 10 300 env "$@" python bench.py --steps 40 --warmup 5 --no-cpu-baseline $BARGS > gpurun_out/bench_one.log 2>&1 || return 1
  echo "$* $BARGS $(tail -1 gpurun_out/bench_one.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), round(d["ms_per_step"],4))')"
  tail -1 gpurun_out/bench_one.log >> gpurun_out/c3_ab.jsonl
}
V=$PWD/rl_ctr_prediction_amd/variants
BARGS="" run CTR_X=main || exit 1
BARGS="" run CTR_HIP_LIB=$V/lib_trbuiltin.so || exit 1
BARGS="" run CTR_HIP_LIB=$V/lib_spread.so || exit 1
BARGS="--sweep-slices 32" run CTR_SWEEP_BLOCKS=256 || exit 1
BARGS="--sweep-slices 32" run CTR_SWEEP_BLOCKS=512 || exit 1
BARGS="--sweep-slices 16" run CTR_SWEEP_BLOCKS=256 || exit 1
BARGS="" run CTR_X=main || exit 1
BARGS="--sharding rows" run CTR_X=main || exit 1
