#!/bin/bash
# Round-3 check 4: GEMM tests on the asm transpose reads, GEMM bench of the library and its
# variants (builtin transpose reads = r02 code; spread LDS-DMA issue), C3 bench per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_planes.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest4.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest4.log | tail -12
[ $rc -eq 0 ] || exit $rc
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
unset CTR_HIP_LIB
for L in main trbuiltin spread main; do
  if [ $L = main ]; then unset CTR_HIP_LIB; else export CTR_HIP_LIB=$PWD/rl_ctr_prediction_amd/variants/lib_$L.so; fi
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_one.log 2>&1 || exit $?
  echo "c3 $L $(tail -1 gpurun_out/bench_one.log | cut -c1-120)"
done
