#!/bin/bash
# Round-3 check 2: GEMM / deferred / sharded tests, flush variants, C3 A/B of the flush
# variants, then a rocprofv3 kernel trace of the C3 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm_planes.py tests/test_gpu_deferred.py tests/test_gpu_sharded.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest2.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest2.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/flush_bench.py --variants 0,1,2 --steps-list 1,20,32,64 --reps 3 > gpurun_out/flush_ab.jsonl 2>&1 || exit $?
cut -c1-200 gpurun_out/flush_ab.jsonl
for v in 0 1 2 0 1 2; do
  CTR_FLUSH_PIPE=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_one.log 2>&1 || exit $?
  echo "pipe=$v $(tail -1 gpurun_out/bench_one.log | cut -c1-140)"
done
OUT=gpurun_out/prof_r03_c3
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_trace.log 2>&1 || exit $?
tail -1 $OUT/bench_trace.log | cut -c1-200
find $OUT -name "*stats*"
