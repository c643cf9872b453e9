#!/bin/bash
# Round-3 check 1: streaming / deferred / FFM / PG tests + GEMM planes tests, the GEMM
# sweep of the new whole-M and XCD-partitioned tilings, then fresh-batch benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm_planes.py tests/test_gpu_streaming.py tests/test_gpu_deferred.py tests/test_gpu_ffm.py tests/test_gpu_models.py::test_pg_graph_learn_sees_load_state_dict -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest1.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest1.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/gemm_planes_bench.py --sweep --only 25,26,27,28,7 --splits 4,8,9,12,16,24,32,43 --shapes dW > gpurun_out/gemm_sweep_dw.jsonl 2>&1 || exit $?
grep best gpurun_out/gemm_sweep_dw.jsonl
timeout -k 10 300 python tools/gemm_planes_bench.py --sweep --only 19,7,13 --splits 1 --xg 1,2,4 --shapes dX,dH1,fwd > gpurun_out/gemm_sweep_dx.jsonl 2>&1 || exit $?
grep -E "best|auto" gpurun_out/gemm_sweep_dx.jsonl
while IFS= read -r args; do
  [ -z "$args" ] && continue
  timeout -k 10 600 python bench.py $args > gpurun_out/bench_one.log 2>&1; rc=$?
  echo "bench[$args] rc=$rc"; tail -1 gpurun_out/bench_one.log | cut -c1-700
  tail -1 gpurun_out/bench_one.log >> gpurun_out/bench_lines.jsonl
  [ $rc -eq 0 ] || exit $rc
done <<< "$BENCH_LIST"
