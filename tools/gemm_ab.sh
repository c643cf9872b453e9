#!/bin/bash
# Planes GEMM change check: its parity tests, the standalone sweep of the C3 shapes, then C3
# bench lines (default library vs CTR_HIP_LIB=$VARIANT when given), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_planes.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_gemm.log 2>&1; rc=$?; tail -2 gpurun_out/t_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_planes_bench.py ${SWEEP_ARGS:---sweep --only 8,29,30,31,34 --splits 1 --shapes fwd0} > gpurun_out/gemm_sweep.jsonl 2>&1 || exit $?
grep -E "best|sum_auto" gpurun_out/gemm_sweep.jsonl
for i in $(seq ${RUNS:-2}); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_base_$i.log 2>&1 || exit $?
  echo "base $(tail -1 gpurun_out/ab_base_$i.log | cut -c1-200 | grep -o '"value": [0-9.]*')"
  if [ -n "$VARIANT" ]; then
    CTR_HIP_LIB=$VARIANT timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_var_$i.log 2>&1 || exit $?
    echo "var  $(tail -1 gpurun_out/ab_var_$i.log | cut -c1-200 | grep -o '"value": [0-9.]*')"
  fi
done
