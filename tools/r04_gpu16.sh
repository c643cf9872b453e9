#!/bin/bash
# Round-4 validation: the whole GPU suite, smoke, the sort phase trace, bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_STOP=--maxfail=10 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
echo smoke ok
CTR_HIP_LIB=rl_ctr_prediction_amd/variants/lib_cptrace.so timeout -k 10 120 python tools/colplan_trace.py > gpurun_out/r04_colplan_trace4.txt 2>&1 || { cat gpurun_out/r04_colplan_trace4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_colplan_trace4.txt | cut -c1-100
timeout -k 10 300 python tools/plan_bench.py --configs c2,c3 > gpurun_out/r04_plan_bench_v5.txt 2>&1 || { cat gpurun_out/r04_plan_bench_v5.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_plan_bench_v5.txt | grep columns
for C in c3 c2 ipnn c3 c2 ipnn; do
  timeout -k 10 600 python bench.py --config $C --steps 20 --warmup 5 --no-driver-loop --no-cpu-baseline > gpurun_out/b16_$C.log 2>&1 || { tail -5 gpurun_out/b16_$C.log; exit 1; }
  echo "$C $(tail -1 gpurun_out/b16_$C.log | grep -o '"value": [0-9.]*' | head -1)"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof16_c3 -o run -- \
  python3 bench.py --config c3 --steps 50 --warmup 3 --no-cpu-baseline --no-driver-loop > gpurun_out/prof16_c3.log 2>&1 || { tail -5 gpurun_out/prof16_c3.log; exit 1; }
grep -E "planes_reduce|deepfm_head|colplan" gpurun_out/prof16_c3/run_kernel_stats.csv | cut -d, -f1-4
