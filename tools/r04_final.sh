#!/bin/bash
# Round-4 evidence. PART=profiles: smoke, rocprofv3 kernel trace + FETCH/WRITE PMC passes of
# the C3, C2, C5 benches (tools/gpu_profile.sh), the six C3 GEMMs' counters
# (tools/gemm_planes_pmc.sh). PART=bench: one bench line per config with its CPU baseline,
# plus a 200-step C3 region. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${PART:-profiles}" = profiles ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
  echo smoke ok
  for CFG in c3 c2 c5 ipnn; do
    CFG=$CFG TAG=r04 bash tools/gpu_profile.sh > gpurun_out/profile_$CFG.log 2>&1 || { echo "profile $CFG failed"; tail -5 gpurun_out/profile_$CFG.log; exit 1; }
    echo "profile $CFG ok"
  done
  bash tools/gemm_planes_pmc.sh > gpurun_out/gemm_pmc.log 2>&1 || { echo "gemm pmc failed"; tail -5 gpurun_out/gemm_pmc.log; exit 1; }
  echo "gemm pmc ok"
else
  : > gpurun_out/r04_bench_lines.jsonl
  for args in "--config c3 --steps 20 --warmup 5" "--config c2 --steps 20 --warmup 5" \
              "--config c5 --steps 20 --warmup 5" "--config ipnn --steps 20 --warmup 5" \
              "--config c4 --steps 20 --warmup 5"; do
    timeout -k 10 600 python bench.py $args > gpurun_out/bench_one.log 2>&1 || { echo "bench $args failed"; tail -5 gpurun_out/bench_one.log; exit 1; }
    tail -1 gpurun_out/bench_one.log >> gpurun_out/r04_bench_lines.jsonl
    echo "bench $args ok"
  done
  timeout -k 10 600 python bench.py --config c3 --steps 200 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c3_long.log 2>&1 || { echo "long c3 failed"; tail -5 gpurun_out/bench_c3_long.log; exit 1; }
  tail -1 gpurun_out/bench_c3_long.log > gpurun_out/r04_bench_c3_200steps.json
  echo "long c3 ok"
fi
