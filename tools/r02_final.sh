#!/bin/bash
# Round-2 evidence: rocprofv3 kernel trace + FETCH/WRITE PMC passes of the C3, C2, C5 benches
# (tools/gpu_profile.sh), then one bench line per config (smoke first). Stops at the first
# failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
echo smoke ok
for CFG in ${PROFILE_CFGS:-c3 c2 c5}; do
  CFG=$CFG TAG=r02 bash tools/gpu_profile.sh > gpurun_out/profile_$CFG.log 2>&1 || { echo "profile $CFG failed"; tail -5 gpurun_out/profile_$CFG.log; exit 1; }
  echo "profile $CFG ok"
done
: > gpurun_out/r02_bench_lines.jsonl
for args in "--config c3 --steps 20 --warmup 5" "--config c2 --steps 20 --warmup 5 --no-cpu-baseline" "--config c5 --steps 20 --warmup 5 --no-cpu-baseline" "--config ipnn --steps 20 --warmup 5 --no-cpu-baseline" "--config c4 --steps 20 --warmup 5 --no-cpu-baseline"; do
  timeout -k 10 600 python bench.py $args > gpurun_out/bench_one.log 2>&1 || { echo "bench $args failed"; tail -5 gpurun_out/bench_one.log; exit 1; }
  tail -1 gpurun_out/bench_one.log >> gpurun_out/r02_bench_lines.jsonl
  echo "bench $args ok"
done
