#!/bin/bash
# Round-2 closing bench lines: smoke, then one bench line per config (the driver's
# --steps 20 --warmup 5), appended to gpurun_out/r02_bench_lines.jsonl. Stops at the first
# failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
echo smoke ok
: > gpurun_out/r02_bench_lines.jsonl
for args in "--config c3 --steps 20 --warmup 5" "--config c2 --steps 20 --warmup 5 --no-cpu-baseline" "--config c5 --steps 20 --warmup 5 --no-cpu-baseline" "--config ipnn --steps 20 --warmup 5 --no-cpu-baseline" "--config c4 --steps 20 --warmup 5 --no-cpu-baseline"; do
  timeout -k 10 420 python bench.py $args > gpurun_out/bench_one.log 2>&1 || { echo "bench $args failed"; tail -5 gpurun_out/bench_one.log; exit 1; }
  tail -1 gpurun_out/bench_one.log >> gpurun_out/r02_bench_lines.jsonl
  echo "bench $args ok: $(tail -1 gpurun_out/bench_one.log | cut -c100-190)"
done
