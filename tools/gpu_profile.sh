#!/bin/bash
# rocprofv3 kernel trace + stats of the bench, then separate PMC passes (FETCH_SIZE,
# WRITE_SIZE) — never combined with tracing domains. Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${CFG:-c3}
TAG=${TAG:-r01}
OUT=gpurun_out/prof_${TAG}_${CFG}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-driver-loop > $OUT/bench_trace.log 2>&1 || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run -- \
    python3 bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-driver-loop > $OUT/bench_$C.log 2>&1 || exit $?
done
find $OUT -name "*.csv" | head -20
