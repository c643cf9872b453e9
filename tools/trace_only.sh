#!/bin/bash
# rocprofv3 kernel trace + stats of the bench for each config in $CFGS (no PMC).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
for CFG in ${CFGS:-c2 c3}; do
  OUT=gpurun_out/prof_${TAG}_${CFG}
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --config $CFG --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench_trace.log 2>&1 || exit $?
  tail -1 $OUT/bench_trace.log | cut -c1-300
done
find gpurun_out -name "*kernel_stats.csv" | head
