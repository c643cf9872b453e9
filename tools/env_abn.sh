#!/bin/bash
# Alternating bench A/B/... of N environment settings: VARIANTS="ENV1|ENV2|..." (each a
# space-separated list of VAR=value, "-" for none), configs $CFGS, $RUNS rounds, extra bench
# arguments $BENCH_ARGS. One line per run: config, variant, examples/s.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS='|' read -ra VS <<< "$VARIANTS"
for i in $(seq ${RUNS:-2}); do
  for CFG in ${CFGS:-c3}; do
    for j in "${!VS[@]}"; do
      E="${VS[$j]}"; [ "$E" = "-" ] && E=""
      env $E timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline $BENCH_ARGS > gpurun_out/abn_${CFG}_${j}_$i.log 2>&1 || exit $?
      echo "$CFG v$j [$E] $(tail -1 gpurun_out/abn_${CFG}_${j}_$i.log | grep -o '"value": [0-9.]*')"
    done
  done
done
