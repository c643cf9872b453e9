#!/bin/bash
# Alternating bench A/B of two environment settings: ENV_A / ENV_B (e.g. "CTR_X=1"; extra
# bench arguments per side: ARGS_A / ARGS_B), configs
# $CFGS, $RUNS rounds; optional parity tests first ($TESTS). One bench line per run in
# gpurun_out/envab_<cfg>_<A|B>_<i>.log; prints the values.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/envab_tests.log 2>&1; rc=$?; tail -2 gpurun_out/envab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq ${RUNS:-2}); do
  for CFG in ${CFGS:-c3}; do
    for V in A B; do
      E=$([ $V = A ] && echo "$ENV_A" || echo "$ENV_B")
      X=$([ $V = A ] && echo "$ARGS_A" || echo "$ARGS_B")
      env $E timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline $BENCH_ARGS $X > gpurun_out/envab_${CFG}_${V}_$i.log 2>&1 || exit $?
      echo "$CFG $V [$E $X] $(tail -1 gpurun_out/envab_${CFG}_${V}_$i.log | grep -o '"value": [0-9.]*')"
    done
  done
done
