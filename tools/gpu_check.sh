#!/bin/bash
# One GPU session: parity tests, smoke, benches. Stops at the first crash/timeout
# (exit codes other than 0 = pass / 1 = test failure end the script).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-1200} python -u -m pytest ${TESTS:-tests -m gpu} -q -p no:cacheprovider --maxfail=60 --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -15
  ok $rc || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
  ok $rc || exit $rc
fi
i=0
while IFS= read -r args; do
  [ -z "$args" ] && continue
  i=$((i+1))
  timeout -k 10 600 python bench.py $args > gpurun_out/bench_$i.log 2>&1; rc=$?
  echo "bench[$args] rc=$rc"; tail -1 gpurun_out/bench_$i.log | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
done <<< "${BENCH_LIST:-"--steps 10 --warmup 3"}"
exit 0
