#!/bin/bash
# GPU tests of the given files (default: the whole -m gpu suite), one process, each test
# bounded; log under gpurun_out/. Usage: bash tools/gpu_tests.sh [pytest args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
[ $# -eq 0 ] && set -- tests
timeout -k 10 1000 python -u -m pytest ${PYTEST_STOP:--x} -v --timeout 300 --timeout-method thread -m gpu "$@" \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests.log
exit $rc
