#!/bin/bash
# Round-4 closing check on the final tree: the whole GPU suite, smoke, the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_STOP=--maxfail=10 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > gpurun_out/b22_default.log 2>&1 || { tail -5 gpurun_out/b22_default.log; exit 1; }
tail -1 gpurun_out/b22_default.log | cut -c1-400
